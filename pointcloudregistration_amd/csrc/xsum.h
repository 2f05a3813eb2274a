// Exact, order-independent sums of f64 terms (the ICP Umeyama step, a8).
//
// A term goes to a signed 128-bit fixed-point integer with LSB 2^-80 (truncated
// toward zero below it; |term| saturates at 2^47); integers add associatively,
// so any split of a pair's points over lanes, waves or workgroups yields the
// same total; the total is rounded once to the nearest f64 (ties to even).
// oracle/pcr_oracle.c (xs_term / xs_to_double) restates the same arithmetic.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pcr {

typedef __int128 xs_t;
constexpr int kXsFrac = 80;

__device__ __forceinline__ xs_t xs_term(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const int e = (int)((b >> 52) & 0x7ff);
    if (e == 0x7ff) return 0;  // non-finite: contributes 0
    const uint64_t f = b & 0x000fffffffffffffull;
    const uint64_t mant = e ? (f | 0x0010000000000000ull) : f;
    const int s = (e ? e : 1) - 1075 + kXsFrac;  // value = mant * 2^(s - 80)
    unsigned __int128 M = mant;
    if (s >= 0) {
        if (s > 74) M = (((unsigned __int128)1) << 127) - 1u;  // saturate
        else M <<= s;
    } else {
        M = (-s >= 64) ? (unsigned __int128)0 : (M >> (-s));
    }
    const xs_t v = (xs_t)M;
    return (b >> 63) ? -v : v;
}

__device__ inline double xs_to_double(xs_t v) {
    const bool neg = v < 0;
    const unsigned __int128 u = neg ? (unsigned __int128)(-(v + 1)) + 1u : (unsigned __int128)v;
    if (u == 0) return 0.0;
    const uint64_t hi = (uint64_t)(u >> 64), lo = (uint64_t)u;
    const int msb = hi ? 127 - __builtin_clzll(hi) : 63 - __builtin_clzll(lo);
    uint64_t m;
    int sh = 0;
    if (msb <= 52) {
        m = lo;
    } else {
        sh = msb - 52;
        m = (uint64_t)(u >> sh);
        const unsigned __int128 rem = u & ((((unsigned __int128)1) << sh) - 1u);
        const unsigned __int128 half = ((unsigned __int128)1) << (sh - 1);
        if (rem > half || (rem == half && (m & 1u))) {
            m += 1u;
            if (m == (1ull << 53)) { m >>= 1; sh += 1; }
        }
    }
    const int k = sh - kXsFrac;  // m * 2^k: both factors exact
    const double p2 = __longlong_as_double((long long)((uint64_t)(k + 1023) << 52));
    const double r = (double)m * p2;
    return neg ? -r : r;
}

__device__ __forceinline__ xs_t xs_shfl_xor(xs_t v, int o) {
    const unsigned long long lo = (unsigned long long)v, hi = (unsigned long long)(v >> 64);
    const unsigned long long l2 = __shfl_xor(lo, o, 64), h2 = __shfl_xor(hi, o, 64);
    return (xs_t)((((unsigned __int128)h2) << 64) | l2);
}

}  // namespace pcr
