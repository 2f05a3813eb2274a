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

// one DPP row rotation of a 128-bit value (ctrl 0x120 + n: row_ror:n)
template <int kCtrl>
__device__ __forceinline__ xs_t xs_dpp(xs_t v) {
    const unsigned __int128 u = (unsigned __int128)v;
    unsigned l[4] = {(unsigned)u, (unsigned)(u >> 32), (unsigned)(u >> 64), (unsigned)(u >> 96)};
#pragma unroll
    for (int k = 0; k < 4; ++k) l[k] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)l[k], kCtrl, 0xf, 0xf, false);
    return (xs_t)(((unsigned __int128)l[3] << 96) | ((unsigned __int128)l[2] << 64) |
                  ((unsigned __int128)l[1] << 32) | (unsigned __int128)l[0]);
}

__device__ __forceinline__ xs_t xs_readlane(xs_t v, int lane) {
    const unsigned __int128 u = (unsigned __int128)v;
    const unsigned l0 = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, lane);
    const unsigned l1 = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), lane);
    const unsigned l2 = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 64), lane);
    const unsigned l3 = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 96), lane);
    return (xs_t)(((unsigned __int128)l3 << 96) | ((unsigned __int128)l2 << 64) |
                  ((unsigned __int128)l1 << 32) | (unsigned __int128)l0);
}

// the wave's total of one 128-bit value per lane (uniform result).  Integer
// sums are exact, so the tree shape is free: rotate-add within each row of 16
// lanes by 1, 2, 4, 8 (DPP, no LDS round trips), then the four row sums.
__device__ __forceinline__ xs_t xs_wave_sum(xs_t x) {
    x += xs_dpp<0x121>(x);
    x += xs_dpp<0x122>(x);
    x += xs_dpp<0x124>(x);
    x += xs_dpp<0x128>(x);
    return (xs_readlane(x, 0) + xs_readlane(x, 16)) + (xs_readlane(x, 32) + xs_readlane(x, 48));
}

__device__ __forceinline__ xs_t xs_shfl_xor(xs_t v, int o) {
    const unsigned long long lo = (unsigned long long)v, hi = (unsigned long long)(v >> 64);
    const unsigned long long l2 = __shfl_xor(lo, o, 64), h2 = __shfl_xor(hi, o, 64);
    return (xs_t)((((unsigned __int128)h2) << 64) | l2);
}

}  // namespace pcr
