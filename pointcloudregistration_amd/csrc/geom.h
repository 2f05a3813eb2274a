// Device-side exact-arithmetic helpers of the registration path.
// Numerical contract: f64, + - * / sqrt only, each operation rounded
// in the written order (the library is built with -ffp-contract=off), so every
// quantity below is bit-reproducible and identical to the CPU oracle's.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pcr {

// ---- Philox4x32-10, counter (itr, pair, 'RANS', block), key = seed --------
__host__ __device__ inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[1] = (uint32_t)p1;
        c[3] = (uint32_t)p0;
        c[0] = n0;
        c[2] = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// sample index j (0..n-1) of hypothesis `itr` of `pair`: uniform in [0, K)
__device__ inline int sample_index(uint64_t seed, uint32_t pair, uint32_t itr, int j, int K) {
    uint32_t c[4] = {itr, pair, 0x52414E53u, (uint32_t)(j >> 2)};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    return (int)(((uint64_t)c[j & 3] * (uint64_t)K) >> 32);
}

// ---- natural log from + - * / only (libm/ocml log are not bit-identical) ---
__device__ inline double det_log(double x) {
    if (!(x > 0.0)) return (x == 0.0) ? -__builtin_inf() : __builtin_nan("");
    if (x == __builtin_inf()) return x;
    uint64_t bits = (uint64_t)__double_as_longlong(x);
    int e = (int)((bits >> 52) & 0x7ff);
    if (e == 0) {
        x = x * 18014398509481984.0;  // 2^54
        bits = (uint64_t)__double_as_longlong(x);
        e = (int)((bits >> 52) & 0x7ff) - 54;
    }
    e -= 1023;
    bits = (bits & 0x000fffffffffffffull) | 0x3ff0000000000000ull;
    double m = __longlong_as_double((long long)bits);
    if (m > 1.4142135623730951) { m = m * 0.5; e += 1; }
    const double z = (m - 1.0) / (m + 1.0);
    const double z2 = z * z;
    double term = z, sum = 0.0;
    for (int k = 1; k <= 41; k += 2) { sum = sum + term / (double)k; term = term * z2; }
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    return ((double)e * ln2_hi + 2.0 * sum) + (double)e * ln2_lo;
}

// RANSAC iteration bound log(1-conf)/log(1-w^n); +inf = "no update"
__device__ inline double est_k_bound(double w, int n, double conf) {
    double pw = 1.0;
    for (int j = 0; j < n; ++j) pw = pw * w;
    if (!(pw > 0.0)) return __builtin_inf();
    if (pw >= 1.0) return 0.0;
    return det_log(1.0 - conf) / det_log(1.0 - pw);
}

// ---- rigid transforms ([R|t] row-major 3x4) ---------------------------------
__device__ __forceinline__ void xform12(const double *T, double px, double py, double pz,
                                        double &ox, double &oy, double &oz) {
    ox = ((T[0] * px + T[1] * py) + T[2] * pz) + T[3];
    oy = ((T[4] * px + T[5] * py) + T[6] * pz) + T[7];
    oz = ((T[8] * px + T[9] * py) + T[10] * pz) + T[11];
}

__device__ __forceinline__ double dist2(double ax, double ay, double az, double bx, double by,
                                        double bz) {
    const double dx = bx - ax, dy = by - ay, dz = bz - az;
    return (dx * dx + dy * dy) + dz * dz;
}

// largest eigenvector of symmetric 4x4 N (cyclic Jacobi), then quaternion -> R
__device__ inline void horn_rotation(const double S[9], double R[9]) {
    double A[4][4], V[4][4];
    const double Sxx = S[0], Sxy = S[1], Sxz = S[2], Syx = S[3], Syy = S[4], Syz = S[5],
                 Szx = S[6], Szy = S[7], Szz = S[8];
    A[0][0] = (Sxx + Syy) + Szz;
    A[0][1] = Syz - Szy;
    A[0][2] = Szx - Sxz;
    A[0][3] = Sxy - Syx;
    A[1][1] = (Sxx - Syy) - Szz;
    A[1][2] = Sxy + Syx;
    A[1][3] = Szx + Sxz;
    A[2][2] = (Syy - Sxx) - Szz;
    A[2][3] = Syz + Szy;
    A[3][3] = (Szz - Sxx) - Syy;
    A[1][0] = A[0][1]; A[2][0] = A[0][2]; A[3][0] = A[0][3];
    A[2][1] = A[1][2]; A[3][1] = A[1][3]; A[3][2] = A[2][3];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) V[a][b] = (a == b) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 16; ++sweep) {
        double off = 0.0;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int r = p + 1; r < 4; ++r) off = off + A[p][r] * A[p][r];
        // converged: off-diagonal mass below 2^-120 of the diagonal's (another
        // sweep moves the eigenvector by ~1e-18 relative; ~4 sweeps instead of
        // the ~6 an exact-zero test takes)
        double dsq = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) dsq = dsq + A[k][k] * A[k][k];
        if (off == 0.0 || off <= 0x1p-120 * dsq) break;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
            for (int r = p + 1; r < 4; ++r) {
                const double apr = A[p][r];
                if (apr != 0.0) {
                    const double theta = (A[r][r] - A[p][p]) / (2.0 * apr);
                    double t = 1.0 / (__builtin_fabs(theta) + __builtin_sqrt(theta * theta + 1.0));
                    if (theta < 0.0) t = -t;
                    const double c = 1.0 / __builtin_sqrt(t * t + 1.0);
                    const double s = t * c;
                    A[p][p] = A[p][p] - t * apr;
                    A[r][r] = A[r][r] + t * apr;
                    A[p][r] = 0.0;
                    A[r][p] = 0.0;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (k == p || k == r) continue;
                        const double akp = A[k][p], akr = A[k][r];
                        A[k][p] = c * akp - s * akr;
                        A[p][k] = A[k][p];
                        A[k][r] = s * akp + c * akr;
                        A[r][k] = A[k][r];
                    }
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const double vkp = V[k][p], vkr = V[k][r];
                        V[k][p] = c * vkp - s * vkr;
                        V[k][r] = s * vkp + c * vkr;
                    }
                }
            }
        }
    }
    // argmax of the diagonal, first index on ties (static register selects)
    double bd = A[0][0];
    double q[4] = {V[0][0], V[1][0], V[2][0], V[3][0]};
#pragma unroll
    for (int k = 1; k < 4; ++k) {
        const bool t = A[k][k] > bd;
        bd = t ? A[k][k] : bd;
#pragma unroll
        for (int e = 0; e < 4; ++e) q[e] = t ? V[e][k] : q[e];
    }
    double nrm = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) nrm = nrm + q[k] * q[k];
    nrm = __builtin_sqrt(nrm);
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = q[k] / nrm;
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    R[0] = ((w * w + x * x) - y * y) - z * z;
    R[1] = 2.0 * (x * y - w * z);
    R[2] = 2.0 * (x * z + w * y);
    R[3] = 2.0 * (x * y + w * z);
    R[4] = ((w * w - x * x) + y * y) - z * z;
    R[5] = 2.0 * (y * z - w * x);
    R[6] = 2.0 * (x * z - w * y);
    R[7] = 2.0 * (y * z + w * x);
    R[8] = ((w * w - x * x) - y * y) + z * z;
}

// T = [R | mt - R ms]
__device__ inline void compose_rt(const double R[9], const double ms[3], const double mt[3],
                                  double *T) {
    for (int a = 0; a < 3; ++a) {
        T[4 * a + 0] = R[3 * a + 0];
        T[4 * a + 1] = R[3 * a + 1];
        T[4 * a + 2] = R[3 * a + 2];
        T[4 * a + 3] =
            mt[a] - ((R[3 * a + 0] * ms[0] + R[3 * a + 1] * ms[1]) + R[3 * a + 2] * ms[2]);
    }
}

// deterministic block reduction of per-lane partials (256 lanes, halving tree)
constexpr int kRedLanes = 256;

// fixed-point inlier error accumulation: q = (uint64)(d2 * 2^40 / thr)
__host__ __device__ inline double fx_scale(double thr) { return 1099511627776.0 / thr; }

// radius threshold as FLANN receives it: float(r*r)
__host__ __device__ inline double radius_thr(double r) { return (double)(float)(r * r); }

}  // namespace pcr
