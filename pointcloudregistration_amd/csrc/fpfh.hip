// f1: normal estimation and FPFH features on the GPU, the
// preprocessing of DataPreparation/RANSAC.py:12-22:
//     pcd.estimate_normals(KDTreeSearchParamHybrid(radius=4*voxel, max_nn=30))
//     compute_fpfh_feature(pcd, KDTreeSearchParamHybrid(radius=7*voxel, max_nn=100))
// i.e. Open3D 0.13's PointCloud::EstimateNormals (ComputeCovariance +
// FastEigen3x3) and pipelines/registration/Feature.cpp (ComputePairFeatures,
// ComputeSPFHFeature, ComputeFPFHFeature).  Open3D is absent and not vendored:
// the semantics are those restated in oracle/fpfh_oracle.c (parity vs Open3D
// unpinned), and every kernel here reproduces that restatement bit for bit
// (f64, + - * / sqrt in the same order, -ffp-contract=off, the det_* elementary
// functions instead of libm/ocml).
//
// Kernels (one wave64 workgroup per point where a point owns a list):
//   hybrid_search  KDTreeFlann::SearchHybrid(r, max_nn) for every point of P
//                  clouds: candidates from the hashed grid (grid.h, cells 2.01 r,
//                  <= 8 distinct slots), d2 < (double)(float)(r*r) appended to an
//                  LDS list by ballot, bitonic-sorted by (d2, index) and cut to
//                  max_nn whenever the list fills; output (P,N,K) idx / d2, (P,N) count.
//   normals        one thread per point: cumulants in list order, covariance,
//                  FastEigen3x3, prior-normal orientation.
//   spfh           wave per point: lanes take the neighbours, pair features ->
//                  3 bins -> LDS counts (order-free), then bin j = incr added
//                  count times (the reference's += sequence, exactly).
//   fpfh           wave per point: lane j < 33 accumulates its bin over the list
//                  in order; lanes 33..35 the three group sums in Open3D's
//                  (neighbour, bin) order; normalise, add the own SPFH.
// All are HBM/L2-latency bound at the reference's sizes (tens of neighbours).
#include "pcr_internal.h"
#include "grid.h"

#include <climits>

namespace pcr {
namespace {

constexpr double kPi = 3.14159265358979311600;
constexpr double kPi2 = 1.57079632679489655800;
constexpr double kPi4 = 0.78539816339744827900;
constexpr double kPi6 = 0.52359877559829892668;
constexpr double kSqrt3 = 1.73205080756887719318;
constexpr double kTanPi12 = 0.26794919243112269546;

// ---- deterministic elementary functions (oracle/fpfh_oracle.c, same ops) ----
__device__ inline double det_atan_unit(double t) {
    double off = 0.0;
    if (t > kTanPi12) {
        t = (t * kSqrt3 - 1.0) / (t + kSqrt3);
        off = kPi6;
    }
    const double t2 = t * t;
    double s = 1.0 / 29.0;
    for (int k = 13; k >= 0; k--) s = ((k & 1) ? -1.0 : 1.0) / (double)(2 * k + 1) + t2 * s;
    return off + t * s;
}

__device__ inline double det_atan2(double y, double x) {
    const double ax = fabs(x), ay = fabs(y);
    double a;
    if (ax == 0.0 && ay == 0.0) {
        a = __builtin_signbit(x) ? kPi : 0.0;
    } else {
        a = ay <= ax ? det_atan_unit(ay / ax) : kPi2 - det_atan_unit(ax / ay);
        if (__builtin_signbit(x)) a = kPi - a;
    }
    return __builtin_signbit(y) ? -a : a;
}

__device__ inline double det_acos(double x) {
    return 2.0 * det_atan2(__builtin_sqrt(1.0 - x), __builtin_sqrt(1.0 + x));
}

__device__ inline double det_cos(double x) {
    double sg = 1.0;
    if (x > kPi2) {
        x = kPi - x;
        sg = -1.0;
    }
    const bool sine = x > kPi4;
    if (sine) x = kPi2 - x;
    const double x2 = x * x;
    double s = 1.0;
    if (sine) {
        for (int k = 10; k >= 1; k--) s = 1.0 - x2 / (double)((2 * k) * (2 * k + 1)) * s;
        return sg * (x * s);
    }
    for (int k = 10; k >= 1; k--) s = 1.0 - x2 / (double)((2 * k - 1) * (2 * k)) * s;
    return sg * s;
}

__device__ inline void cross3(const double a[3], const double b[3], double o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

__device__ inline double dot3(const double a[3], const double b[3]) {
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}

// ---- hybrid search ---------------------------------------------------------

constexpr int kCap = 512;     // LDS list entries per wave
constexpr int kMaxNN = kCap - kWave;

struct SearchArgs {
    const float *xyz;          // (P, N, 3)
    const int32_t *n;          // (P) or NULL
    int N, K;
    double r, thr;             // radius, (double)(float)(r*r)
    GridBatch g;
    int32_t *idx;              // (P, N, K)
    double *d2;                // (P, N, K)
    int32_t *cnt;              // (P, N)
};

__device__ __forceinline__ int count_of(const int32_t *n, int p, int N) {
    return n ? min(max(n[p], 0), N) : N;
}

// ascending bitonic sort of (key, idx) over m = pow2 entries, one wave
__device__ void wave_sort(unsigned long long *key, int *id, int m) {
    const int lane = threadIdx.x;
    for (int k = 2; k <= m; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = lane; t < (m >> 1); t += kWave) {
                const int i = 2 * t - (t & (j - 1));
                const int l = i + j;
                const unsigned long long ka = key[i], kb = key[l];
                const int ia = id[i], ib = id[l];
                const bool gt = ka > kb || (ka == kb && ia > ib);
                if (gt == ((i & k) == 0)) {
                    key[i] = kb; key[l] = ka;
                    id[i] = ib; id[l] = ia;
                }
            }
            __syncthreads();
        }
    }
}

// sort list[0..n) and keep the first min(n, K); returns the new length
__device__ int sort_cut(unsigned long long *key, int *id, int n, int K) {
    int m = 2;
    while (m < n) m <<= 1;
    for (int t = n + threadIdx.x; t < m; t += kWave) {
        key[t] = ~0ull;
        id[t] = INT_MAX;
    }
    __syncthreads();
    wave_sort(key, id, m);
    return n < K ? n : K;
}

__global__ __launch_bounds__(64) void hybrid_search_kernel(SearchArgs a) {
    __shared__ unsigned long long key[kCap];
    __shared__ int id[kCap];
    const int p = blockIdx.y, i = blockIdx.x, lane = threadIdx.x;
    const int n = count_of(a.n, p, a.N);
    if (i >= n) {
        if (i < a.N && lane == 0) a.cnt[(size_t)p * a.N + i] = 0;
        return;
    }
    const float *P = a.xyz + (size_t)p * a.N * 3;
    const double px = P[3 * i], py = P[3 * i + 1], pz = P[3 * i + 2];
    int len = 0;  // wave-uniform
    auto offer = [&](bool pass, double d, int j) {
        const unsigned long long m = __ballot(pass);
        const int c = __popcll(m);
        if (c == 0) return;
        if (len + c > kCap) len = sort_cut(key, id, len, a.K);
        if (pass) {
            const int pos = len + __popcll(m & ((1ull << lane) - 1ull));
            key[pos] = (unsigned long long)__double_as_longlong(d);
            id[pos] = j;
        }
        len += c;
    };
    const GridView g = a.g.view(p);
    const double rr = 1.001 * a.r, ic = g.inv_cell;
    const double fx0 = (px - rr) * ic, fx1 = (px + rr) * ic, fy0 = (py - rr) * ic,
                 fy1 = (py + rr) * ic, fz0 = (pz - rr) * ic, fz1 = (pz + rr) * ic;
    const double lim = 1073741824.0;  // 2^30 cells: beyond, int cell coordinates are unsafe
    const bool finite = __builtin_isfinite(px) && __builtin_isfinite(py) && __builtin_isfinite(pz);
    if (finite && fabs(fx0) < lim && fabs(fx1) < lim && fabs(fy0) < lim && fabs(fy1) < lim &&
        fabs(fz0) < lim && fabs(fz1) < lim) {
        const int x0 = (int)floor(fx0), x1 = (int)floor(fx1), y0 = (int)floor(fy0),
                  y1 = (int)floor(fy1), z0 = (int)floor(fz0), z1 = (int)floor(fz1);
        unsigned hs[8];
        int nh = 0;
        for (int x = x0; x <= x1; ++x)
            for (int y = y0; y <= y1; ++y)
                for (int z = z0; z <= z1; ++z) {
                    const unsigned h = cell_hash(x, y, z, g.S);
                    bool dup = false;
                    for (int t = 0; t < nh; ++t) dup |= hs[t] == h;
                    if (!dup && nh < 8) hs[nh++] = h;
                }
        for (int c = 0; c < nh; ++c) {
            const int s0 = (int)g.start[hs[c]], s1 = (int)g.start[hs[c] + 1];
            for (int b = s0; b < s1; b += kWave) {
                const int s = b + lane;
                double d = 0.0;
                int j = 0;
                bool pass = false;
                if (s < s1) {
                    const float4 c = g.pts[s];
                    d = dist2(px, py, pz, (double)c.x, (double)c.y, (double)c.z);
                    j = __float_as_int(c.w);
                    pass = d < a.thr;
                }
                offer(pass, d, j);
            }
        }
    } else if (finite) {
        // far outside the integer cell range: every point of the cloud
        for (int b = 0; b < n; b += kWave) {
            const int s = b + lane;
            double d = 0.0;
            bool pass = false;
            if (s < n) {
                d = dist2(px, py, pz, (double)P[3 * s], (double)P[3 * s + 1], (double)P[3 * s + 2]);
                pass = d < a.thr;
            }
            offer(pass, d, s);
        }
    }
    if (len > 0) len = sort_cut(key, id, len, a.K);
    const size_t o = ((size_t)p * a.N + i) * a.K;
    for (int t = lane; t < a.K; t += kWave) {
        a.idx[o + t] = t < len ? id[t] : -1;
        a.d2[o + t] = t < len ? __longlong_as_double((long long)key[t]) : 0.0;
    }
    if (lane == 0) a.cnt[(size_t)p * a.N + i] = len;
}

// ---- normals ---------------------------------------------------------------

__device__ void eigvec0(const double A[9], double ev, double o[3]) {
    const double r0[3] = {A[0] - ev, A[1], A[2]};
    const double r1[3] = {A[1], A[4] - ev, A[5]};
    const double r2[3] = {A[2], A[5], A[8] - ev};
    double c01[3], c02[3], c12[3];
    cross3(r0, r1, c01);
    cross3(r0, r2, c02);
    cross3(r1, r2, c12);
    const double d0 = dot3(c01, c01), d1 = dot3(c02, c02), d2 = dot3(c12, c12);
    double dmax = d0;
    int imax = 0;
    if (d1 > dmax) { dmax = d1; imax = 1; }
    if (d2 > dmax) imax = 2;
    const double *c = imax == 0 ? c01 : (imax == 1 ? c02 : c12);
    const double s = __builtin_sqrt(imax == 0 ? d0 : (imax == 1 ? d1 : d2));
    for (int k = 0; k < 3; k++) o[k] = c[k] / s;
}

__device__ void eigvec1(const double A[9], const double e0[3], double ev, double o[3]) {
    double U[3], V[3];
    if (fabs(e0[0]) > fabs(e0[1])) {
        const double il = 1.0 / __builtin_sqrt(e0[0] * e0[0] + e0[2] * e0[2]);
        U[0] = -e0[2] * il; U[1] = 0.0; U[2] = e0[0] * il;
    } else {
        const double il = 1.0 / __builtin_sqrt(e0[1] * e0[1] + e0[2] * e0[2]);
        U[0] = 0.0; U[1] = e0[2] * il; U[2] = -e0[1] * il;
    }
    cross3(e0, U, V);
    const double AU[3] = {(A[0] * U[0] + A[1] * U[1]) + A[2] * U[2],
                          (A[1] * U[0] + A[4] * U[1]) + A[5] * U[2],
                          (A[2] * U[0] + A[5] * U[1]) + A[8] * U[2]};
    const double AV[3] = {(A[0] * V[0] + A[1] * V[1]) + A[2] * V[2],
                          (A[1] * V[0] + A[4] * V[1]) + A[5] * V[2],
                          (A[2] * V[0] + A[5] * V[1]) + A[8] * V[2]};
    double m00 = ((U[0] * AU[0] + U[1] * AU[1]) + U[2] * AU[2]) - ev;
    double m01 = (U[0] * AV[0] + U[1] * AV[1]) + U[2] * AV[2];
    double m11 = ((V[0] * AV[0] + V[1] * AV[1]) + V[2] * AV[2]) - ev;
    const double a00 = fabs(m00), a01 = fabs(m01), a11 = fabs(m11);
    if (a00 >= a11) {
        const double mx = a00 > a01 ? a00 : a01;
        if (mx > 0) {
            if (a00 >= a01) { m01 /= m00; m00 = 1.0 / __builtin_sqrt(1.0 + m01 * m01); m01 *= m00; }
            else { m00 /= m01; m01 = 1.0 / __builtin_sqrt(1.0 + m00 * m00); m00 *= m01; }
            for (int k = 0; k < 3; k++) o[k] = m01 * U[k] - m00 * V[k];
        } else {
            for (int k = 0; k < 3; k++) o[k] = U[k];
        }
    } else {
        const double mx = a11 > a01 ? a11 : a01;
        if (mx > 0) {
            if (a11 >= a01) { m01 /= m11; m11 = 1.0 / __builtin_sqrt(1.0 + m01 * m01); m01 *= m11; }
            else { m11 /= m01; m01 = 1.0 / __builtin_sqrt(1.0 + m11 * m11); m11 *= m01; }
            for (int k = 0; k < 3; k++) o[k] = m11 * U[k] - m01 * V[k];
        } else {
            for (int k = 0; k < 3; k++) o[k] = U[k];
        }
    }
}

// FastEigen3x3 (Eberly): eigenvector of the smallest eigenvalue; 0 for C = 0
__device__ void fast_eigen3x3(const double C[9], double n[3]) {
    double mc = C[0];
    for (int k = 1; k < 9; k++) mc = C[k] > mc ? C[k] : mc;
    if (mc == 0.0) { n[0] = n[1] = n[2] = 0.0; return; }
    double A[9];
    for (int k = 0; k < 9; k++) A[k] = C[k] / mc;
    const double norm = (A[1] * A[1] + A[2] * A[2]) + A[5] * A[5];
    if (norm > 0) {
        const double q = ((A[0] + A[4]) + A[8]) / 3.0;
        const double b00 = A[0] - q, b11 = A[4] - q, b22 = A[8] - q;
        const double p = __builtin_sqrt((((b00 * b00 + b11 * b11) + b22 * b22) + norm * 2.0) / 6.0);
        const double c00 = b11 * b22 - A[5] * A[5];
        const double c01 = A[1] * b22 - A[5] * A[2];
        const double c02 = A[1] * A[5] - b11 * A[2];
        const double det = ((b00 * c00 - A[1] * c01) + A[2] * c02) / ((p * p) * p);
        double hd = det * 0.5;
        hd = hd > -1.0 ? hd : -1.0;
        hd = hd < 1.0 ? hd : 1.0;
        const double angle = det_acos(hd) / 3.0;
        const double beta2 = det_cos(angle) * 2.0;
        const double beta0 = det_cos(angle + 2.09439510239319549) * 2.0;
        const double beta1 = -(beta0 + beta2);
        const double e0 = q + p * beta0, e1 = q + p * beta1, e2 = q + p * beta2;
        double v0[3], v1[3], v2[3];
        if (hd >= 0) {
            eigvec0(A, e2, v2);
            if (e2 < e0 && e2 < e1) { n[0] = v2[0]; n[1] = v2[1]; n[2] = v2[2]; return; }
            eigvec1(A, v2, e1, v1);
            if (e1 < e0 && e1 < e2) { n[0] = v1[0]; n[1] = v1[1]; n[2] = v1[2]; return; }
            cross3(v1, v2, n);
        } else {
            eigvec0(A, e0, v0);
            if (e0 < e1 && e0 < e2) { n[0] = v0[0]; n[1] = v0[1]; n[2] = v0[2]; return; }
            eigvec1(A, v0, e1, v1);
            if (e1 < e0 && e1 < e2) { n[0] = v1[0]; n[1] = v1[1]; n[2] = v1[2]; return; }
            cross3(v0, v1, n);
        }
    } else {
        double B[9];
        for (int k = 0; k < 9; k++) B[k] = A[k] * mc;
        n[0] = n[1] = n[2] = 0.0;
        if (B[0] < B[4] && B[0] < B[8]) n[0] = 1.0;
        else if (B[4] < B[0] && B[4] < B[8]) n[1] = 1.0;
        else n[2] = 1.0;
    }
}

struct NormalArgs {
    const float *xyz;
    const int32_t *n;
    int N, K;
    const int32_t *idx, *cnt;
    const double *prior;   // (P,N,3) or NULL
    double *normals;       // (P,N,3)
};

__global__ __launch_bounds__(256) void normals_kernel(NormalArgs a) {
    const int p = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count_of(a.n, p, a.N)) return;
    const float *P = a.xyz + (size_t)p * a.N * 3;
    const size_t pi = (size_t)p * a.N + i;
    const int k = a.cnt[pi];
    double C[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, v[3];
    if (k >= 3) {
        const int32_t *nb = a.idx + pi * a.K;
        double c[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int t = 0; t < k; t++) {
            const int j = nb[t];
            const double x = P[3 * j], y = P[3 * j + 1], z = P[3 * j + 2];
            c[0] += x; c[1] += y; c[2] += z;
            c[3] += x * x; c[4] += x * y; c[5] += x * z;
            c[6] += y * y; c[7] += y * z; c[8] += z * z;
        }
        for (int t = 0; t < 9; t++) c[t] /= (double)k;
        C[0] = c[3] - c[0] * c[0];
        C[4] = c[6] - c[1] * c[1];
        C[8] = c[8] - c[2] * c[2];
        C[1] = C[3] = c[4] - c[0] * c[1];
        C[2] = C[6] = c[5] - c[0] * c[2];
        C[5] = C[7] = c[7] - c[1] * c[2];
    }
    fast_eigen3x3(C, v);
    const double *pr = a.prior ? a.prior + 3 * pi : nullptr;
    if (__builtin_sqrt(dot3(v, v)) == 0.0) {
        if (pr) { v[0] = pr[0]; v[1] = pr[1]; v[2] = pr[2]; }
        else { v[0] = 0.0; v[1] = 0.0; v[2] = 1.0; }
    }
    if (pr && dot3(v, pr) < 0.0)
        for (int t = 0; t < 3; t++) v[t] *= -1.0;
    double *o = a.normals + 3 * pi;
    o[0] = v[0]; o[1] = v[1]; o[2] = v[2];
}

// ---- SPFH / FPFH -----------------------------------------------------------

struct FeatArgs {
    const float *xyz;
    const double *normals;
    const int32_t *n;
    int N, K;
    const int32_t *idx, *cnt;
    const double *d2;
    double *spfh;          // (P,N,33)
    double *fpfh;          // (P,N,33)
    float *fpfh32;         // (P,N,33) or NULL
};

__device__ __forceinline__ int clamp_bin(int h) { return h < 0 ? 0 : (h >= 11 ? 10 : h); }

// ComputePairFeatures + the three bin indices of ComputeSPFHFeature
__device__ void pair_bins(const double p1[3], const double n1[3], const double p2[3],
                          const double n2[3], int h[3]) {
    double f0 = 0.0, f1 = 0.0, f2 = 0.0;
    double dp[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    const double f3 = __builtin_sqrt(dot3(dp, dp));
    if (f3 != 0.0) {
        const double *na = n1, *nb = n2;
        const double ang1 = dot3(n1, dp) / f3;
        const double ang2 = dot3(n2, dp) / f3;
        double g2;
        if (det_acos(fabs(ang1)) > det_acos(fabs(ang2))) {
            na = n2; nb = n1;
            for (int k = 0; k < 3; k++) dp[k] *= -1.0;
            g2 = -ang2;
        } else {
            g2 = ang1;
        }
        double v[3], w[3];
        cross3(dp, na, v);
        const double vn = __builtin_sqrt(dot3(v, v));
        if (vn != 0.0) {
            for (int k = 0; k < 3; k++) v[k] /= vn;
            cross3(na, v, w);
            f2 = g2;
            f1 = dot3(v, nb);
            f0 = det_atan2(dot3(w, nb), dot3(na, nb));
        }
    }
    h[0] = clamp_bin((int)floor(11.0 * (f0 + kPi) / (2.0 * kPi)));
    h[1] = clamp_bin((int)floor(11.0 * (f1 + 1.0) * 0.5));
    h[2] = clamp_bin((int)floor(11.0 * (f2 + 1.0) * 0.5));
}

__global__ __launch_bounds__(64) void spfh_kernel(FeatArgs a) {
    __shared__ int hist[33];
    const int p = blockIdx.y, i = blockIdx.x, lane = threadIdx.x;
    if (i >= count_of(a.n, p, a.N)) return;
    const size_t pi = (size_t)p * a.N + i;
    const int k = a.cnt[pi];
    double *S = a.spfh + pi * 33;
    if (k <= 1) {
        if (lane < 33) S[lane] = 0.0;
        return;
    }
    if (lane < 33) hist[lane] = 0;
    __syncthreads();
    const float *P = a.xyz + (size_t)p * a.N * 3;
    const double *Nm = a.normals + (size_t)p * a.N * 3;
    const double p1[3] = {P[3 * i], P[3 * i + 1], P[3 * i + 2]};
    const double n1[3] = {Nm[3 * i], Nm[3 * i + 1], Nm[3 * i + 2]};
    const int32_t *nb = a.idx + pi * a.K;
    for (int t = 1 + lane; t < k; t += kWave) {
        const int j = nb[t];
        const double p2[3] = {P[3 * j], P[3 * j + 1], P[3 * j + 2]};
        const double n2[3] = {Nm[3 * j], Nm[3 * j + 1], Nm[3 * j + 2]};
        int h[3];
        pair_bins(p1, n1, p2, n2, h);
        atomicAdd(&hist[h[0]], 1);
        atomicAdd(&hist[11 + h[1]], 1);
        atomicAdd(&hist[22 + h[2]], 1);
    }
    __syncthreads();
    if (lane < 33) {
        const double incr = 100.0 / (double)(k - 1);
        double v = 0.0;
        for (int c = hist[lane]; c > 0; --c) v += incr;
        S[lane] = v;
    }
}

__global__ __launch_bounds__(64) void fpfh_kernel(FeatArgs a) {
    const int p = blockIdx.y, i = blockIdx.x, lane = threadIdx.x;
    if (i >= count_of(a.n, p, a.N)) return;
    const size_t pi = (size_t)p * a.N + i;
    const int k = a.cnt[pi];
    double acc = 0.0;
    if (k > 1) {
        const int32_t *nb = a.idx + pi * a.K;
        const double *dd = a.d2 + pi * a.K;
        const double *SP = a.spfh + (size_t)p * a.N * 33;
        if (lane < 33) {
            for (int t = 1; t < k; t++) {
                const double dist = dd[t];
                if (dist == 0.0) continue;
                acc += SP[(size_t)nb[t] * 33 + lane] / dist;
            }
        } else if (lane < 36) {
            const int g = lane - 33;
            for (int t = 1; t < k; t++) {
                const double dist = dd[t];
                if (dist == 0.0) continue;
                const double *S = SP + (size_t)nb[t] * 33 + 11 * g;
                for (int u = 0; u < 11; u++) acc += S[u] / dist;
            }
            if (acc != 0.0) acc = 100.0 / acc;
        }
    }
    const double scale = __shfl(acc, 33 + (lane < 33 ? lane / 11 : 0), kWave);
    if (lane < 33) {
        double f = 0.0;
        if (k > 1) f = acc * scale + a.spfh[pi * 33 + lane];
        a.fpfh[pi * 33 + lane] = f;
        if (a.fpfh32) a.fpfh32[pi * 33 + lane] = (float)f;
    }
}

// ---- host ------------------------------------------------------------------

int run_search(const float *xyz, int P, int N, const int32_t *n, double r, int K, hipStream_t s,
               int ws_grid, int ws_lists, SearchArgs &a) {
    PCR_REQUIRE(r > 0.0 && r < 1e300, PCR_ERR_ARG, "hybrid search: radius must be finite and > 0");
    PCR_REQUIRE(K >= 1 && K <= kMaxNN, PCR_ERR_ARG, "hybrid search: max_nn must be in [1, %d]", kMaxNN);
    PCR_REQUIRE(P <= 65535, PCR_ERR_ARG, "hybrid search: P=%d > 65535", P);
    a.xyz = xyz;
    a.n = n;
    a.N = N;
    a.K = K;
    a.r = r;
    a.thr = radius_thr(r);
    int rc = build_grids(xyz, n, P, N, r, s, ws_grid, a.g);
    if (rc != PCR_OK) return rc;
    if (ws_lists >= 0) {
        const size_t pn = (size_t)P * N;
        char *ws = (char *)workspace(ws_lists, pn * K * 12 + pn * 4 + 256);
        PCR_REQUIRE(ws, PCR_ERR_NOMEM, "hybrid search: %s", pcr_last_error());
        a.d2 = (double *)ws;
        a.idx = (int32_t *)(ws + pn * K * 8);
        a.cnt = (int32_t *)(ws + pn * K * 12);
    }
    hipLaunchKernelGGL(hybrid_search_kernel, dim3(N, P), dim3(kWave), 0, s, a);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

}  // namespace
}  // namespace pcr

extern "C" int pcr_hybrid_search(const float *xyz, int32_t P, int32_t Nmax, const int32_t *n_pts,
                                 double radius, int32_t max_nn, int32_t *idx, double *d2,
                                 int32_t *counts, pcr_stream_t stream) {
    using namespace pcr;
    clear_error();
    PCR_REQUIRE(P >= 0 && Nmax >= 0, PCR_ERR_ARG, "hybrid_search: negative size");
    if (P == 0 || Nmax == 0) return PCR_OK;
    PCR_REQUIRE(xyz && idx && d2 && counts, PCR_ERR_ARG, "hybrid_search: null pointer");
    SearchArgs a{};
    a.idx = idx;
    a.d2 = d2;
    a.cnt = counts;
    return run_search(xyz, P, Nmax, n_pts, radius, max_nn, as_stream(stream), 24, -1, a);
}

extern "C" int pcr_estimate_normals(const float *xyz, int32_t P, int32_t Nmax, const int32_t *n_pts,
                                    double radius, int32_t max_nn, const double *prior_normals,
                                    double *normals, pcr_stream_t stream) {
    using namespace pcr;
    clear_error();
    PCR_REQUIRE(P >= 0 && Nmax >= 0, PCR_ERR_ARG, "estimate_normals: negative size");
    if (P == 0 || Nmax == 0) return PCR_OK;
    PCR_REQUIRE(xyz && normals, PCR_ERR_ARG, "estimate_normals: null pointer");
    hipStream_t s = as_stream(stream);
    SearchArgs a{};
    int rc = run_search(xyz, P, Nmax, n_pts, radius, max_nn, s, 24, 25, a);
    if (rc != PCR_OK) return rc;
    NormalArgs b{xyz, n_pts, Nmax, max_nn, a.idx, a.cnt, prior_normals, normals};
    hipLaunchKernelGGL(normals_kernel, dim3((Nmax + 255) / 256, P), dim3(256), 0, s, b);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

extern "C" int pcr_compute_fpfh(const float *xyz, const double *normals, int32_t P, int32_t Nmax,
                                const int32_t *n_pts, double radius, int32_t max_nn, double *fpfh,
                                float *fpfh_f32, double *spfh, pcr_stream_t stream) {
    using namespace pcr;
    clear_error();
    PCR_REQUIRE(P >= 0 && Nmax >= 0, PCR_ERR_ARG, "compute_fpfh: negative size");
    if (P == 0 || Nmax == 0) return PCR_OK;
    PCR_REQUIRE(xyz && normals && fpfh, PCR_ERR_ARG, "compute_fpfh: null pointer");
    hipStream_t s = as_stream(stream);
    SearchArgs a{};
    int rc = run_search(xyz, P, Nmax, n_pts, radius, max_nn, s, 24, 25, a);
    if (rc != PCR_OK) return rc;
    if (!spfh) {
        spfh = (double *)workspace(26, sizeof(double) * 33 * (size_t)P * Nmax);
        PCR_REQUIRE(spfh, PCR_ERR_NOMEM, "compute_fpfh: %s", pcr_last_error());
    }
    FeatArgs f{xyz, normals, n_pts, Nmax, max_nn, a.idx, a.cnt, a.d2, spfh, fpfh, fpfh_f32};
    hipLaunchKernelGGL(spfh_kernel, dim3(Nmax, P), dim3(kWave), 0, s, f);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(fpfh_kernel, dim3(Nmax, P), dim3(kWave), 0, s, f);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}
