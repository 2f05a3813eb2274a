// a4: DIP local reference frames for batches of query points
// (dip/lrf.py:19-78, lrf.get; called 2 x 2048 times per pair by dip/demo.py:109-114).
//
// Contract (oracle_lrf, oracle/pcr_oracle.c): radius neighbours d2 < float(r*r)
// sorted by (d2, index); ptnn = all but the first; cov = 1/3 * scatter; the
// smallest-eigenvalue eigenvector by cyclic Jacobi; zp sign; xp from the
// alpha*beta weighted projections; yp = xp x zp (left-handed, as the
// reference); patch rows lRg^T (p - pt) / kernel picked by the caller's
// np.random.choice indices (the draw stays on the host so the reference's RNG
// stream is reproduced), zero rows past the neighbour count.  Every sum uses
// the oracle's 256-lane order (lane = i mod 256, then a halving tree), so
// results are bit-identical to the oracle.
//
// MI355X design: one 256-thread workgroup per query.  Phase 1 (pcr_lrf_count)
// counts neighbours (brute force over the cloud, f64).  Phase 2 gathers the
// neighbours into LDS (capacity KCAP, chosen from the host's max count),
// bitonic-sorts them by (d2, idx), runs the lane-partitioned sums as six
// parallel LDS trees, one lane solves the 3x3 eigenproblem, and the 256 patch
// rows are written by 256 threads.  All f64: the work is ~k*40 flops per
// query, latency- not throughput-bound; the cloud sweep (N x 24 B per query)
// is the traffic.
#include "pcr_internal.h"
#include "geom.h"

namespace pcr {
namespace {

constexpr int kT = 256;

__device__ __forceinline__ int cnt_of(const int32_t *n, int p, int nmax) {
    return n ? min(max(n[p], 0), nmax) : nmax;
}

__device__ __forceinline__ double lrf_thr(double kernel) { return (double)(float)(kernel * kernel); }

// block-wide sum in the oracle's order: s[t] holds lane t's sequential partial
__device__ __forceinline__ double tree_sum(double *s) {
    for (int w = kT / 2; w >= 1; w >>= 1) {
        __syncthreads();
        if ((int)threadIdx.x < w) s[threadIdx.x] = s[threadIdx.x] + s[threadIdx.x + w];
    }
    __syncthreads();
    const double r = s[0];
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(kT) void lrf_count_kernel(const double *pts, int Nmax,
                                                       const int32_t *n_pts, const double *qs,
                                                       int Qmax, const int32_t *n_q, double kernel,
                                                       int32_t *counts) {
    const int p = blockIdx.y, qi = blockIdx.x;
    if (qi >= cnt_of(n_q, p, Qmax)) return;
    const int n = cnt_of(n_pts, p, Nmax);
    const double *P = pts + (size_t)p * Nmax * 3;
    const double *q = qs + ((size_t)p * Qmax + qi) * 3;
    const double qx = q[0], qy = q[1], qz = q[2], thr = lrf_thr(kernel);
    int c = 0;
    for (int i = threadIdx.x; i < n; i += kT) {
        const double dx = P[3 * i] - qx, dy = P[3 * i + 1] - qy, dz = P[3 * i + 2] - qz;
        c += ((dx * dx + dy * dy) + dz * dz) < thr;
    }
    for (int o = 32; o; o >>= 1) c += __shfl_xor(c, o, 64);
    __shared__ int wc[kT / 64];
    if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) counts[(size_t)p * Qmax + qi] = (wc[0] + wc[1]) + (wc[2] + wc[3]);
}

// cyclic Jacobi on a symmetric 3x3 (same operation order as oracle sym3_smallest)
__device__ void sym3_smallest(const double C[6], double v[3]) {
    double A[3][3] = {{C[0], C[1], C[2]}, {C[1], C[3], C[4]}, {C[2], C[4], C[5]}};
    double V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int sweep = 0; sweep < 32; ++sweep) {
        const double off = (A[0][1] * A[0][1] + A[0][2] * A[0][2]) + A[1][2] * A[1][2];
        if (off == 0.0) break;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int r = p + 1; r < 3; ++r) {
                const double apr = A[p][r];
                if (apr != 0.0) {
                    const double theta = (A[r][r] - A[p][p]) / (2.0 * apr);
                    double t = 1.0 / (__builtin_fabs(theta) + __builtin_sqrt(theta * theta + 1.0));
                    if (theta < 0.0) t = -t;
                    const double c = 1.0 / __builtin_sqrt(t * t + 1.0), s = t * c;
                    A[p][p] = A[p][p] - t * apr;
                    A[r][r] = A[r][r] + t * apr;
                    A[p][r] = 0.0;
                    A[r][p] = 0.0;
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        if (k == p || k == r) continue;
                        const double akp = A[k][p], akr = A[k][r];
                        A[k][p] = c * akp - s * akr;
                        A[p][k] = A[k][p];
                        A[k][r] = s * akp + c * akr;
                        A[r][k] = A[k][r];
                    }
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        const double vkp = V[k][p], vkr = V[k][r];
                        V[k][p] = c * vkp - s * vkr;
                        V[k][r] = s * vkp + c * vkr;
                    }
                }
            }
    }
    int m = 0;
    if (A[1][1] < A[m][m]) m = 1;
    if (A[2][2] < A[m][m]) m = 2;
    const double n = __builtin_sqrt((V[0][m] * V[0][m] + V[1][m] * V[1][m]) + V[2][m] * V[2][m]);
#pragma unroll
    for (int k = 0; k < 3; ++k) v[k] = V[k][m] / n;
}

struct LrfArgs {
    const double *pts, *qs;
    const int32_t *n_pts, *n_q, *inds;
    int Nmax, Qmax, patch_size;
    double kernel;
    double *patches, *T;
    int32_t *counts;
};

template <int KCAP>
__global__ __launch_bounds__(kT) void lrf_frame_kernel(LrfArgs a) {
    __shared__ double hd[KCAP];
    __shared__ int hi[KCAP];
    __shared__ double red[6][kT];
    __shared__ double frame[12];  // xp yp zp pt
    __shared__ int s_k;
    const int p = blockIdx.y, qi = blockIdx.x, t = threadIdx.x;
    if (qi >= cnt_of(a.n_q, p, a.Qmax)) return;
    const int n = cnt_of(a.n_pts, p, a.Nmax);
    const double *P = a.pts + (size_t)p * a.Nmax * 3;
    const double *q = a.qs + ((size_t)p * a.Qmax + qi) * 3;
    const double qx = q[0], qy = q[1], qz = q[2], thr = lrf_thr(a.kernel);
    if (t == 0) s_k = 0;
    __syncthreads();
    // 1. gather (order fixed later by the sort; keys (d2, idx) are unique)
    for (int i = t; i < n; i += kT) {
        const double dx = P[3 * i] - qx, dy = P[3 * i + 1] - qy, dz = P[3 * i + 2] - qz;
        const double d2 = (dx * dx + dy * dy) + dz * dz;
        if (d2 < thr) {
            const int e = atomicAdd(&s_k, 1);
            if (e < KCAP) { hd[e] = d2; hi[e] = i; }
        }
    }
    __syncthreads();
    const int k = s_k;
    const size_t qo = (size_t)p * a.Qmax + qi;
    if (t == 0 && a.counts) a.counts[qo] = k;
    double *Tout = a.T + qo * 16;
    double *patch = a.patches + qo * (size_t)a.patch_size * 3;
    if (k > KCAP) {  // host chose the capacity from phase 1; never taken
        for (int i = t; i < 16; i += kT) Tout[i] = __builtin_nan("");
        return;
    }
    // 2. bitonic sort by (d2, idx) over the next power of two
    int np2 = 1;
    while (np2 < k) np2 <<= 1;
    for (int i = k + t; i < np2; i += kT) { hd[i] = __builtin_inf(); hi[i] = 0x7fffffff; }
    __syncthreads();
    for (int size = 2; size <= np2; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = t; i < np2; i += kT) {
                const int j = i ^ stride;
                if (j > i) {
                    const bool up = (i & size) == 0;
                    const double di = hd[i], dj = hd[j];
                    const int ii = hi[i], ij = hi[j];
                    const bool gt = (di > dj) || (di == dj && ii > ij);
                    if (gt == up) { hd[i] = dj; hd[j] = di; hi[i] = ij; hi[j] = ii; }
                }
            }
            __syncthreads();
        }
    // 3. covariance of ptnn = sorted[1:]
    const int kn = k > 0 ? k - 1 : 0;
    {
        double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0, s4 = 0.0, s5 = 0.0;
        for (int i = t; i < kn; i += kT) {
            const double *pp = P + 3 * hi[i + 1];
            const double dx = pp[0] - qx, dy = pp[1] - qy, dz = pp[2] - qz;
            s0 = s0 + dx * dx;
            s1 = s1 + dx * dy;
            s2 = s2 + dx * dz;
            s3 = s3 + dy * dy;
            s4 = s4 + dy * dz;
            s5 = s5 + dz * dz;
        }
        red[0][t] = s0; red[1][t] = s1; red[2][t] = s2;
        red[3][t] = s3; red[4][t] = s4; red[5][t] = s5;
    }
    for (int w = kT / 2; w >= 1; w >>= 1) {
        __syncthreads();
        if (t < w)
#pragma unroll
            for (int e = 0; e < 6; ++e) red[e][t] = red[e][t] + red[e][t + w];
    }
    __syncthreads();
    if (t == 0) {
        double C[6], nh[3];
#pragma unroll
        for (int e = 0; e < 6; ++e) C[e] = (1.0 / 3.0) * red[e][0];
        sym3_smallest(C, nh);
        frame[0] = nh[0]; frame[1] = nh[1]; frame[2] = nh[2];
    }
    __syncthreads();
    const double h0 = frame[0], h1 = frame[1], h2 = frame[2];
    // 4. z sign
    {
        double s = 0.0;
        for (int i = t; i < kn; i += kT) {
            const double *pp = P + 3 * hi[i + 1];
            s = s + ((h0 * (qx - pp[0]) + h1 * (qy - pp[1])) + h2 * (qz - pp[2]));
        }
        red[0][t] = s;
    }
    const double zs = tree_sum(red[0]);
    const double z0 = zs > 0.0 ? h0 : -h0, z1 = zs > 0.0 ? h1 : -h1, z2 = zs > 0.0 ? h2 : -h2;
    // 5. x axis
    {
        double sx = 0.0, sy = 0.0, sz = 0.0;
        for (int i = t; i < kn; i += kT) {
            const double *pp = P + 3 * hi[i + 1];
            const double dx = pp[0] - qx, dy = pp[1] - qy, dz = pp[2] - qz;
            const double proj = (dx * z0 + dy * z1) + dz * z2;
            const double ex = qx - pp[0], ey = qy - pp[1], ez = qz - pp[2];
            const double nr = __builtin_sqrt((ex * ex + ey * ey) + ez * ez);
            const double al = (a.kernel - nr) * (a.kernel - nr);
            const double w = al * (proj * proj);
            sx = sx + (dx - proj * z0) * w;
            sy = sy + (dy - proj * z1) * w;
            sz = sz + (dz - proj * z2) * w;
        }
        red[0][t] = sx; red[1][t] = sy; red[2][t] = sz;
    }
    for (int w = kT / 2; w >= 1; w >>= 1) {
        __syncthreads();
        if (t < w) {
            red[0][t] = red[0][t] + red[0][t + w];
            red[1][t] = red[1][t] + red[1][t + w];
            red[2][t] = red[2][t] + red[2][t + w];
        }
    }
    __syncthreads();
    if (t == 0) {
        const double xs0 = red[0][0], xs1 = red[1][0], xs2 = red[2][0];
        const double xn = 1.0 / __builtin_sqrt((xs0 * xs0 + xs1 * xs1) + xs2 * xs2);
        const double x0 = xn * xs0, x1 = xn * xs1, x2 = xn * xs2;
        const double y0 = x1 * z2 - x2 * z1, y1 = x2 * z0 - x0 * z2, y2 = x0 * z1 - x1 * z0;
        frame[0] = x0; frame[1] = x1; frame[2] = x2;
        frame[3] = y0; frame[4] = y1; frame[5] = y2;
        frame[6] = z0; frame[7] = z1; frame[8] = z2;
        const double xv[3] = {x0, x1, x2}, yv[3] = {y0, y1, y2}, zv[3] = {z0, z1, z2};
        const double qv[3] = {qx, qy, qz};
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            Tout[4 * r + 0] = xv[r];
            Tout[4 * r + 1] = yv[r];
            Tout[4 * r + 2] = zv[r];
            Tout[4 * r + 3] = qv[r];
        }
        Tout[12] = 0.0; Tout[13] = 0.0; Tout[14] = 0.0; Tout[15] = 1.0;
    }
    __syncthreads();
    // 6. patch rows
    const double x0 = frame[0], x1 = frame[1], x2 = frame[2];
    const double y0 = frame[3], y1 = frame[4], y2 = frame[5];
    const int32_t *ind = a.inds + qo * (size_t)a.patch_size;
    for (int i = t; i < a.patch_size; i += kT) {
        const int s = ind[i];
        double o0 = 0.0, o1 = 0.0, o2 = 0.0;
        if (s >= 0 && s < k) {
            const double *pp = P + 3 * hi[s];
            const double dx = pp[0] - qx, dy = pp[1] - qy, dz = pp[2] - qz;
            o0 = ((x0 * dx + x1 * dy) + x2 * dz) / a.kernel;
            o1 = ((y0 * dx + y1 * dy) + y2 * dz) / a.kernel;
            o2 = ((z0 * dx + z1 * dy) + z2 * dz) / a.kernel;
        }
        patch[3 * i + 0] = o0;
        patch[3 * i + 1] = o1;
        patch[3 * i + 2] = o2;
    }
}

}  // namespace
}  // namespace pcr

extern "C" int pcr_lrf_count(const double *pts, int32_t P, int32_t Nmax, const int32_t *n_pts,
                             const double *queries, int32_t Qmax, const int32_t *n_q,
                             double kernel, int32_t *counts, pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(P >= 0 && Nmax >= 0 && Qmax >= 0, PCR_ERR_ARG, "lrf_count: negative size");
    if (P == 0 || Qmax == 0) return PCR_OK;
    PCR_REQUIRE(P <= 65535, PCR_ERR_ARG, "lrf_count: P=%d > 65535", P);
    PCR_REQUIRE(queries && counts && (pts || Nmax == 0), PCR_ERR_ARG, "lrf_count: null pointer");
    PCR_REQUIRE(kernel > 0.0, PCR_ERR_ARG, "lrf_count: kernel must be > 0");
    hipStream_t s = pcr::as_stream(stream);
    hipLaunchKernelGGL(pcr::lrf_count_kernel, dim3(Qmax, P), dim3(pcr::kT), 0, s, pts, Nmax, n_pts,
                       queries, Qmax, n_q, kernel, counts);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

extern "C" int pcr_lrf_compute(const double *pts, int32_t P, int32_t Nmax, const int32_t *n_pts,
                               const double *queries, int32_t Qmax, const int32_t *n_q,
                               double kernel, int32_t patch_size, const int32_t *inds,
                               int32_t max_count, double *patches, double *T, int32_t *counts,
                               pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(P >= 0 && Nmax >= 0 && Qmax >= 0, PCR_ERR_ARG, "lrf: negative size");
    if (P == 0 || Qmax == 0) return PCR_OK;
    PCR_REQUIRE(P <= 65535, PCR_ERR_ARG, "lrf: P=%d > 65535", P);
    PCR_REQUIRE(queries && inds && patches && T && (pts || Nmax == 0), PCR_ERR_ARG,
                "lrf: null pointer");
    PCR_REQUIRE(kernel > 0.0 && patch_size > 0, PCR_ERR_ARG, "lrf: kernel and patch_size must be > 0");
    PCR_REQUIRE(max_count >= 0 && max_count <= 8192, PCR_ERR_ARG,
                "lrf: max_count=%d outside [0, 8192] (neighbour list capacity)", max_count);
    pcr::LrfArgs a;
    a.pts = pts; a.qs = queries; a.n_pts = n_pts; a.n_q = n_q; a.inds = inds;
    a.Nmax = Nmax; a.Qmax = Qmax; a.patch_size = patch_size; a.kernel = kernel;
    a.patches = patches; a.T = T; a.counts = counts;
    hipStream_t s = pcr::as_stream(stream);
    const dim3 g(Qmax, P), b(pcr::kT);
    if (max_count <= 512) hipLaunchKernelGGL(pcr::lrf_frame_kernel<512>, g, b, 0, s, a);
    else if (max_count <= 2048) hipLaunchKernelGGL(pcr::lrf_frame_kernel<2048>, g, b, 0, s, a);
    else hipLaunchKernelGGL(pcr::lrf_frame_kernel<8192>, g, b, 0, s, a);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}
