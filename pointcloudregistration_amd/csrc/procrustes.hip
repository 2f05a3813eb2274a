// a9: batched weighted 3x3 Procrustes / Kabsch, the kernel behind the drop-ins
// for ROPNet weighted_icp (ROPNet/src/models/model_utils.py:105-139) and NDP
// rigid_fit (c2p-net/deformationpyramid/model/geometry.py:8-34).
// Contract: oracle_procrustes (pcr_oracle.c):
//   W = sum(w') + eps, w' = |w| (rigid_fit) or w (weighted_icp)
//   mu_s = sum src*(w/W), mu_t = sum tgt*(w/W)
//   S_ab = sum ((src_a - mu_s_a)*(w/W)) * (tgt_b - mu_t_b)
//   R = Horn(S) (= SVD + det fix optimum), t = mu_t - R mu_s
// All sums use the deterministic 256-lane order; one 256-thread block per item.
#include "pcr_internal.h"
#include "geom.h"

namespace pcr {
namespace {

__device__ inline void tree256x(double (*red)[9], int nv) {
    for (int s = 128; s >= 1; s >>= 1) {
        if ((int)threadIdx.x < s)
            for (int v = 0; v < nv; ++v) red[threadIdx.x][v] = red[threadIdx.x][v] + red[threadIdx.x + s][v];
        __syncthreads();
    }
}

// Scalar = float (the f32 tensors of the drop-ins) or double (f64 callers:
// the same sums, no narrowing of the inputs)
template <typename Scalar>
__global__ __launch_bounds__(256) void procrustes_kernel(const Scalar *src, const Scalar *tgt,
                                                         const Scalar *w, int N, int absw, double eps,
                                                         double *T) {
    const int b = blockIdx.x, t = threadIdx.x;
    const Scalar *S = src + (size_t)b * N * 3;
    const Scalar *G = tgt + (size_t)b * N * 3;
    const Scalar *Wt = w + (size_t)b * N;
    __shared__ double red[256][9];
    double v = 0.0;
    for (int i = t; i < N; i += 256) {
        const double wi = (double)Wt[i];
        v = v + (absw ? __builtin_fabs(wi) : wi);
    }
    red[t][0] = v;
    __syncthreads();
    tree256x(red, 1);
    const double W = red[0][0] + eps;
    __syncthreads();
    double m[6] = {0, 0, 0, 0, 0, 0};
    for (int i = t; i < N; i += 256) {
        const double wn = (double)Wt[i] / W;
        for (int c = 0; c < 3; ++c) {
            m[c] = m[c] + (double)S[3 * i + c] * wn;
            m[3 + c] = m[3 + c] + (double)G[3 * i + c] * wn;
        }
    }
    for (int k = 0; k < 6; ++k) red[t][k] = m[k];
    __syncthreads();
    tree256x(red, 6);
    const double ms[3] = {red[0][0], red[0][1], red[0][2]};
    const double mt[3] = {red[0][3], red[0][4], red[0][5]};
    __syncthreads();
    double q[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = t; i < N; i += 256) {
        const double wn = (double)Wt[i] / W;
        for (int x = 0; x < 3; ++x) {
            const double sx = ((double)S[3 * i + x] - ms[x]) * wn;
            for (int y = 0; y < 3; ++y) q[3 * x + y] = q[3 * x + y] + sx * ((double)G[3 * i + y] - mt[y]);
        }
    }
    for (int k = 0; k < 9; ++k) red[t][k] = q[k];
    __syncthreads();
    tree256x(red, 9);
    if (t == 0) {
        double Sm[9], R[9];
        for (int k = 0; k < 9; ++k) Sm[k] = red[0][k];
        horn_rotation(Sm, R);
        compose_rt(R, ms, mt, T + (size_t)b * 12);
    }
}

}  // namespace
}  // namespace pcr

namespace pcr {
template <typename Scalar>
static int procrustes_launch(const Scalar *src, const Scalar *tgt, const Scalar *weights, int32_t B,
                             int32_t N, int32_t abs_weights, double eps, double *T,
                             pcr_stream_t stream) {
    clear_error();
    PCR_REQUIRE(B >= 0 && N >= 0, PCR_ERR_ARG, "procrustes: negative size");
    if (B == 0) return PCR_OK;
    PCR_REQUIRE(src && tgt && weights && T, PCR_ERR_ARG, "procrustes: null pointer");
    hipLaunchKernelGGL(procrustes_kernel<Scalar>, dim3(B), dim3(256), 0, as_stream(stream), src,
                       tgt, weights, N, abs_weights, eps, T);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}
}  // namespace pcr

extern "C" int pcr_procrustes_batch(const float *src, const float *tgt, const float *weights,
                                    int32_t B, int32_t N, int32_t abs_weights, double eps,
                                    double *T, pcr_stream_t stream) {
    return pcr::procrustes_launch(src, tgt, weights, B, N, abs_weights, eps, T, stream);
}

extern "C" int pcr_procrustes_batch_f64(const double *src, const double *tgt, const double *weights,
                                        int32_t B, int32_t N, int32_t abs_weights, double eps,
                                        double *T, pcr_stream_t stream) {
    return pcr::procrustes_launch(src, tgt, weights, B, N, abs_weights, eps, T, stream);
}

// ---------------------------------------------------------------------------
// apply per-item rigid transforms: out = (float)(R p + t) in f64, T (B,16)
// row-major 4x4 (the registration outputs).  The pipeline's "transform" stage
// (aligned source for the Chamfer quality check) -- one fused pass instead of a
// f64 batched GEMM plus casts.  float4 loads/stores over the flat (B*N*3) array.
// ---------------------------------------------------------------------------
namespace pcr {
namespace {
__global__ __launch_bounds__(256) void transform_kernel(const float *xyz, int N, const double *T,
                                                        float *out) {
    const int b = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const double *M = T + (size_t)b * 16;
    const float *p = xyz + ((size_t)b * N + i) * 3;
    double x, y, z;
    xform12(M, (double)p[0], (double)p[1], (double)p[2], x, y, z);
    float *o = out + ((size_t)b * N + i) * 3;
    o[0] = (float)x;
    o[1] = (float)y;
    o[2] = (float)z;
}
}  // namespace
}  // namespace pcr

extern "C" int pcr_transform_batch(const float *xyz, int32_t B, int32_t N, const double *T,
                                   float *out, pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(B >= 0 && N >= 0, PCR_ERR_ARG, "transform_batch: negative size");
    if (B == 0 || N == 0) return PCR_OK;
    PCR_REQUIRE(xyz && T && out, PCR_ERR_ARG, "transform_batch: null pointer");
    PCR_REQUIRE(B <= 65535, PCR_ERR_ARG, "transform_batch: B=%d > 65535", B);
    hipLaunchKernelGGL(pcr::transform_kernel, dim3((N + 255) / 256, B), dim3(256), 0,
                       pcr::as_stream(stream), xyz, N, T, out);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

// ---------------------------------------------------------------------------
// C4 pipeline records (pcr_pipeline_step): one 1024-thread block per pair; the
// Chamfer means as f64 sums of the f32 distances in a fixed order (thread t
// sums indices t, t + 1024, ... in 8-wide unrolled runs, then a fixed shuffle
// tree per wave and the 16 wave totals in order), then / N and / M.
// ---------------------------------------------------------------------------
namespace pcr {
namespace {
__global__ __launch_bounds__(1024) void pipeline_records_kernel(pcr_pipeline_io io) {
    const int p = blockIdx.x, t = threadIdx.x, lane = t & 63, wid = t >> 6;
    __shared__ double red[2][16];
    // loads of a run issued together (independent), summed in index order
    auto sum = [&](const float *d, int len) {
        double acc = 0.0;
        for (int i0 = t; i0 < len; i0 += 8 * 1024) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = i0 + u * 1024;
                v[u] = i < len ? d[i] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += (double)v[u];
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
        return acc;
    };
    const double s1 = sum(io.d1 + (size_t)p * io.N, io.N);
    const double s2 = sum(io.d2 + (size_t)p * io.M, io.M);
    if (lane == 0) { red[0][wid] = s1; red[1][wid] = s2; }
    __syncthreads();
    if (t == 0) {
        double a1 = 0.0, a2 = 0.0;
        for (int w = 0; w < 16; ++w) { a1 += red[0][w]; a2 += red[1][w]; }
        red[0][0] = a1;
        red[1][0] = a2;
    }
    __syncthreads();
    double *r = io.records + (size_t)p * 40;
    if (t < 16) {
        r[t] = io.T_ransac[(size_t)p * 16 + t];
        r[16 + t] = io.T_icp[(size_t)p * 16 + t];
    }
    if (t == 0) {
        r[32] = io.fit_ransac[2 * p];
        r[33] = io.fit_ransac[2 * p + 1];
        r[34] = io.fit_icp[2 * p];
        r[35] = io.fit_icp[2 * p + 1];
        r[36] = red[0][0] / (double)io.N + red[1][0] / (double)io.M;
        r[37] = (double)io.stats_ransac[(size_t)p * 5];
        r[38] = (double)io.stats_ransac[(size_t)p * 5 + 3];
        r[39] = (double)io.n_corres[p];
    }
}
}  // namespace

int pipeline_records(const pcr_pipeline_io *io, hipStream_t s) {
    PCR_REQUIRE(io->N >= 1 && io->M >= 1, PCR_ERR_ARG, "pipeline_records: empty clouds");
    hipLaunchKernelGGL(pipeline_records_kernel, dim3(io->P), dim3(1024), 0, s, *io);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}
}  // namespace pcr
