// a8: batched point-to-point ICP (Open3D 0.13 RegistrationICP as called from
// DataPreparation/RANSAC.py:61-63 and dip/preprocess_correspondences.py:48,83).
// Contract: oracle_icp (pcr_oracle.c).
//
// MI355X design: one 1024-thread workgroup per pair runs the whole ICP loop
// (no host round trips).  Per iteration: 1024 threads query the target hash grid
// for every (in-place transformed, f64) source point; Umeyama over the
// correspondences uses the deterministic 256-lane reduction (lane = source index
// mod 256, fixed halving tree), so the update is bit-reproducible; thread 0
// solves Horn and composes T <- U*T; convergence is decided in-kernel.
#include "pcr_internal.h"
#include "geom.h"
#include "grid.h"

namespace pcr {
namespace {

struct IArgs {
    const float *src, *tgt;
    const int32_t *n_src, *n_tgt;
    int Nmax, Mmax;
    const double *init;  // P x 16
    double d, thr, rel_fit, rel_rmse;
    int max_iter;
    GridBatch grid;
    double *P3;   // P x Nmax x 3 workspace
    int *cj;      // P x Nmax workspace
    double *T_out, *fit_out;
    int32_t *stats;
    int32_t *corr_tgt;  // optional (P, Nmax): final correspondence per source point
    const int32_t *order;  // (P, Nmax) spatial order of the source points, or null
};

__device__ __forceinline__ int cnt_of(const int32_t *n, int p, int mx) {
    return n ? min(max(n[p], 0), mx) : mx;
}

// fixed halving tree over red[0..256) x nv values (all 1024 threads call)
__device__ inline void tree256(double (*red)[9], int nv) {
    for (int s = 128; s >= 1; s >>= 1) {
        if ((int)threadIdx.x < s)
            for (int v = 0; v < nv; ++v) red[threadIdx.x][v] = red[threadIdx.x][v] + red[threadIdx.x + s][v];
        __syncthreads();
    }
}

struct IShared {  // LDS header; the grid copy (if any) follows
    double red[256][9];
    double T[16], U[12];
    unsigned long long s_acc[16];
    int s_cnt[16];
    double s_fit, s_rmse;
    int s_count;
    int chunk;  // next 64-query chunk of the current sweep
};

template <bool kLds>
__global__ __launch_bounds__(1024) void icp_kernel(IArgs a) {
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    IShared &sh = *reinterpret_cast<IShared *>(dsm);
    double (*red)[9] = sh.red;
    double *T = sh.T, *U = sh.U;
    const int p = blockIdx.x;
    const int n = cnt_of(a.n_src, p, a.Nmax);
    const int m = cnt_of(a.n_tgt, p, a.Mmax);
    const int tid = threadIdx.x;
    double *P3 = a.P3 + (size_t)p * a.Nmax * 3;
    int *cj = a.cj + (size_t)p * a.Nmax;
    const float *S = a.src + (size_t)p * a.Nmax * 3;
    const float *G = a.tgt + (size_t)p * a.Mmax * 3;
    if (tid < 16) T[tid] = a.init[(size_t)p * 16 + tid];
    if (tid == 0) sh.chunk = 0;
    __syncthreads();
    const bool valid = a.d > 0.0 && n > 0 && m > 0;
    bool ident = true;
    for (int k = 0; k < 16; ++k) ident = ident && (T[k] == ((k % 5 == 0) ? 1.0 : 0.0));
    for (int i = tid; i < n; i += 1024) {
        double x = (double)S[3 * i], y = (double)S[3 * i + 1], z = (double)S[3 * i + 2];
        if (!ident) {
            double ox, oy, oz;
            xform12(T, x, y, z, ox, oy, oz);
            x = ox; y = oy; z = oz;
        }
        P3[3 * i] = x; P3[3 * i + 1] = y; P3[3 * i + 2] = z;
    }
    GridT<uint16_t> gl{};
    GridView gg{};
    if (valid) {
        if constexpr (kLds) gl = grid_to_lds(a.grid, p, m, dsm + ((sizeof(IShared) + 15) & ~size_t(15)));
        else gg = a.grid.view(p);
    }
    __syncthreads();
    const double scale = fx_scale(a.thr);
    auto evaluate = [&]() {
        unsigned long long acc = 0;
        int cnt = 0;
        const int32_t *ord = a.order ? a.order + (size_t)p * a.Nmax : nullptr;
        const int nch = (n + 63) >> 6, lane = tid & 63;
        for (;;) {  // 64-query chunks in spatial order, taken dynamically
            int c = 0;
            if (lane == 0) c = atomicAdd(&sh.chunk, 1);
            c = __shfl(c, 0, 64);
            if (c >= nch) break;
            const int k = (c << 6) + lane;
            if (k < n) {
                const int i = ord ? ord[k] : k;
                double d2;
                int j;
                if constexpr (kLds) j = grid_query(gl, a.d, a.thr, P3[3 * i], P3[3 * i + 1], P3[3 * i + 2], d2);
                else j = grid_query(gg, a.d, a.thr, P3[3 * i], P3[3 * i + 1], P3[3 * i + 2], d2);
                cj[i] = j;
                if (j >= 0) { ++cnt; acc += (unsigned long long)(d2 * scale); }
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            acc += __shfl_xor(acc, o, 64);
            cnt += __shfl_xor(cnt, o, 64);
        }
        if ((tid & 63) == 0) { sh.s_acc[tid >> 6] = acc; sh.s_cnt[tid >> 6] = cnt; }
        __syncthreads();
        if (tid == 0) {
            unsigned long long A = 0;
            int C = 0;
            for (int w = 0; w < 16; ++w) { A += sh.s_acc[w]; C += sh.s_cnt[w]; }
            sh.s_count = C;
            sh.chunk = 0;  // next sweep (published by the barrier below)
            if (C > 0) {
                sh.s_fit = (double)C / (double)n;
                sh.s_rmse = __builtin_sqrt(((double)A / scale) / (double)C);
            } else {
                sh.s_fit = 0.0;
                sh.s_rmse = 0.0;
            }
        }
        __syncthreads();
    };
    int it = 0;
    if (valid) {
        evaluate();
        for (it = 0; it < a.max_iter;) {
            if (sh.s_count == 0) break;
            // --- Umeyama over correspondences: means
            if (tid < 256) {
                double v[6] = {0, 0, 0, 0, 0, 0};
                // four entries of this lane's sequence are loaded before they are
                // added in sequence order: the same sums, overlapped gathers
                int i = tid;
                for (; i + 768 < n; i += 1024) {
                    int jj[4];
                    double a3[4][3], b3[4][3];
#pragma unroll
                    for (int u = 0; u < 4; ++u) jj[u] = cj[i + 256 * u];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int ii = i + 256 * u, j = jj[u] < 0 ? 0 : jj[u];
                        a3[u][0] = P3[3 * ii]; a3[u][1] = P3[3 * ii + 1]; a3[u][2] = P3[3 * ii + 2];
                        b3[u][0] = (double)G[3 * j]; b3[u][1] = (double)G[3 * j + 1]; b3[u][2] = (double)G[3 * j + 2];
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (jj[u] >= 0) {
                            v[0] = v[0] + a3[u][0];
                            v[1] = v[1] + a3[u][1];
                            v[2] = v[2] + a3[u][2];
                            v[3] = v[3] + b3[u][0];
                            v[4] = v[4] + b3[u][1];
                            v[5] = v[5] + b3[u][2];
                        }
                }
                for (; i < n; i += 256) {
                    const int j = cj[i];
                    if (j < 0) continue;
                    v[0] = v[0] + P3[3 * i];
                    v[1] = v[1] + P3[3 * i + 1];
                    v[2] = v[2] + P3[3 * i + 2];
                    v[3] = v[3] + (double)G[3 * j];
                    v[4] = v[4] + (double)G[3 * j + 1];
                    v[5] = v[5] + (double)G[3 * j + 2];
                }
                for (int k = 0; k < 6; ++k) red[tid][k] = v[k];
            }
            __syncthreads();
            tree256(red, 6);
            const double inv = 1.0 / (double)sh.s_count;
            const double ms0 = red[0][0] * inv, ms1 = red[0][1] * inv, ms2 = red[0][2] * inv;
            const double mt0 = red[0][3] * inv, mt1 = red[0][4] * inv, mt2 = red[0][5] * inv;
            __syncthreads();
            // --- cross covariance
            if (tid < 256) {
                double v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
                auto add = [&](double s0, double s1, double s2, double t0, double t1, double t2) {
                    v[0] = v[0] + s0 * t0; v[1] = v[1] + s0 * t1; v[2] = v[2] + s0 * t2;
                    v[3] = v[3] + s1 * t0; v[4] = v[4] + s1 * t1; v[5] = v[5] + s1 * t2;
                    v[6] = v[6] + s2 * t0; v[7] = v[7] + s2 * t1; v[8] = v[8] + s2 * t2;
                };
                int i = tid;
                for (; i + 768 < n; i += 1024) {  // as above: loads first, sums in order
                    int jj[4];
                    double a3[4][3], b3[4][3];
#pragma unroll
                    for (int u = 0; u < 4; ++u) jj[u] = cj[i + 256 * u];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int ii = i + 256 * u, j = jj[u] < 0 ? 0 : jj[u];
                        a3[u][0] = P3[3 * ii] - ms0; a3[u][1] = P3[3 * ii + 1] - ms1; a3[u][2] = P3[3 * ii + 2] - ms2;
                        b3[u][0] = (double)G[3 * j] - mt0; b3[u][1] = (double)G[3 * j + 1] - mt1;
                        b3[u][2] = (double)G[3 * j + 2] - mt2;
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (jj[u] >= 0) add(a3[u][0], a3[u][1], a3[u][2], b3[u][0], b3[u][1], b3[u][2]);
                }
                for (; i < n; i += 256) {
                    const int j = cj[i];
                    if (j < 0) continue;
                    add(P3[3 * i] - ms0, P3[3 * i + 1] - ms1, P3[3 * i + 2] - ms2, (double)G[3 * j] - mt0,
                        (double)G[3 * j + 1] - mt1, (double)G[3 * j + 2] - mt2);
                }
                for (int k = 0; k < 9; ++k) red[tid][k] = v[k];
            }
            __syncthreads();
            tree256(red, 9);
            if (tid == 0) {
                double Sm[9], R[9], ms[3] = {ms0, ms1, ms2}, mt[3] = {mt0, mt1, mt2};
                for (int k = 0; k < 9; ++k) Sm[k] = red[0][k];
                horn_rotation(Sm, R);
                compose_rt(R, ms, mt, U);
                double Tn[16];
                for (int r = 0; r < 4; ++r)
                    for (int c = 0; c < 4; ++c) {
                        const double u0 = r < 3 ? U[4 * r + 0] : 0.0, u1 = r < 3 ? U[4 * r + 1] : 0.0,
                                     u2 = r < 3 ? U[4 * r + 2] : 0.0, u3 = r < 3 ? U[4 * r + 3] : 1.0;
                        Tn[4 * r + c] =
                            ((u0 * T[c] + u1 * T[4 + c]) + u2 * T[8 + c]) + u3 * T[12 + c];
                    }
                for (int k = 0; k < 16; ++k) T[k] = Tn[k];
            }
            __syncthreads();
            for (int i = tid; i < n; i += 1024) {
                double ox, oy, oz;
                xform12(U, P3[3 * i], P3[3 * i + 1], P3[3 * i + 2], ox, oy, oz);
                P3[3 * i] = ox; P3[3 * i + 1] = oy; P3[3 * i + 2] = oz;
            }
            __syncthreads();
            const double pf = sh.s_fit, pr = sh.s_rmse;
            __syncthreads();
            evaluate();
            ++it;
            if (__builtin_fabs(pf - sh.s_fit) < a.rel_fit && __builtin_fabs(pr - sh.s_rmse) < a.rel_rmse) break;
        }
    }
    if (a.corr_tgt)
        for (int i = tid; i < a.Nmax; i += 1024)
            a.corr_tgt[(size_t)p * a.Nmax + i] = (valid && i < n) ? cj[i] : -1;
    if (tid == 0) {
        for (int k = 0; k < 16; ++k) a.T_out[(size_t)p * 16 + k] = T[k];
        a.fit_out[2 * p] = valid ? sh.s_fit : 0.0;
        a.fit_out[2 * p + 1] = valid ? sh.s_rmse : 0.0;
        a.stats[2 * p] = it;
        a.stats[2 * p + 1] = valid ? sh.s_count : 0;
    }
}

}  // namespace

int icp_impl(const float *src, const float *tgt, int P, int Nmax, int Mmax, const int32_t *n_src,
             const int32_t *n_tgt, const double *init, const pcr_icp_params *prm, double *T_out,
             double *fit_out, int32_t *stats, int32_t *corr_tgt, hipStream_t s) {
    IArgs a;
    a.src = src; a.tgt = tgt; a.n_src = n_src; a.n_tgt = n_tgt; a.Nmax = Nmax; a.Mmax = Mmax;
    a.init = init;
    a.order = nullptr;
    a.d = prm->max_correspondence_distance;
    a.thr = radius_thr(a.d);
    a.rel_fit = prm->relative_fitness;
    a.rel_rmse = prm->relative_rmse;
    a.max_iter = prm->max_iteration;
    if (a.d > 0.0) {
        int rc = build_grids(tgt, n_tgt, P, Mmax, a.d, s, 7, a.grid);
        if (rc != PCR_OK) return rc;
        if (Nmax > 0) {
            rc = spatial_order(src, n_src, P, Nmax, a.grid.cell, s, 14, &a.order);
            if (rc != PCR_OK) return rc;
        }
    } else {
        a.grid = GridBatch{};
        a.grid.S = 1;
        a.grid.cell = 1.0;
    }
    char *ws = (char *)workspace(8, (sizeof(double) * 3 + sizeof(int)) * (size_t)P * (Nmax ? Nmax : 1) + 64);
    PCR_REQUIRE(ws, PCR_ERR_NOMEM, "icp: %s", pcr_last_error());
    a.P3 = (double *)ws;
    a.cj = (int *)(ws + sizeof(double) * 3 * (size_t)P * (Nmax ? Nmax : 1));
    a.T_out = T_out; a.fit_out = fit_out; a.stats = stats; a.corr_tgt = corr_tgt;
    const size_t hdr = (sizeof(IShared) + 15) & ~size_t(15);
    const size_t gbytes = (a.d > 0.0 && Mmax > 0) ? grid_lds_bytes(Mmax, a.grid.S, 160 * 1024 - hdr) : 0;
    prof_begin(s, kProfIcp);
    if (gbytes > 0) {
        PCR_HIP_CHECK(hipFuncSetAttribute((const void *)icp_kernel<true>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)(hdr + gbytes)));
        hipLaunchKernelGGL(icp_kernel<true>, dim3(P), dim3(1024), hdr + gbytes, s, a);
    } else {
        PCR_HIP_CHECK(hipFuncSetAttribute((const void *)icp_kernel<false>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)hdr));
        hipLaunchKernelGGL(icp_kernel<false>, dim3(P), dim3(1024), hdr, s, a);
    }
    PCR_LAUNCH_CHECK();
    prof_end(s, kProfIcp);
    return PCR_OK;
}

}  // namespace pcr

extern "C" int pcr_icp_batch(const float *src_xyz, const float *tgt_xyz, int32_t P, int32_t Nmax,
                             int32_t Mmax, const int32_t *n_src, const int32_t *n_tgt,
                             const double *init, const pcr_icp_params *params, double *T,
                             double *fitness_rmse, int32_t *stats, int32_t *corr_tgt,
                             pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(P >= 0 && Nmax >= 0 && Mmax >= 0, PCR_ERR_ARG, "icp: negative size");
    if (P == 0) return PCR_OK;
    PCR_REQUIRE(src_xyz && tgt_xyz && init && params && T && fitness_rmse && stats, PCR_ERR_ARG,
                "icp: null pointer");
    return pcr::icp_impl(src_xyz, tgt_xyz, P, Nmax, Mmax, n_src, n_tgt, init, params, T,
                         fitness_rmse, stats, corr_tgt, pcr::as_stream(stream));
}
