// a6/a7: batched RANSAC hypothesize-and-verify over P cloud pairs.
//
// Reference: Open3D 0.13 RegistrationRANSACBasedOnCorrespondence as driven by
// registration_ransac_based_on_feature_matching (DataPreparation/RANSAC.py:43-52,
// dip/demo.py:43-52, c2p-net/ngenet/utils/o3d.py:174-180).  Contract: the
// SEQUENTIAL loop of oracle_ransac (pcr_oracle.c) on the Philox hypothesis stream
// keyed by (seed, pair, itr).
//
// MI355X design: hypotheses are processed in waves of W iterations for all pairs
// at once.  (1) one thread per (pair, itr) samples, solves Umeyama (Horn, f64)
// and runs the checkers; (2) one workgroup per surviving hypothesis transforms
// every source point and queries the target hash grid (the HBM/L2-bound kernel),
// reducing inlier count and a fixed-point error sum (exact, order-free), plus the
// inlier ratio over the correspondence set; (3) one thread per pair replays the
// wave IN ITERATION ORDER with Open3D's update rule (better = fitness up, or tie
// and rmse down; est_k = min(est_k, ceil(log(1-conf)/log(1-w^n)))).  Hypotheses
// beyond the bound are evaluated but ignored, so the result is exactly the
// sequential one, independent of W and scheduling.  The host reads one counter
// per wave to stop (W doubles each wave up to 1024).
#include "pcr_internal.h"
#include "geom.h"
#include "grid.h"

namespace pcr {
namespace {

constexpr int kMaxRansacN = 8;

struct HypRec {
    double T[12];
    double fit, rmse;
    int pass;  // -1 skipped, 0 failed checks, 1 passed
    int cin;   // corres inliers (d2 < d*d)
};

struct PairState {
    double T[12];
    double fit, rmse;
    int est_k, iters, validated, best_itr;
    int done, status, pad0, pad1;
};

struct RArgs {
    const float *src, *tgt;
    const int32_t *n_src, *n_tgt;
    const int32_t *corres, *n_corres;
    const uint32_t *pair_ids;
    int Nmax, Mmax, Kmax;
    double d, thr, dd, edge, dcheck, conf;
    int rn, max_iter;
    uint64_t seed;
    GridBatch grid;
    PairState *st;
    HypRec *rec;  // P x W
    int base, W;
    int *remaining;
};

__device__ __forceinline__ int cnt_of(const int32_t *n, int p, int mx) {
    return n ? min(max(n[p], 0), mx) : mx;
}

__global__ void ransac_init(RArgs a, int P) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    PairState &s = a.st[p];
    for (int k = 0; k < 12; ++k) s.T[k] = (k % 5 == 0) ? 1.0 : 0.0;
    s.fit = 0.0; s.rmse = 0.0;
    s.est_k = a.max_iter; s.iters = 0; s.validated = 0; s.best_itr = -1;
    const int K = a.n_corres ? min(max(a.n_corres[p], 0), a.Kmax) : a.Kmax;
    const bool ok = a.rn >= 3 && a.rn <= kMaxRansacN && K >= a.rn && a.d > 0.0 &&
                    cnt_of(a.n_src, p, a.Nmax) > 0 && cnt_of(a.n_tgt, p, a.Mmax) > 0;
    s.done = ok ? 0 : 1;
    s.status = ok ? 0 : -1;
}

__global__ void ransac_hyp(RArgs a, int P) {
    const int h = blockIdx.x * blockDim.x + threadIdx.x;
    const int p = blockIdx.y;
    if (h >= a.W) return;
    HypRec &r = a.rec[(size_t)p * a.W + h];
    const PairState &s = a.st[p];
    const int itr = a.base + h;
    if (s.done || itr >= a.max_iter || itr >= s.est_k) { r.pass = -1; return; }
    const int K = a.n_corres ? min(max(a.n_corres[p], 0), a.Kmax) : a.Kmax;
    const uint32_t pid = a.pair_ids ? a.pair_ids[p] : (uint32_t)p;
    const int32_t *co = a.corres + (size_t)p * a.Kmax * 2;
    const float *S = a.src + (size_t)p * a.Nmax * 3;
    const float *G = a.tgt + (size_t)p * a.Mmax * 3;
    double ss[3 * kMaxRansacN], tt[3 * kMaxRansacN];
    for (int j = 0; j < a.rn; ++j) {
        const int c = sample_index(a.seed, pid, (uint32_t)itr, j, K);
        const int si = co[2 * c], ti = co[2 * c + 1];
        for (int q = 0; q < 3; ++q) {
            ss[3 * j + q] = (double)S[3 * si + q];
            tt[3 * j + q] = (double)G[3 * ti + q];
        }
    }
    // Umeyama on the minimal sample (sequential sums, Eigen mean = sum * (1/n))
    double ms[3] = {0, 0, 0}, mt[3] = {0, 0, 0};
    for (int j = 0; j < a.rn; ++j)
        for (int q = 0; q < 3; ++q) { ms[q] = ms[q] + ss[3 * j + q]; mt[q] = mt[q] + tt[3 * j + q]; }
    const double inv = 1.0 / (double)a.rn;
    for (int q = 0; q < 3; ++q) { ms[q] = ms[q] * inv; mt[q] = mt[q] * inv; }
    double Sm[9];
    for (int k = 0; k < 9; ++k) Sm[k] = 0.0;
    for (int j = 0; j < a.rn; ++j)
        for (int x = 0; x < 3; ++x)
            for (int y = 0; y < 3; ++y)
                Sm[3 * x + y] = Sm[3 * x + y] + (ss[3 * j + x] - ms[x]) * (tt[3 * j + y] - mt[y]);
    double R[9];
    horn_rotation(Sm, R);
    compose_rt(R, ms, mt, r.T);
    bool ok = true;
    if (a.edge > 0.0) {
        for (int i = 0; i < a.rn && ok; ++i)
            for (int j = i + 1; j < a.rn && ok; ++j) {
                const double ds = __builtin_sqrt(dist2(ss[3 * i], ss[3 * i + 1], ss[3 * i + 2],
                                                       ss[3 * j], ss[3 * j + 1], ss[3 * j + 2]));
                const double dt = __builtin_sqrt(dist2(tt[3 * i], tt[3 * i + 1], tt[3 * i + 2],
                                                       tt[3 * j], tt[3 * j + 1], tt[3 * j + 2]));
                if (ds < dt * a.edge || dt < ds * a.edge) ok = false;
            }
    }
    if (ok && a.dcheck > 0.0) {
        for (int j = 0; j < a.rn && ok; ++j) {
            double px, py, pz;
            xform12(r.T, ss[3 * j], ss[3 * j + 1], ss[3 * j + 2], px, py, pz);
            if (__builtin_sqrt(dist2(px, py, pz, tt[3 * j], tt[3 * j + 1], tt[3 * j + 2])) > a.dcheck)
                ok = false;
        }
    }
    r.pass = ok ? 1 : 0;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// one 256-thread block per (hypothesis h, pair p)
__global__ __launch_bounds__(256) void ransac_validate(RArgs a) {
    const int h = blockIdx.x, p = blockIdx.y;
    HypRec &r = a.rec[(size_t)p * a.W + h];
    if (r.pass != 1) return;
    __shared__ double T[12];
    __shared__ unsigned long long s_acc[4];
    __shared__ int s_cnt[4], s_cin[4];
    if (threadIdx.x < 12) T[threadIdx.x] = r.T[threadIdx.x];
    __syncthreads();
    const int n = cnt_of(a.n_src, p, a.Nmax);
    const float *S = a.src + (size_t)p * a.Nmax * 3;
    const GridView g = a.grid.view(p);
    const double scale = fx_scale(a.thr);
    unsigned long long acc = 0;
    int cnt = 0;
    for (int i = threadIdx.x; i < n; i += 256) {
        double px, py, pz, d2;
        xform12(T, (double)S[3 * i], (double)S[3 * i + 1], (double)S[3 * i + 2], px, py, pz);
        const int j = grid_query(g, a.d, a.thr, px, py, pz, d2);
        if (j >= 0) { ++cnt; acc += (unsigned long long)(d2 * scale); }
    }
    // inlier ratio over the correspondence set (EvaluateInlierCorrespondenceRatio)
    const int K = a.n_corres ? min(max(a.n_corres[p], 0), a.Kmax) : a.Kmax;
    const int32_t *co = a.corres + (size_t)p * a.Kmax * 2;
    const float *G = a.tgt + (size_t)p * a.Mmax * 3;
    int cin = 0;
    for (int k = threadIdx.x; k < K; k += 256) {
        const int si = co[2 * k], ti = co[2 * k + 1];
        double px, py, pz;
        xform12(T, (double)S[3 * si], (double)S[3 * si + 1], (double)S[3 * si + 2], px, py, pz);
        if (dist2(px, py, pz, (double)G[3 * ti], (double)G[3 * ti + 1], (double)G[3 * ti + 2]) < a.dd)
            ++cin;
    }
    acc = wave_sum_u64(acc);
    cnt = wave_sum_i(cnt);
    cin = wave_sum_i(cin);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { s_acc[w] = acc; s_cnt[w] = cnt; s_cin[w] = cin; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long A = 0;
        int C = 0, CI = 0;
        for (int k = 0; k < 4; ++k) { A += s_acc[k]; C += s_cnt[k]; CI += s_cin[k]; }
        if (C > 0) {
            r.fit = (double)C / (double)n;
            r.rmse = __builtin_sqrt(((double)A / scale) / (double)C);
        } else {
            r.fit = 0.0;
            r.rmse = 0.0;
        }
        r.cin = CI;
    }
}

__global__ void ransac_select(RArgs a, int P) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    PairState &s = a.st[p];
    if (s.done) return;
    const int K = a.n_corres ? min(max(a.n_corres[p], 0), a.Kmax) : a.Kmax;
    int itr = a.base;
    bool stop = false;
    for (int h = 0; h < a.W; ++h, ++itr) {
        if (itr >= a.max_iter || itr >= s.est_k) { stop = true; break; }
        const HypRec &r = a.rec[(size_t)p * a.W + h];
        if (r.pass != 1) continue;
        s.validated += 1;
        if (r.fit > s.fit || (r.fit == s.fit && r.rmse < s.rmse)) {
            s.fit = r.fit;
            s.rmse = r.rmse;
            s.best_itr = itr;
            for (int k = 0; k < 12; ++k) s.T[k] = r.T[k];
            const double kd = est_k_bound((double)r.cin / (double)K, a.rn, a.conf);
            if (kd < (double)s.est_k) s.est_k = (int)__builtin_ceil(kd);
        }
    }
    if (!stop && (itr >= a.max_iter || itr >= s.est_k)) stop = true;
    s.iters = itr;
    if (stop) {
        s.done = 1;
        s.status = s.best_itr >= 0 ? 1 : 0;
    } else {
        atomicAdd(a.remaining, 1);
    }
}

// correspondence set / inlier mask of the best transformation
struct FArgs {
    const float *src;
    const int32_t *n_src;
    int Nmax, words;
    double d, thr;
    GridBatch grid;
    const PairState *st;
    double *T_out, *fit_out;
    int32_t *stats, *corr_tgt;
    uint32_t *mask;
};

__global__ __launch_bounds__(256) void ransac_final(FArgs a) {
    const int p = blockIdx.x;
    const PairState &s = a.st[p];
    const int n = cnt_of(a.n_src, p, a.Nmax);
    __shared__ int s_cnt[4];
    const bool found = s.status == 1;
    const GridView g = a.grid.view(p);
    const float *S = a.src + (size_t)p * a.Nmax * 3;
    int cnt = 0;
    for (int base = 0; base < a.Nmax; base += 256) {
        const int i = base + threadIdx.x;
        int j = -1;
        if (found && i < n) {
            double px, py, pz, d2;
            xform12(s.T, (double)S[3 * i], (double)S[3 * i + 1], (double)S[3 * i + 2], px, py, pz);
            j = grid_query(g, a.d, a.thr, px, py, pz, d2);
        }
        if (i < a.Nmax && a.corr_tgt) a.corr_tgt[(size_t)p * a.Nmax + i] = j;
        cnt += (j >= 0);
        if (a.mask) {
            const unsigned long long bits = __ballot(j >= 0);
            const int l = threadIdx.x & 63;
            const int word = (base + (threadIdx.x & ~63)) >> 5;
            if (l == 0 && word < a.words) a.mask[(size_t)p * a.words + word] = (uint32_t)bits;
            if (l == 32 && word + 1 < a.words) a.mask[(size_t)p * a.words + word + 1] = (uint32_t)(bits >> 32);
        }
    }
    cnt = wave_sum_i(cnt);
    if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        double *T = a.T_out + (size_t)p * 16;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) T[4 * r + c] = s.T[4 * r + c];
        T[12] = 0.0; T[13] = 0.0; T[14] = 0.0; T[15] = 1.0;
        a.fit_out[2 * p] = s.fit;
        a.fit_out[2 * p + 1] = s.rmse;
        int32_t *st = a.stats + (size_t)p * 5;
        st[0] = s.iters;
        st[1] = s.validated;
        st[2] = s.best_itr;
        st[3] = s.status;
        st[4] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
    }
}

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace

int ransac_impl(const float *src, const float *tgt, int P, int Nmax, int Mmax,
                const int32_t *n_src, const int32_t *n_tgt, const int32_t *corres,
                const int32_t *n_corres, int Kmax, const uint32_t *pair_ids,
                const pcr_ransac_params *prm, double *T_out, double *fit_out, int32_t *stats,
                int32_t *corr_tgt, uint32_t *mask, hipStream_t s) {
    PCR_REQUIRE(prm->ransac_n >= 3 && prm->ransac_n <= kMaxRansacN, PCR_ERR_ARG,
                "ransac: ransac_n=%d unsupported (3..%d)", prm->ransac_n, kMaxRansacN);
    RArgs a;
    a.src = src; a.tgt = tgt; a.n_src = n_src; a.n_tgt = n_tgt; a.corres = corres;
    a.n_corres = n_corres; a.pair_ids = pair_ids; a.Nmax = Nmax; a.Mmax = Mmax; a.Kmax = Kmax;
    a.d = prm->max_correspondence_distance;
    a.thr = radius_thr(a.d);
    a.dd = a.d * a.d;
    a.edge = prm->edge_length_ratio;
    a.dcheck = prm->distance_check;
    a.conf = prm->confidence;
    a.rn = prm->ransac_n;
    a.max_iter = prm->max_iteration;
    a.seed = prm->seed;
    if (a.d > 0.0) {
        int rc = build_grids(tgt, n_tgt, P, Mmax, a.d, s, 4, a.grid);
        if (rc != PCR_OK) return rc;
    } else {
        a.grid = GridBatch{nullptr, nullptr, 1, 0, 1.0};
    }
    constexpr int kWmax = 1024;
    char *ws = (char *)workspace(5, sizeof(PairState) * (size_t)P + sizeof(HypRec) * (size_t)P * kWmax + 64);
    PCR_REQUIRE(ws, PCR_ERR_NOMEM, "ransac: %s", pcr_last_error());
    a.st = (PairState *)ws;
    a.rec = (HypRec *)(ws + ((sizeof(PairState) * (size_t)P + 15) & ~size_t(15)));
    int *dev_rem = (int *)workspace(6, 64);
    PCR_REQUIRE(dev_rem, PCR_ERR_NOMEM, "ransac: %s", pcr_last_error());
    a.remaining = dev_rem;
    static thread_local int *host_rem = nullptr;
    if (!host_rem) PCR_HIP_CHECK(hipHostMalloc((void **)&host_rem, sizeof(int)));
    hipLaunchKernelGGL(ransac_init, dim3(cdiv(P, 256)), dim3(256), 0, s, a, P);
    PCR_LAUNCH_CHECK();
    int W = 64;
    for (a.base = 0; a.base < a.max_iter;) {
        a.W = W;
        PCR_HIP_CHECK(hipMemsetAsync(dev_rem, 0, sizeof(int), s));
        prof_begin(s, kProfRansacHyp);
        hipLaunchKernelGGL(ransac_hyp, dim3(cdiv(W, 64), P), dim3(64), 0, s, a, P);
        PCR_LAUNCH_CHECK();
        prof_end(s, kProfRansacHyp);
        prof_begin(s, kProfRansacValidate);
        hipLaunchKernelGGL(ransac_validate, dim3(W, P), dim3(256), 0, s, a);
        PCR_LAUNCH_CHECK();
        prof_end(s, kProfRansacValidate);
        hipLaunchKernelGGL(ransac_select, dim3(cdiv(P, 256)), dim3(256), 0, s, a, P);
        PCR_LAUNCH_CHECK();
        PCR_HIP_CHECK(hipMemcpyAsync(host_rem, dev_rem, sizeof(int), hipMemcpyDeviceToHost, s));
        PCR_HIP_CHECK(hipStreamSynchronize(s));
        a.base += W;
        if (*host_rem == 0) break;
        W = W * 2 > kWmax ? kWmax : W * 2;
    }
    FArgs f;
    f.src = src; f.n_src = n_src; f.Nmax = Nmax; f.words = cdiv(Nmax, 32); f.d = a.d;
    f.thr = a.thr; f.grid = a.grid; f.st = a.st; f.T_out = T_out; f.fit_out = fit_out;
    f.stats = stats; f.corr_tgt = corr_tgt; f.mask = mask;
    hipLaunchKernelGGL(ransac_final, dim3(P), dim3(256), 0, s, f);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

}  // namespace pcr

extern "C" int pcr_ransac_batch(const float *src_xyz, const float *tgt_xyz, int32_t P,
                                int32_t Nmax, int32_t Mmax, const int32_t *n_src,
                                const int32_t *n_tgt, const int32_t *corres,
                                const int32_t *n_corres, int32_t Kmax, const uint32_t *pair_ids,
                                const pcr_ransac_params *params, double *T, double *fitness_rmse,
                                int32_t *stats, int32_t *corr_tgt, uint32_t *inlier_mask,
                                pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(P >= 0 && Nmax >= 0 && Mmax >= 0 && Kmax >= 0, PCR_ERR_ARG, "ransac: negative size");
    if (P == 0) return PCR_OK;
    PCR_REQUIRE(src_xyz && tgt_xyz && corres && params && T && fitness_rmse && stats, PCR_ERR_ARG,
                "ransac: null pointer");
    PCR_REQUIRE(P <= 65535, PCR_ERR_ARG, "ransac: P=%d > 65535", P);
    return pcr::ransac_impl(src_xyz, tgt_xyz, P, Nmax, Mmax, n_src, n_tgt, corres, n_corres, Kmax,
                            pair_ids, params, T, fitness_rmse, stats, corr_tgt, inlier_mask,
                            pcr::as_stream(stream));
}
