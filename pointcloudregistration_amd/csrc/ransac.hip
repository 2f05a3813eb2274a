// a6/a7: batched RANSAC hypothesize-and-verify over P cloud pairs.
//
// Reference: Open3D 0.13 RegistrationRANSACBasedOnCorrespondence as driven by
// registration_ransac_based_on_feature_matching (DataPreparation/RANSAC.py:43-52,
// dip/demo.py:43-52, c2p-net/ngenet/utils/o3d.py:174-180).  Contract: the
// SEQUENTIAL loop of oracle_ransac (pcr_oracle.c) on the Philox hypothesis stream
// keyed by (seed, pair_id, itr).
//
// MI355X design: ONE persistent 1024-thread workgroup per pair, one launch for
// the whole RANSAC of all pairs (no host round trips):
//  * the pair's target hash grid is copied into LDS (u16 indices, 128 KiB at
//    8192 points; global-memory grid when it does not fit);
//  * 1024 hypotheses at a time, one per thread: Philox sample, Umeyama (Horn,
//    f64), edge-length and distance checkers;
//  * the passing ones are compacted IN ITERATION ORDER (wave ballots + prefix);
//  * they are then validated one after another by the whole workgroup (every
//    thread transforms and queries 8 source points; inlier count + exact
//    fixed-point error sum; inlier ratio over the correspondences), and
//    thread 0 applies Open3D's update rule with the live bound
//    est_k = min(est_k, ceil(log(1-conf)/log(1-w^n))) -- hypotheses at or beyond
//    the bound are never validated, so no work is wasted and the result is
//    exactly the sequential one;
//  * the correspondence set / inlier mask of the best transformation is written
//    by the same launch.
#include "pcr_internal.h"
#include "geom.h"
#include "grid.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace pcr {
namespace {

constexpr int kMaxRansacN = 8;
constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;
constexpr int kCap = 128;  // passing hypotheses kept per hypothesis wave

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
    double *T_out, *fit_out;
    int32_t *stats, *corr_tgt;
    uint32_t *mask;
    int words;
    unsigned long long *timing;  // debug (PCR_RANSAC_TIMING): per pair, 6 phase clocks
    const int32_t *order;        // (P, Nmax) spatial order of the source points, or null
    int32_t *cand;               // (P, 2, Nmax): target index per source point of a sweep,
                                 // two buffers: the best hypothesis' and the current one's
};

__device__ __forceinline__ int cnt_of(const int32_t *n, int p, int mx) {
    return n ? min(max(n[p], 0), mx) : mx;
}

// hypothesis `itr`: sample, Umeyama (Horn), checkers; T written, returns pass.
// RN = ransac_n (compile time so the sample arrays stay in registers)
template <int RN>
__device__ bool make_hypothesis(const RArgs &a, int p, int K, uint32_t pid, int itr, double *T) {
    const int32_t *co = a.corres + (size_t)p * a.Kmax * 2;
    const float *S = a.src + (size_t)p * a.Nmax * 3;
    const float *G = a.tgt + (size_t)p * a.Mmax * 3;
    double ss[3 * RN], tt[3 * RN];
#pragma unroll
    for (int j = 0; j < RN; ++j) {
        const int c = sample_index(a.seed, pid, (uint32_t)itr, j, K);
        const int si = co[2 * c], ti = co[2 * c + 1];
        for (int q = 0; q < 3; ++q) {
            ss[3 * j + q] = (double)S[3 * si + q];
            tt[3 * j + q] = (double)G[3 * ti + q];
        }
    }
    // Umeyama on the minimal sample (sequential sums, Eigen mean = sum * (1/n))
    double ms[3] = {0, 0, 0}, mt[3] = {0, 0, 0};
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int q = 0; q < 3; ++q) { ms[q] = ms[q] + ss[3 * j + q]; mt[q] = mt[q] + tt[3 * j + q]; }
    const double inv = 1.0 / (double)RN;
    for (int q = 0; q < 3; ++q) { ms[q] = ms[q] * inv; mt[q] = mt[q] * inv; }
    double Sm[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) Sm[k] = 0.0;
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int x = 0; x < 3; ++x)
#pragma unroll
            for (int y = 0; y < 3; ++y)
                Sm[3 * x + y] = Sm[3 * x + y] + (ss[3 * j + x] - ms[x]) * (tt[3 * j + y] - mt[y]);
    double R[9];
    horn_rotation(Sm, R);
    compose_rt(R, ms, mt, T);
    if (a.edge > 0.0) {
#pragma unroll
        for (int i = 0; i < RN; ++i)
#pragma unroll
            for (int j = i + 1; j < RN; ++j) {
                const double ds = __builtin_sqrt(dist2(ss[3 * i], ss[3 * i + 1], ss[3 * i + 2],
                                                       ss[3 * j], ss[3 * j + 1], ss[3 * j + 2]));
                const double dt = __builtin_sqrt(dist2(tt[3 * i], tt[3 * i + 1], tt[3 * i + 2],
                                                       tt[3 * j], tt[3 * j + 1], tt[3 * j + 2]));
                if (ds < dt * a.edge || dt < ds * a.edge) return false;
            }
    }
    if (a.dcheck > 0.0) {
#pragma unroll
        for (int j = 0; j < RN; ++j) {
            double px, py, pz;
            xform12(T, ss[3 * j], ss[3 * j + 1], ss[3 * j + 2], px, py, pz);
            if (__builtin_sqrt(dist2(px, py, pz, tt[3 * j], tt[3 * j + 1], tt[3 * j + 2])) > a.dcheck)
                return false;
        }
    }
    return true;
}

struct Shared {  // LDS header (the grid copy follows)
    double listT[kCap][12];
    int listItr[kCap];
    int wcnt[kWaves];
    unsigned long long racc[kWaves];
    int rcnt[kWaves], rcin[kWaves];
    double bestT[12];
    double best_fit, best_rmse;
    int est_k, best_itr, validated, last_upd, base, found;
    int chunk;     // next 64-query chunk of the current sweep (dynamic balance across waves)
    int misses;    // source points without a correspondence so far in this sweep
    int best_cnt;  // inlier count of the best hypothesis (0: none yet)
    int cur_buf, best_buf;  // cand buffer of the running sweep / of the best hypothesis
};

template <bool kLds, int RN>
__global__ __launch_bounds__(kThreads) void ransac_pair_kernel(RArgs a) {
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    Shared &sh = *reinterpret_cast<Shared *>(dsm);
    const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int n = cnt_of(a.n_src, p, a.Nmax), m = cnt_of(a.n_tgt, p, a.Mmax);
    const int K = a.n_corres ? min(max(a.n_corres[p], 0), a.Kmax) : a.Kmax;
    const uint32_t pid = a.pair_ids ? a.pair_ids[p] : (uint32_t)p;
    const bool ok = K >= RN && a.d > 0.0 && n > 0 && m > 0;
    if (tid == 0) {
        for (int k = 0; k < 12; ++k) sh.bestT[k] = (k % 5 == 0) ? 1.0 : 0.0;
        sh.best_fit = 0.0; sh.best_rmse = 0.0;
        sh.est_k = a.max_iter; sh.best_itr = -1; sh.validated = 0; sh.last_upd = -1; sh.base = 0;
        sh.chunk = 0; sh.misses = 0; sh.best_cnt = 0; sh.cur_buf = 0; sh.best_buf = 0;
    }
    const float *S = a.src + (size_t)p * a.Nmax * 3;
    const float *Gt = a.tgt + (size_t)p * a.Mmax * 3;
    const int32_t *co = a.corres + (size_t)p * a.Kmax * 2;
    const int32_t *ord = a.order ? a.order + (size_t)p * a.Nmax : nullptr;
    GridT<uint16_t> gl{};
    GridView gg{};
    if (ok) {
        if constexpr (kLds) gl = grid_to_lds(a.grid, p, m, dsm + ((sizeof(Shared) + 15) & ~size_t(15)));
        else gg = a.grid.view(p);
    }
    __syncthreads();
    unsigned long long tm_hyp = 0, tm_val = 0, tm0 = 0, tm_a = 0;
    const bool tmg = a.timing != nullptr && tid == 0;
    if (tmg) tm0 = tm_a = __builtin_readcyclecounter();
    const double scale = fx_scale(a.thr);
    while (ok) {
        const int base = sh.base;
        const int lim = min(a.max_iter, sh.est_k);
        if (base >= lim) break;  // uniform
        const int itr = base + tid;
        double T[12];
        const bool pass = itr < lim && make_hypothesis<RN>(a, p, K, pid, itr, T);
        // stable compaction in iteration order
        const unsigned long long bal = __ballot(pass);
        const int below = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) sh.wcnt[wid] = __popcll(bal);
        __syncthreads();
        int woff = 0, total = 0;
        for (int w = 0; w < kWaves; ++w) {
            const int c = sh.wcnt[w];
            woff += (w < wid) ? c : 0;
            total += c;
        }
        const int pos = woff + below;
        if (pass && pos < kCap) {
            for (int k = 0; k < 12; ++k) sh.listT[pos][k] = T[k];
            sh.listItr[pos] = itr;
        }
        __syncthreads();
        if (tmg) { const unsigned long long t = __builtin_readcyclecounter(); tm_hyp += t - tm_a; tm_a = t; }
        const int nlist = min(total, kCap);
        const int next_base = total > kCap ? sh.listItr[kCap - 1] + 1 : base + kThreads;
        for (int e = 0; e < nlist; ++e) {
            const int itr_e = sh.listItr[e];
            if (itr_e >= sh.est_k) break;  // uniform: LDS value after a barrier
            const double *Te = sh.listT[e];
            unsigned long long acc = 0;
            int cnt = 0, cin = 0;
            // waves take 64-query chunks (spatial order) from an LDS counter:
            // dense and sparse regions cost different time, a static split
            // left waves idle at the barrier
            const int nch = (n + 63) >> 6;
            // a hypothesis with more than n - best_cnt misses cannot reach the
            // best fitness (not even tie it): Open3D's rule can never accept
            // it, so its sweep stops there (exact; no effect on T, fitness,
            // rmse or est_k)
            const int lim_miss = sh.best_cnt > 0 ? n - sh.best_cnt : 0x7fffffff;
            int32_t *cbuf = a.cand + ((size_t)p * 2 + sh.cur_buf) * a.Nmax;
            for (;;) {
                int c = 0;
                if (lane == 0) c = atomicAdd(&sh.chunk, 1);
                c = __shfl(c, 0, 64);
                if (c >= nch) break;
                const int k = (c << 6) + lane;
                int j = 0;
                if (k < n) {
                    const int i = ord ? ord[k] : k;
                    double px, py, pz, d2;
                    xform12(Te, (double)S[3 * i], (double)S[3 * i + 1], (double)S[3 * i + 2], px, py, pz);
                    if constexpr (kLds) j = grid_query(gl, a.d, a.thr, px, py, pz, d2);
                    else j = grid_query(gg, a.d, a.thr, px, py, pz, d2);
                    if (j >= 0) { ++cnt; acc += (unsigned long long)(d2 * scale); }
                    cbuf[i] = j;
                }
                const int miss = __popcll(__ballot(k < n && j < 0));
                int tot = 0;
                if (lane == 0) tot = atomicAdd(&sh.misses, miss) + miss;
                tot = __shfl(tot, 0, 64);
                if (tot > lim_miss) break;
            }
            const bool hopeless = __atomic_load_n(&sh.misses, __ATOMIC_RELAXED) > lim_miss;
            if (!hopeless)
                for (int k = tid; k < K; k += kThreads) {
                    const int si = co[2 * k], ti = co[2 * k + 1];
                    double px, py, pz;
                    xform12(Te, (double)S[3 * si], (double)S[3 * si + 1], (double)S[3 * si + 2], px, py, pz);
                    if (dist2(px, py, pz, (double)Gt[3 * ti], (double)Gt[3 * ti + 1], (double)Gt[3 * ti + 2]) < a.dd)
                        ++cin;
                }
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
                acc += __shfl_xor(acc, o, 64);
                cnt += __shfl_xor(cnt, o, 64);
                cin += __shfl_xor(cin, o, 64);
            }
            if (lane == 0) { sh.racc[wid] = acc; sh.rcnt[wid] = cnt; sh.rcin[wid] = cin; }
            __syncthreads();
            if (tid == 0) {
                unsigned long long A = 0;
                int C = 0, CI = 0;
                for (int w = 0; w < kWaves; ++w) { A += sh.racc[w]; C += sh.rcnt[w]; CI += sh.rcin[w]; }
                double fit = 0.0, rmse = 0.0;
                if (C > 0) {
                    fit = (double)C / (double)n;
                    rmse = __builtin_sqrt(((double)A / scale) / (double)C);
                }
                const bool cut = sh.misses > lim_miss;  // sweep stopped early: cannot win
                sh.validated += 1;
                sh.chunk = 0;  // next sweep (published by the barrier below)
                sh.misses = 0;
                if (!cut && (fit > sh.best_fit || (fit == sh.best_fit && rmse < sh.best_rmse))) {
                    sh.best_cnt = C;
                    sh.best_fit = fit;
                    sh.best_rmse = rmse;
                    sh.best_itr = itr_e;
                    sh.last_upd = itr_e;
                    sh.best_buf = sh.cur_buf;  // its correspondences stay; the next sweep
                    sh.cur_buf ^= 1;           // writes the other buffer
                    for (int k = 0; k < 12; ++k) sh.bestT[k] = Te[k];
                    const double kd = est_k_bound((double)CI / (double)K, RN, a.conf);
                    if (kd < (double)sh.est_k) sh.est_k = (int)__builtin_ceil(kd);
                }
            }
            __syncthreads();
        }
        if (tid == 0) sh.base = next_base;
        __syncthreads();
        if (tmg) { const unsigned long long t = __builtin_readcyclecounter(); tm_val += t - tm_a; tm_a = t; }
    }
    // loop exit iteration of the sequential algorithm: first itr >= est_k after the
    // last bound update (or max_iter)
    const int iters = ok ? min(a.max_iter, max(sh.last_upd + 1, sh.est_k)) : 0;
    const bool found = ok && sh.best_itr >= 0;
    // correspondence set of the best transformation: the targets its validation
    // sweep found (a sweep that became the best ran to completion, and the same
    // grid_query on the same transform gives the same answer); the inlier mask is
    // assembled with atomicOr on words zeroed first
    if (a.mask)
        for (int w = tid; w < a.words; w += kThreads) a.mask[(size_t)p * a.words + w] = 0u;
    __syncthreads();
    int cnt = 0;
    const int32_t *bbuf = a.cand + ((size_t)p * 2 + sh.best_buf) * a.Nmax;
    for (int i = tid; i < a.Nmax; i += kThreads) {
        const int j = (found && i < n) ? bbuf[i] : -1;
        if (a.corr_tgt) a.corr_tgt[(size_t)p * a.Nmax + i] = j;
        cnt += (j >= 0);
        if (a.mask && j >= 0) atomicOr(a.mask + (size_t)p * a.words + (i >> 5), 1u << (i & 31));
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if (lane == 0) sh.rcnt[wid] = cnt;
    __syncthreads();
    if (tid == 0) {
        int C = 0;
        for (int w = 0; w < kWaves; ++w) C += sh.rcnt[w];
        double *Tp = a.T_out + (size_t)p * 16;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) Tp[4 * r + c] = sh.bestT[4 * r + c];
        Tp[12] = 0.0; Tp[13] = 0.0; Tp[14] = 0.0; Tp[15] = 1.0;
        a.fit_out[2 * p] = sh.best_fit;
        a.fit_out[2 * p + 1] = sh.best_rmse;
        int32_t *st = a.stats + (size_t)p * 5;
        st[0] = iters;
        st[1] = ok ? sh.validated : 0;
        st[2] = ok ? sh.best_itr : -1;
        st[3] = ok ? (found ? 1 : 0) : -1;
        st[4] = C;
        if (a.timing) {
            unsigned long long *tt = a.timing + (size_t)p * 6;
            const unsigned long long t = __builtin_readcyclecounter();
            tt[0] = tm_hyp; tt[1] = tm_val; tt[2] = t - tm_a; tt[3] = t - tm0;
            tt[4] = (unsigned long long)sh.validated; tt[5] = (unsigned long long)sh.base;
        }
    }
}

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
    a.T_out = T_out; a.fit_out = fit_out; a.stats = stats; a.corr_tgt = corr_tgt; a.mask = mask;
    a.words = (Nmax + 31) / 32;
    a.timing = nullptr;
    a.order = nullptr;
    a.cand = (int32_t *)workspace(21, sizeof(int32_t) * 2 * (size_t)P * (size_t)(Nmax > 0 ? Nmax : 1));
    PCR_REQUIRE(a.cand, PCR_ERR_NOMEM, "ransac: %s", pcr_last_error());
    const bool want_timing = getenv("PCR_RANSAC_TIMING") != nullptr;
    if (want_timing) {
        a.timing = (unsigned long long *)workspace(12, sizeof(unsigned long long) * 6 * (size_t)P);
        PCR_REQUIRE(a.timing, PCR_ERR_NOMEM, "ransac timing: %s", pcr_last_error());
        PCR_HIP_CHECK(hipMemsetAsync(a.timing, 0, sizeof(unsigned long long) * 6 * (size_t)P, s));
    }
    a.grid = GridBatch{};
    a.grid.S = 1;
    a.grid.cell = 1.0;
    if (a.d > 0.0 && Mmax > 0) {
        int rc = build_grids(tgt, n_tgt, P, Mmax, a.d, s, 4, a.grid);
        if (rc != PCR_OK) return rc;
        if (Nmax > 0) {
            rc = spatial_order(src, n_src, P, Nmax, a.grid.cell, s, 13, &a.order);
            if (rc != PCR_OK) return rc;
        }
    }
    const size_t hdr = (sizeof(Shared) + 15) & ~size_t(15);
    const size_t budget = 160 * 1024 - hdr;
    const size_t gbytes = (a.d > 0.0 && Mmax > 0) ? grid_lds_bytes(Mmax, a.grid.S, budget) : 0;
    const bool lds = gbytes > 0;
    const size_t sm = lds ? hdr + gbytes : hdr;
    const void *fn = nullptr;
    switch (a.rn * 2 + (lds ? 1 : 0)) {
#define PCR_RCASE(N)                                                             \
    case 2 * N: fn = (const void *)ransac_pair_kernel<false, N>; break;          \
    case 2 * N + 1: fn = (const void *)ransac_pair_kernel<true, N>; break;
        PCR_RCASE(3) PCR_RCASE(4) PCR_RCASE(5) PCR_RCASE(6) PCR_RCASE(7) PCR_RCASE(8)
#undef PCR_RCASE
        default: set_error("ransac: bad ransac_n"); return PCR_ERR_ARG;
    }
    PCR_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm));
    prof_begin(s, kProfRansacValidate);
    {
        void *args[] = {&a};
        PCR_HIP_CHECK(hipLaunchKernel(fn, dim3(P), dim3(kThreads), args, sm, s));
    }
    PCR_LAUNCH_CHECK();
    prof_end(s, kProfRansacValidate);
    if (want_timing) {  // debug: phase split in shader clocks (s_memtime), to stderr
        std::vector<unsigned long long> h(6 * (size_t)P);
        PCR_HIP_CHECK(hipMemcpyAsync(h.data(), a.timing, h.size() * 8, hipMemcpyDeviceToHost, s));
        PCR_HIP_CHECK(hipStreamSynchronize(s));
        double m[6] = {0, 0, 0, 0, 0, 0}, mx = 0;
        for (int p = 0; p < P; ++p) {
            for (int k = 0; k < 6; ++k) m[k] += (double)h[6 * p + k] / P;
            mx = std::max(mx, (double)h[6 * p + 3]);
        }
        fprintf(stderr, "ransac timing (clocks, mean over %d pairs): hyp %.0f val %.0f final %.0f "
                "total %.0f (max %.0f) validated %.1f last_base %.0f\n", P, m[0], m[1], m[2], m[3],
                mx, m[4], m[5]);
    }
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
    PCR_REQUIRE(P <= 2147483647 / 2, PCR_ERR_ARG, "ransac: P too large");
    return pcr::ransac_impl(src_xyz, tgt_xyz, P, Nmax, Mmax, n_src, n_tgt, corres, n_corres, Kmax,
                            pair_ids, params, T, fitness_rmse, stats, corr_tgt, inlier_mask,
                            pcr::as_stream(stream));
}
