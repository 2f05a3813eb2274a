// a6/a7: batched RANSAC hypothesize-and-verify over P cloud pairs.
//
// Reference: Open3D 0.13 RegistrationRANSACBasedOnCorrespondence as driven by
// registration_ransac_based_on_feature_matching (DataPreparation/RANSAC.py:43-52,
// dip/demo.py:43-52, c2p-net/ngenet/utils/o3d.py:174-180).  Contract: the
// SEQUENTIAL loop of oracle_ransac (pcr_oracle.c) on the Philox hypothesis stream
// keyed by (seed, pair_id, itr).
//
// MI355X design, in rounds of hypotheses (round 1: iterations [0, 1024), then
// 4096 at a time while some pair's bound est_k still lies beyond the round):
//  * ransac_hyp_kernel (256-thread workgroups, one thread per hypothesis, all
//    pairs in one launch): Philox sample, Umeyama by Horn's 4x4 Jacobi in f64,
//    edge-length and distance checkers; the pass bits (one ballot word per 64
//    iterations) and the passing transforms go to HBM.  The Jacobi state needs
//    ~440 VGPRs: a kernel of its own runs it at one wave per SIMD without
//    spilling (inside the 1024-thread verification kernel it spilled ~320 VGPRs
//    to scratch);
//  * ransac_val_kernel (1024 threads, the pair's target hash grid copied to
//    LDS): walks the pass bits in iteration order and validates each passing
//    hypothesis below the live bound est_k -- every source point transformed
//    and queried (64-query chunks in spatial order taken from a counter),
//    inlier count + exact fixed-point error sum + inlier ratio over the
//    correspondences -- then applies Open3D's update rule and
//    est_k = min(est_k, ceil(log(1-conf)/log(1-w^n))).  The result is exactly
//    the sequential one whatever the round boundaries.  With fewer pairs than
//    CUs a pair's sweeps are split over G workgroups (cooperative launch, coop.h)
//    that add integer partials and take the same decision;
//  * the pair's correspondence set / inlier mask come from the best
//    hypothesis' own sweep (double-buffered target indices), written by the
//    round in which the pair finishes.
#include "pcr_internal.h"
#include "coop.h"
#include "geom.h"
#include "grid.h"
#include <algorithm>
#include <vector>

namespace pcr {
namespace {

constexpr int kMaxRansacN = 8;
constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;
constexpr int kHypThreads = 256;
constexpr int kRound0 = 1024;   // hypotheses of the first round
constexpr int kRoundN = 4096;   // hypotheses of every later round

// per-pair state carried across rounds (HBM)
struct RState {
    double bestT[12];
    double best_fit, best_rmse;
    int est_k, best_itr, validated, last_upd;
    int best_cnt;   // inlier count of the best hypothesis (0: none yet)
    int cur_buf, best_buf;  // cand buffer of the running sweep / of the best hypothesis
    int active;     // 1 while hypotheses remain below min(max_iter, est_k)
};

// integer partials of one split sweep (G > 1), per pair and parity
struct SweepAcc {
    unsigned long long acc;
    int cnt, cin, misses, chunk;
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
    double *T_out, *fit_out;
    int32_t *stats, *corr_tgt;
    uint32_t *mask;
    int words;
    const int32_t *order;   // (P, Nmax) spatial order of the source points, or null
    int32_t *cand;          // (P, 2, Nmax): target per source point, best / current sweep
    RState *state;          // (P)
    double *hypT;           // (P, hcap, 12) passing transforms of the round
    unsigned long long *hypbits;  // (P, hcap / 64) pass bits of the round
    int hcap;               // hypotheses per round slot (multiple of 256)
    int b0, b1;             // iterations of this round
    int G;                  // workgroups per pair (val kernel)
    SweepAcc *sacc;         // (P, 2) when G > 1
    unsigned *bar;          // (P, 2) when G > 1
    int *active_count;      // pairs still active after the round
};

__device__ __forceinline__ int cnt_of(const int32_t *n, int p, int mx) {
    return n ? min(max(n[p], 0), mx) : mx;
}

__device__ __forceinline__ bool pair_ok(const RArgs &a, int p, int RN) {
    const int n = cnt_of(a.n_src, p, a.Nmax), m = cnt_of(a.n_tgt, p, a.Mmax);
    const int K = a.n_corres ? min(max(a.n_corres[p], 0), a.Kmax) : a.Kmax;
    return K >= RN && a.d > 0.0 && n > 0 && m > 0;
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

// grid (ceil(span / 256), P): thread = iteration b0 + x*256 + tid of pair y
template <int RN>
__global__ __launch_bounds__(kHypThreads) void ransac_hyp_kernel(RArgs a) {
    const int p = blockIdx.y;
    const int off = blockIdx.x * kHypThreads + threadIdx.x;
    const int itr = a.b0 + off;
    bool live = off < a.hcap && itr < a.b1 && pair_ok(a, p, RN);
    int lim = a.max_iter;
    if (live && a.b0 > 0) {   // later rounds: only pairs still running, below their bound
        const RState &st = a.state[p];
        live = st.active != 0;
        lim = min(lim, st.est_k);
    }
    live = live && itr < lim;
    double T[12];
    bool pass = false;
    if (live) {
        const int K = a.n_corres ? min(max(a.n_corres[p], 0), a.Kmax) : a.Kmax;
        const uint32_t pid = a.pair_ids ? a.pair_ids[p] : (uint32_t)p;
        pass = make_hypothesis<RN>(a, p, K, pid, itr, T);
    }
    const unsigned long long bal = __ballot(pass);
    if (off < a.hcap && (threadIdx.x & 63) == 0)
        a.hypbits[(size_t)p * (a.hcap / 64) + (off >> 6)] = bal;
    if (pass) {
        double *o = a.hypT + ((size_t)p * a.hcap + off) * 12;
#pragma unroll
        for (int k = 0; k < 12; ++k) o[k] = T[k];
    }
}

struct Shared {  // LDS header (the grid copy follows)
    RState st;
    double Te[12];
    unsigned long long racc[kWaves];
    int rcnt[kWaves], rcin[kWaves];
    int chunk;     // next 64-query chunk of the current sweep (G = 1)
    int misses;    // source points without a correspondence so far in this sweep (G = 1)
    int nsweep;    // sweeps done in this launch (parity of the split accumulators)
    int done;
};

// one WG per pair (G = 1) or G WGs per pair (cooperative launch): blockIdx = p*G + g
template <bool kLds, int RN>
__global__ __launch_bounds__(kThreads) void ransac_val_kernel(RArgs a) {
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    Shared &sh = *reinterpret_cast<Shared *>(dsm);
    const int G = a.G;
    const int p = blockIdx.x / G, g = blockIdx.x - p * G;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int n = cnt_of(a.n_src, p, a.Nmax), m = cnt_of(a.n_tgt, p, a.Mmax);
    const int K = a.n_corres ? min(max(a.n_corres[p], 0), a.Kmax) : a.Kmax;
    const bool ok = pair_ok(a, p, RN);
    if (tid == 0) {
        if (a.b0 == 0) {
            RState &s = sh.st;
            for (int k = 0; k < 12; ++k) s.bestT[k] = (k % 5 == 0) ? 1.0 : 0.0;
            s.best_fit = 0.0; s.best_rmse = 0.0;
            s.est_k = a.max_iter; s.best_itr = -1; s.validated = 0; s.last_upd = -1;
            s.best_cnt = 0; s.cur_buf = 0; s.best_buf = 0; s.active = ok ? 1 : 0;
        } else {
            sh.st = a.state[p];
        }
        sh.chunk = 0; sh.misses = 0; sh.nsweep = 0; sh.done = 0;
    }
    __syncthreads();
    const bool was_active = sh.st.active != 0 || (a.b0 == 0);  // round 0 finishes invalid pairs
    if (!was_active) return;  // uniform over the pair's G workgroups
    const float *S = a.src + (size_t)p * a.Nmax * 3;
    const float *Gt = a.tgt + (size_t)p * a.Mmax * 3;
    const int32_t *co = a.corres + (size_t)p * a.Kmax * 2;
    const int32_t *ord = a.order ? a.order + (size_t)p * a.Nmax : nullptr;
    GridT<uint16_t> gl{};
    GridView gg{};
    if (ok && sh.st.active) {
        if constexpr (kLds) gl = grid_to_lds(a.grid, p, m, dsm + ((sizeof(Shared) + 15) & ~size_t(15)));
        else gg = a.grid.view(p);
    }
    __syncthreads();
    const double scale = fx_scale(a.thr);
    const int nch = (n + 63) >> 6;
    const int hw = a.hcap / 64;
    const unsigned long long *bits = a.hypbits + (size_t)p * hw;
    const int span = min(a.b1, a.max_iter) - a.b0;
    bool stop = !(ok && sh.st.active);
    for (int w = 0; !stop && w * 64 < span; ++w) {
        unsigned long long word = bits[w];
        while (word) {
            const int e = __builtin_ctzll(word);
            word &= word - 1ull;
            const int itr_e = a.b0 + w * 64 + e;
            if (itr_e >= sh.st.est_k) { stop = true; break; }  // uniform: LDS value after a barrier
            if (tid < 12) sh.Te[tid] = a.hypT[((size_t)p * a.hcap + (itr_e - a.b0)) * 12 + tid];
            __syncthreads();
            double Te[12];
#pragma unroll
            for (int k = 0; k < 12; ++k) Te[k] = sh.Te[k];
            SweepAcc *sa = (G > 1) ? a.sacc + (size_t)p * 2 + (sh.nsweep & 1) : nullptr;
            unsigned long long acc = 0;
            int cnt = 0, cin = 0;
            // a hypothesis with more than n - best_cnt misses cannot reach the
            // best fitness (not even tie it): Open3D's rule can never accept
            // it, so its sweep stops there (exact; no effect on T, fitness,
            // rmse or est_k)
            const int lim_miss = sh.st.best_cnt > 0 ? n - sh.st.best_cnt : 0x7fffffff;
            int32_t *cbuf = a.cand + ((size_t)p * 2 + sh.st.cur_buf) * a.Nmax;
            for (;;) {
                int c = 0;
                if (lane == 0) c = (G > 1) ? coop_fetch_add(&sa->chunk, 1) : atomicAdd(&sh.chunk, 1);
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
                if (lane == 0)
                    tot = ((G > 1) ? coop_fetch_add(&sa->misses, miss) : atomicAdd(&sh.misses, miss)) + miss;
                tot = __shfl(tot, 0, 64);
                if (tot > lim_miss) break;
            }
            const int seen = (G > 1) ? coop_load(&sa->misses) : __atomic_load_n(&sh.misses, __ATOMIC_RELAXED);
            // (not unrolled: an unrolled copy of this loop spilled ~260 VGPRs)
            if (seen <= lim_miss)  // not (yet) hopeless: this WG's share of the inlier ratio
#pragma unroll 1
                for (int q = g * kThreads + tid; q < K; q += G * kThreads) {
                    const int si = co[2 * q], ti = co[2 * q + 1];
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
            unsigned long long A = 0;
            int C = 0, CI = 0, MS = 0;
            if (tid == 0) {
                for (int ww = 0; ww < kWaves; ++ww) { A += sh.racc[ww]; C += sh.rcnt[ww]; CI += sh.rcin[ww]; }
                if (G > 1) {
                    __hip_atomic_fetch_add(&sa->acc, A, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    coop_fetch_add(&sa->cnt, C);
                    coop_fetch_add(&sa->cin, CI);
                } else {
                    MS = sh.misses;
                }
            }
            if (G > 1) {
                pair_barrier(a.bar + 2 * (size_t)p, G);
                if (tid == 0) {
                    A = __hip_atomic_load(&sa->acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    C = coop_load(&sa->cnt);
                    CI = coop_load(&sa->cin);
                    MS = coop_load(&sa->misses);
                }
            }
            if (tid == 0) {
                RState &s = sh.st;
                double fit = 0.0, rmse = 0.0;
                if (C > 0) {
                    fit = (double)C / (double)n;
                    rmse = __builtin_sqrt(((double)A / scale) / (double)C);
                }
                const bool cut = MS > lim_miss;  // sweep stopped early: cannot win
                s.validated += 1;
                sh.chunk = 0;  // next sweep (published by the barrier below)
                sh.misses = 0;
                sh.nsweep += 1;
                if (!cut && (fit > s.best_fit || (fit == s.best_fit && rmse < s.best_rmse))) {
                    s.best_cnt = C;
                    s.best_fit = fit;
                    s.best_rmse = rmse;
                    s.best_itr = itr_e;
                    s.last_upd = itr_e;
                    s.best_buf = s.cur_buf;  // its correspondences stay; the next sweep
                    s.cur_buf ^= 1;          // writes the other buffer
                    for (int k = 0; k < 12; ++k) s.bestT[k] = Te[k];
                    const double kd = est_k_bound((double)CI / (double)K, RN, a.conf);
                    if (kd < (double)s.est_k) s.est_k = (int)__builtin_ceil(kd);
                }
            }
            if (G > 1) {
                // the OTHER parity was last read before the previous sweep's second
                // barrier: WG 0 clears it for the next sweep, and this barrier
                // publishes both the clear and the decision
                if (g == 0 && tid == 0) {
                    SweepAcc *nx = a.sacc + (size_t)p * 2 + (sh.nsweep & 1);
                    nx->acc = 0ull; nx->cnt = 0; nx->cin = 0; nx->misses = 0; nx->chunk = 0;
                }
                pair_barrier(a.bar + 2 * (size_t)p, G);
            } else {
                __syncthreads();
            }
        }
    }
    // round end: the pair is finished once the next iteration would be at or
    // beyond min(max_iter, est_k)
    if (tid == 0) {
        RState &s = sh.st;
        const bool fin = !ok || a.b1 >= min(a.max_iter, s.est_k);
        s.active = fin ? 0 : 1;
        sh.done = fin ? 1 : 0;
        if (g == 0) {
            a.state[p] = s;
            if (!fin) atomicAdd(a.active_count, 1);
        }
    }
    __syncthreads();
    if (!sh.done) return;
    // outputs.  Loop exit iteration of the sequential algorithm: first itr >=
    // est_k after the last bound update (or max_iter)
    const RState &s = sh.st;
    const int iters = ok ? min(a.max_iter, max(s.last_upd + 1, s.est_k)) : 0;
    const bool found = ok && s.best_itr >= 0;
    // correspondence set of the best transformation: the targets its validation
    // sweep found (a sweep that became the best ran to completion)
    const int32_t *bbuf = a.cand + ((size_t)p * 2 + s.best_buf) * a.Nmax;
    if (a.corr_tgt)
        for (int i = g * kThreads + tid; i < a.Nmax; i += G * kThreads)
            a.corr_tgt[(size_t)p * a.Nmax + i] = (found && i < n) ? bbuf[i] : -1;
    if (a.mask)
        for (int w = g * kThreads + tid; w < a.words; w += G * kThreads) {
            uint32_t bitsw = 0u;
            if (found)
                for (int b = 0; b < 32; ++b) {
                    const int i = 32 * w + b;
                    if (i < n && bbuf[i] >= 0) bitsw |= 1u << b;
                }
            a.mask[(size_t)p * a.words + w] = bitsw;
        }
    if (g == 0 && tid == 0) {
        double *Tp = a.T_out + (size_t)p * 16;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) Tp[4 * r + c] = s.bestT[4 * r + c];
        Tp[12] = 0.0; Tp[13] = 0.0; Tp[14] = 0.0; Tp[15] = 1.0;
        a.fit_out[2 * p] = s.best_fit;
        a.fit_out[2 * p + 1] = s.best_rmse;
        int32_t *st = a.stats + (size_t)p * 5;
        st[0] = iters;
        st[1] = ok ? s.validated : 0;
        st[2] = ok ? s.best_itr : -1;
        st[3] = ok ? (found ? 1 : 0) : -1;
        st[4] = found ? s.best_cnt : 0;
    }
}

template <int RN>
const void *hyp_fn() { return (const void *)ransac_hyp_kernel<RN>; }

template <int RN>
const void *val_fn(bool lds) {
    return lds ? (const void *)ransac_val_kernel<true, RN> : (const void *)ransac_val_kernel<false, RN>;
}

}  // namespace

int ransac_impl(const float *src, const float *tgt, int P, int Nmax, int Mmax,
                const int32_t *n_src, const int32_t *n_tgt, const int32_t *corres,
                const int32_t *n_corres, int Kmax, const uint32_t *pair_ids,
                const pcr_ransac_params *prm, double *T_out, double *fit_out, int32_t *stats,
                int32_t *corr_tgt, uint32_t *mask, hipStream_t s) {
    PCR_REQUIRE(prm->ransac_n >= 3 && prm->ransac_n <= kMaxRansacN, PCR_ERR_ARG,
                "ransac: ransac_n=%d unsupported (3..%d)", prm->ransac_n, kMaxRansacN);
    PCR_REQUIRE(prm->max_iteration >= 0, PCR_ERR_ARG, "ransac: negative max_iteration");
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
    a.order = nullptr;
    const size_t nm = (size_t)(Nmax > 0 ? Nmax : 1);
    a.cand = (int32_t *)workspace(21, sizeof(int32_t) * 2 * (size_t)P * nm);
    PCR_REQUIRE(a.cand, PCR_ERR_NOMEM, "ransac: %s", pcr_last_error());
    a.hcap = kRoundN;  // >= kRound0, multiple of 256
    a.state = (RState *)workspace(22, sizeof(RState) * (size_t)P);
    a.hypT = (double *)workspace(23, sizeof(double) * 12 * (size_t)P * a.hcap);
    a.hypbits = (unsigned long long *)workspace(24, sizeof(unsigned long long) * (size_t)P * (a.hcap / 64));
    char *misc = (char *)workspace(25, (sizeof(SweepAcc) * 2 + sizeof(unsigned) * 2) * (size_t)P + 256);
    PCR_REQUIRE(a.state && a.hypT && a.hypbits && misc, PCR_ERR_NOMEM, "ransac: %s", pcr_last_error());
    a.active_count = (int *)misc;
    a.sacc = (SweepAcc *)(misc + 256);
    a.bar = (unsigned *)(misc + 256 + sizeof(SweepAcc) * 2 * (size_t)P);
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
    const void *hfn = nullptr, *vfn = nullptr;
    switch (a.rn) {
#define PCR_RCASE(N)                  \
    case N:                           \
        hfn = hyp_fn<N>();            \
        vfn = val_fn<N>(lds);         \
        break;
        PCR_RCASE(3) PCR_RCASE(4) PCR_RCASE(5) PCR_RCASE(6) PCR_RCASE(7) PCR_RCASE(8)
#undef PCR_RCASE
        default: set_error("ransac: bad ransac_n"); return PCR_ERR_ARG;
    }
    PCR_HIP_CHECK(hipFuncSetAttribute(vfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm));
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, vfn, kThreads, sm) != hipSuccess) {
        (void)hipGetLastError();
        per_cu = 0;
    }
    a.G = coop_groups(P, per_cu);
    prof_begin(s, kProfRansacValidate);
    // rounds: [0, kRound0), then kRoundN at a time while a pair is still running
    a.b0 = 0;
    a.b1 = std::min(a.max_iter, kRound0);
    for (;;) {
        PCR_HIP_CHECK(hipMemsetAsync(a.active_count, 0, sizeof(int), s));
        const int span = a.b1 - a.b0;
        if (span > 0) {
            void *args[] = {&a};
            PCR_HIP_CHECK(hipLaunchKernel(hfn, dim3((span + kHypThreads - 1) / kHypThreads, P),
                                          dim3(kHypThreads), args, 0, s));
            PCR_LAUNCH_CHECK();
        }
        {
            if (a.G > 1)  // split-sweep accumulators (both parities) and barriers
                PCR_HIP_CHECK(hipMemsetAsync(a.sacc, 0, (sizeof(SweepAcc) * 2 + sizeof(unsigned) * 2) * (size_t)P, s));
            void *args[] = {&a};
            PCR_HIP_CHECK(coop_launch(vfn, P, a.G, kThreads, args, sm, s));
            PCR_LAUNCH_CHECK();
        }
        if (a.b1 >= a.max_iter) break;
        int active = 0;
        PCR_HIP_CHECK(hipMemcpyAsync(&active, a.active_count, sizeof(int), hipMemcpyDeviceToHost, s));
        PCR_HIP_CHECK(hipStreamSynchronize(s));
        if (active == 0) break;
        a.b0 = a.b1;
        a.b1 = std::min(a.max_iter, a.b0 + kRoundN);
    }
    prof_end(s, kProfRansacValidate);
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
    PCR_REQUIRE(P <= 65535, PCR_ERR_ARG, "ransac: P=%d > 65535 pairs per call", P);
    return pcr::ransac_impl(src_xyz, tgt_xyz, P, Nmax, Mmax, n_src, n_tgt, corres, n_corres, Kmax,
                            pair_ids, params, T, fitness_rmse, stats, corr_tgt, inlier_mask,
                            pcr::as_stream(stream));
}
