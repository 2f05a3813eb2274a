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
//    spilling;
//  * ransac_task_kernel: the round's tasks = the passing hypotheses below the
//    pair's live bound, in iteration order;
//  * ransac_sweep_kernel (persistent 1024-thread workgroups, one per CU, the
//    task's target hash grid copied to LDS): validates the tasks of ALL pairs
//    speculatively and in parallel -- rank-major (every pair's first passing
//    hypothesis, then every pair's second, ...) from a global counter, so a
//    pair with many hypotheses no longer holds one CU for the whole launch
//    while the others idle.  A sweep transforms and queries every source point
//    (64-query chunks in spatial order), counts inliers, sums the exact
//    fixed-point error and the inlier ratio over the correspondences.  Results
//    are independent of each other; two exact shortcuts use the pair's already
//    finished tasks (cut bound, skip beyond est_k: see the kernel);
//  * ransac_replay_kernel (one workgroup per pair): Open3D's update rule and
//    est_k = min(est_k, ceil(log(1-conf)/log(1-w^n))) applied to the results in
//    iteration order, stopping at the first hypothesis at or beyond est_k --
//    exactly the sequential loop's decisions, `validated` count included.
//    The best hypothesis' targets come from its sweep's slot (or one more sweep
//    when it had none); outputs are written in the round the pair finishes.
#include "pcr_internal.h"
#include "geom.h"
#include "grid.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kRansacKW = 4;  // candidates per grid-walk step in the sweeps (2 / 4 / 6 / 8 measured, round 4)

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
    int fix;        // 1: bestbuf does not hold the best hypothesis' targets (no slot)
    int active;     // 1 while hypotheses remain below min(max_iter, est_k)
    int pad;
};

// one speculative validation: hypothesis `tasks[p][r]` swept over all source points
struct TaskRes {
    unsigned long long acc;  // fixed-point sum of the inliers' d2
    int cnt, cin;            // inliers, inlier correspondences
    int status;              // kPending / kDone / kCut / kSkipped
    int misses;              // split sweeps: misses of both halves so far
    int hdone;               // split sweeps: halves finished
    int pad;
};

// one part of a split sweep (the last part to finish combines them)
struct TaskPart {
    unsigned long long acc;
    int cnt, cin;
    int flag;  // kDone / kCut / kSkipped as this half saw it
    int lb;    // its final cut bound
};
constexpr int kPending = 0, kDone = 1, kCut = 2, kSkipped = 3;

// round-global counters (zeroed before every round)
struct RHeader {
    int task_ctr;      // next task of the persistent sweep kernel
    int maxtask;       // max tasks of one pair in this round
    int active_count;  // pairs still active after the round
    int bad;           // replay met a task it needed that was never swept (bug guard)
    int n_done, n_cut, n_skip, n_chunks;  // diagnostics (PCR_RANSAC_STATS=1 prints them)
};

static_assert(2 * sizeof(RHeader) / sizeof(int) <= 256, "ransac_hyp_kernel clears the headers with one thread per word");

struct RArgs {
    const float *src, *tgt;
    const int32_t *n_src, *n_tgt;
    const int32_t *corres, *n_corres;
    const uint32_t *pair_ids;
    int P, Nmax, Mmax, Kmax;
    double d, thr, dd, edge, dcheck, conf;
    int rn, max_iter;
    uint64_t seed;
    GridBatch grid;
    double *T_out, *fit_out;
    int32_t *stats, *corr_tgt;
    uint32_t *mask;
    int words;
    const int32_t *order;   // (P, Nmax) spatial order of the source points, or null
    const float *srcp;      // (P, Nmax, 3) the source points in that order, or null
    RState *state;          // (P)
    double *hypT;           // (P, hcap, 12) passing transforms of the round
    unsigned long long *hypbits;  // (P, hcap / 64) pass bits of the round
    int hcap;               // hypotheses per round slot (multiple of 256)
    int b0, b1;             // iterations of this round
    int *ntask;             // (P) tasks of the round per pair
    int *tasks;             // (P, hcap) their iterations, ascending
    TaskRes *res;           // (P, hcap)
    int32_t *slots;         // (P, nslots, Nmax) targets found by task r < nslots
    int nslots;
    int32_t *bestbuf;       // (P, Nmax) targets of the best hypothesis so far
    RHeader *hdr;
    int split;              // workgroups per task (1, 2, 4 or 8: more when the pairs are few)
    TaskPart *parts;        // (P, hcap, split) when split > 1
    const int *prev_active; // later rounds launched without a host decision: the previous
                            // round's active_count (0: every kernel of this round returns)
    int clear_hdr;          // ransac_hyp_kernel clears hdr[0..2) (the gated rounds' first launch)
};

__device__ __forceinline__ bool round_off(const RArgs &a) {
    return a.prev_active != nullptr && *a.prev_active == 0;
}

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

// grid (x, P): block x takes the 256-iteration chunks x, x + gridDim.x, ... of
// the round (a later round can span up to max_iter, but stops at the pair's
// bound); thread = iteration b0 + chunk*256 + tid of pair y
template <int RN>
__global__ __launch_bounds__(kHypThreads) void ransac_hyp_kernel(RArgs a) {
    if (round_off(a)) return;
    // device-gated rounds: the first round's first block clears both rounds'
    // headers (every later reader is a later launch on the stream)
    if (a.clear_hdr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 2 * sizeof(RHeader) / sizeof(int))
        reinterpret_cast<int *>(a.hdr)[threadIdx.x] = 0;
    const int p = blockIdx.y;
    int lim = min(a.b1, a.max_iter);
    if (a.b0 > 0) {   // later rounds: only pairs still running, below their bound
        const RState &st = a.state[p];
        if (!st.active) return;
        lim = min(lim, st.est_k);
    }
    const bool okp = pair_ok(a, p, RN);
    const int K = a.n_corres ? min(max(a.n_corres[p], 0), a.Kmax) : a.Kmax;
    const uint32_t pid = a.pair_ids ? a.pair_ids[p] : (uint32_t)p;
    for (int cx = blockIdx.x; a.b0 + cx * kHypThreads < lim; cx += gridDim.x) {
        const int off = cx * kHypThreads + threadIdx.x;
        const int itr = a.b0 + off;
        const bool live = okp && off < a.hcap && itr < lim;
        double T[12];
        bool pass = false;
        if (live) pass = make_hypothesis<RN>(a, p, K, pid, itr, T);
        const unsigned long long bal = __ballot(pass);
        if (off < a.hcap && (threadIdx.x & 63) == 0)
            a.hypbits[(size_t)p * (a.hcap / 64) + (off >> 6)] = bal;
        if (pass) {
            double *o = a.hypT + ((size_t)p * a.hcap + off) * 12;
#pragma unroll
            for (int k = 0; k < 12; ++k) o[k] = T[k];
        }
    }
}

struct Shared {  // LDS header (the grid copy follows)
    RState st;
    double Te[12];
    unsigned long long racc[kWaves];
    int rcnt[kWaves], rcin[kWaves];
    int chunk;     // next 64-query chunk of the running sweep
    int misses;    // source points without a correspondence so far in this sweep
    int task, lb, skip, gp;  // current task, its cut bound, skip flag, pair whose grid is loaded
    int best_r, done;
};

// One step of the sequential loop (Open3D's rule) for validated hypothesis
// `itr` with sweep result r; T (may be null) is copied when it becomes the best.
__device__ inline bool apply_result(RState &s, int itr, const TaskRes &r, const double *T, int n,
                                    int K, double scale, double conf, int RN) {
    const bool cut = r.status == kCut;  // its inliers were below the best's: cannot win
    double fit = 0.0, rmse = 0.0;
    if (!cut && r.cnt > 0) {
        fit = (double)r.cnt / (double)n;
        rmse = __builtin_sqrt(((double)r.acc / scale) / (double)r.cnt);
    }
    s.validated += 1;
    if (!cut && (fit > s.best_fit || (fit == s.best_fit && rmse < s.best_rmse))) {
        s.best_cnt = r.cnt;
        s.best_fit = fit;
        s.best_rmse = rmse;
        s.best_itr = itr;
        s.last_upd = itr;
        if (T)
            for (int k = 0; k < 12; ++k) s.bestT[k] = T[k];
        const double kd = est_k_bound((double)r.cin / (double)K, RN, conf);
        if (kd < (double)s.est_k) s.est_k = (int)__builtin_ceil(kd);
        return true;
    }
    return false;
}

// One workgroup sweeps every source point of pair p under Te: inliers, exact
// fixed-point error sum and (unless cut) the inlier correspondences, in
// 64-query chunks of the spatial order taken from an LDS counter.  Cut bound:
// sh.lb (set by the caller; 0 = none) -- the sweep stops once its misses exceed
// n - lb.  With prs (the pair's tasks of lower rank, npr of them) every wave
// polls their finished inlier counts every 4 chunks and raises the bound.
// cbuf (may be null): target per point, by position k in the sweep order
// (coalesced stores) when by_order, else by source index.
template <bool kLds, int RN, typename Grid>
__device__ TaskRes sweep_pair(const RArgs &a, Shared &sh, const Grid &gr, int p, int n, int K,
                              const double *Te, const TaskRes *prs, int npr, int32_t *cbuf,
                              bool by_order, int c_lo = 0, int c_hi = 0x7fffffff,
                              int *gmiss = nullptr, int h = 0, int nh = 1) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const float *S = a.src + (size_t)p * a.Nmax * 3;
    const float *Gt = a.tgt + (size_t)p * a.Mmax * 3;
    const int32_t *co = a.corres + (size_t)p * a.Kmax * 2;
    const int32_t *ord = a.order ? a.order + (size_t)p * a.Nmax : nullptr;
    const float *Sp = (a.srcp && ord) ? a.srcp + (size_t)p * a.Nmax * 3 : nullptr;
    const double scale = fx_scale(a.thr);
    const int nch = min((n + 63) >> 6, c_hi);
    unsigned long long acc = 0;
    int cnt = 0, cin = 0;
    int lb = sh.lb;
    for (int nc = 1;; ++nc) {
        int c = 0;
        if (lane == 0) c = c_lo + atomicAdd(&sh.chunk, 1);
        c = __shfl(c, 0, 64);
        if (c >= nch) break;
        const int k = (c << 6) + lane;
        int j = 0;
        if (k < n) {
            // the chunk's points: a contiguous run of the ordered copy, or gathered
            float sx, sy, sz;
            if (Sp) {
                sx = Sp[3 * k]; sy = Sp[3 * k + 1]; sz = Sp[3 * k + 2];
            } else {
                const int i = ord ? ord[k] : k;
                sx = S[3 * i]; sy = S[3 * i + 1]; sz = S[3 * i + 2];
            }
            double px, py, pz, d2;
            xform12(Te, (double)sx, (double)sy, (double)sz, px, py, pz);
            j = grid_query<Grid, false, kRansacKW>(gr, a.d, a.thr, px, py, pz, d2);
            if (j >= 0) { ++cnt; acc += (unsigned long long)(d2 * scale); }
            // written through (sc1): finish_task's release fence writes back the
            // XCD L2's dirty lines, and a sweep's targets are 32 KB of them
            if (cbuf) __hip_atomic_store(cbuf + (by_order ? k : (ord ? ord[k] : k)), j, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        }
        const int miss = __popcll(__ballot(k < n && j < 0));
        int tot = 0;
        if (lane == 0) {
            tot = atomicAdd(&sh.misses, miss) + miss;
            if (gmiss)  // split sweep: the task's total over both halves
                tot = __hip_atomic_fetch_add(gmiss, miss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + miss;
        }
        tot = __shfl(tot, 0, 64);
        if ((nc & 3) == 0 && npr > 0) {  // earlier tasks finished meanwhile: a higher bound
            int c2 = 0;
            if (lane < npr &&
                __hip_atomic_load(&prs[lane].status, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == kDone)
                c2 = prs[lane].cnt;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) c2 = max(c2, __shfl_xor(c2, o, 64));
            if (c2 > lb) {
                lb = c2;
                if (lane == 0) atomicMax(&sh.lb, lb);
            }
        }
        if (lb > 0 && tot > n - lb) break;
    }
    // every wave's misses and bound are in: one cut decision for all (a wave
    // that stopped saw misses above n - its bound >= n - the final bound)
    __syncthreads();
    const int msum = gmiss ? __hip_atomic_load(gmiss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : sh.misses;
    const bool cut = sh.lb > 0 && msum > n - sh.lb;
    // (not unrolled: an unrolled copy of this loop spilled ~260 VGPRs)
    if (!cut)  // the inlier ratio over the correspondences (est_k of a new best)
#pragma unroll 1
        for (int q = h * kThreads + tid; q < K; q += nh * kThreads) {
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
    if (tid == 0) atomicAdd(&a.hdr->n_chunks, min(sh.chunk, max(nch - c_lo, 0)));
    TaskRes r{};
    for (int w = 0; w < kWaves; ++w) { r.acc += sh.racc[w]; r.cnt += sh.rcnt[w]; r.cin += sh.rcin[w]; }
    r.status = cut ? kCut : kDone;
    __syncthreads();  // racc / chunk / misses are reused by the caller's next sweep
    if (tid == 0) { sh.chunk = 0; sh.misses = 0; }
    return r;
}

// Round setup, one wave per pair: the round-0 state, then the round's tasks =
// the passing hypotheses below min(b1, max_iter, est_k), in iteration order.
__global__ __launch_bounds__(64) void ransac_task_kernel(RArgs a, int RN) {
    if (round_off(a)) return;
    const int p = blockIdx.x, lane = threadIdx.x;
    RState *sp = a.state + p;
    if (a.b0 == 0 && lane == 0) {
        RState s;
        for (int k = 0; k < 12; ++k) s.bestT[k] = (k % 5 == 0) ? 1.0 : 0.0;
        s.best_fit = 0.0; s.best_rmse = 0.0;
        s.est_k = a.max_iter; s.best_itr = -1; s.validated = 0; s.last_upd = -1;
        s.best_cnt = 0; s.fix = 0; s.pad = 0;
        s.active = pair_ok(a, p, RN) ? 1 : 0;
        *sp = s;
    }
    __syncthreads();
    const RState &s = *sp;
    int nt = 0;
    if (s.active) {
        const int lim = min(min(a.b1, a.max_iter), s.est_k) - a.b0;
        const unsigned long long *bits = a.hypbits + (size_t)p * (a.hcap / 64);
        int *tk = a.tasks + (size_t)p * a.hcap;
        TaskRes *rs = a.res + (size_t)p * a.hcap;
        for (int w0 = 0; w0 * 64 < lim; w0 += 64) {
            const int w = w0 + lane;
            unsigned long long word = (w * 64 < lim) ? bits[w] : 0ull;
            if ((w + 1) * 64 > lim && w * 64 < lim) word &= (lim - w * 64 >= 64) ? ~0ull : ((1ull << (lim - w * 64)) - 1ull);
            const int c = __popcll(word);
            int pre = c;  // inclusive prefix over the lanes
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int v = __shfl_up(pre, o, 64);
                if (lane >= o) pre += v;
            }
            int at = nt + pre - c;
            while (word) {
                const int e = __builtin_ctzll(word);
                word &= word - 1ull;
                tk[at] = a.b0 + w * 64 + e;
                TaskRes z{};
                z.status = kPending;
                rs[at] = z;
                ++at;
            }
            nt += __shfl(pre, 63, 64);
        }
    }
    if (lane == 0) {
        a.ntask[p] = nt;
        if (nt > 0) atomicMax(&a.hdr->maxtask, nt);
    }
}

// Publish a sweep result (thread 0).  Unsplit: the status store is released
// after the fields.  Split: each part parks its partial; the part that finishes
// last adds them and publishes -- skipped if any part proved the task beyond
// est_k, cut if any part stopped or the summed misses exceed n - the largest
// bound (a stopped part saw misses above n - its bound), else done.
__device__ inline void finish_task(const RArgs &a, TaskRes *rt, int p, int r, int h, TaskRes out,
                                   int lb) {
    if (a.split > 1) {
        TaskPart *pp = a.parts + ((size_t)p * a.hcap + r) * a.split;
        pp[h].acc = out.acc;
        pp[h].cnt = out.cnt;
        pp[h].cin = out.cin;
        pp[h].flag = out.status;
        pp[h].lb = lb;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const int before = __hip_atomic_fetch_add(&rt->hdone, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (before != a.split - 1) return;  // another part publishes
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        out.acc = 0ull;
        out.cnt = 0;
        out.cin = 0;
        int lbm = 0;
        bool skipped = false, stopped = false;
        for (int q = 0; q < a.split; ++q) {
            const TaskPart pq = pp[q];
            out.acc += pq.acc;
            out.cnt += pq.cnt;
            out.cin += pq.cin;
            lbm = max(lbm, pq.lb);
            skipped = skipped || pq.flag == kSkipped;
            stopped = stopped || pq.flag == kCut;
        }
        const int n = cnt_of(a.n_src, p, a.Nmax);
        const int ms = __hip_atomic_load(&rt->misses, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (skipped) out.status = kSkipped;
        else if (stopped || (lbm > 0 && ms > n - lbm)) out.status = kCut;
        else out.status = kDone;
    }
    atomicAdd(out.status == kSkipped ? &a.hdr->n_skip : out.status == kCut ? &a.hdr->n_cut : &a.hdr->n_done, 1);
    rt->acc = out.acc;
    rt->cnt = out.cnt;
    rt->cin = out.cin;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_store(&rt->status, out.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Persistent sweep workgroups take tasks t = ((r * P + p) * split + part) from a
// global counter: every pair's first hypothesis (rank r = 0), then every
// pair's second, ...; with split > 1 a task's chunks are shared by `split`
// consecutive parts (finish_task combines them).  Each sweep is independent of
// the others; the sequential rule is applied afterwards
// (ransac_replay_kernel).  Two exact shortcuts from the
// tasks of the same pair that are already finished:
//  * cut bound: a hypothesis with more than n - c misses, c = the inliers of
//    any earlier finished hypothesis, is below the best at its turn (whose
//    inliers are >= c): it cannot be accepted, so its sweep stops there;
//  * skip: replaying the finished prefix of the pair's tasks gives an est_k
//    that can only fall further; a task at or beyond it is never validated.
template <bool kLds, int RN>
__global__ __launch_bounds__(kThreads) void ransac_sweep_kernel(RArgs a) {
    if (round_off(a)) return;
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    Shared &sh = *reinterpret_cast<Shared *>(dsm);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int maxtask = a.hdr->maxtask;
    const double scale = fx_scale(a.thr);
    if (tid == 0) { sh.chunk = 0; sh.misses = 0; sh.gp = -1; }
    for (;;) {
        __syncthreads();
        if (tid == 0) sh.task = atomicAdd(&a.hdr->task_ctr, 1);
        __syncthreads();
        const int t = sh.task;
        // t = (r * P + p) * split + h: the halves of a split task are taken together
        const int tq = t / a.split, h = t - tq * a.split;
        const int r = tq / a.P, p = tq - r * a.P;
        if (r >= maxtask) break;
        const int nt = a.ntask[p];
        if (r >= nt) continue;
        const int n = cnt_of(a.n_src, p, a.Nmax);
        const int K = a.n_corres ? min(max(a.n_corres[p], 0), a.Kmax) : a.Kmax;
        const int *tk = a.tasks + (size_t)p * a.hcap;
        TaskRes *rs = a.res + (size_t)p * a.hcap;
        const int itr = tk[r];
        if (wid == 0) {  // cut bound and skip test from the finished prefix
            RState s = a.state[p];
            int lb = s.best_cnt;
            bool replay = true, skip = false;
            for (int b = 0; b < r && replay && !skip; b += 64) {
                const int rr = b + lane;
                int st = kPending, c = 0, ci = 0, it = 0;
                unsigned long long ac = 0;
                if (rr < r) {
                    st = __hip_atomic_load(&rs[rr].status, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                    if (st == kDone || st == kCut) { c = rs[rr].cnt; ci = rs[rr].cin; ac = rs[rr].acc; }
                    it = tk[rr];
                    if (st == kDone) lb = max(lb, c);
                }
                const int m = min(64, r - b);
                for (int e = 0; e < m; ++e) {
                    const int ste = __shfl(st, e, 64), ite = __shfl(it, e, 64);
                    if (ste == kPending) { replay = false; break; }
                    if (ste == kSkipped || ite >= s.est_k) { skip = true; break; }
                    TaskRes tr;
                    tr.status = ste;
                    tr.cnt = __shfl(c, e, 64);
                    tr.cin = __shfl(ci, e, 64);
                    tr.acc = __shfl(ac, e, 64);
                    apply_result(s, ite, tr, nullptr, n, K, scale, a.conf, RN);
                }
            }
            if (!skip && itr >= s.est_k) skip = true;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) lb = max(lb, __shfl_xor(lb, o, 64));
            if (lane == 0) { sh.lb = lb; sh.skip = skip ? 1 : 0; }
        }
        if (tid < 12) sh.Te[tid] = a.hypT[((size_t)p * a.hcap + (itr - a.b0)) * 12 + tid];
        __syncthreads();
        if (sh.skip) {
            if (tid == 0) {
                TaskRes out{};
                out.status = kSkipped;
                finish_task(a, rs + r, p, r, h, out, 0);
            }
            continue;
        }
        char *glds = dsm + ((sizeof(Shared) + 15) & ~size_t(15));
        if (kLds && sh.gp != p) {  // this pair's grid into LDS (kept while the next task is the same pair)
            (void)grid_to_lds4(a.grid, p, cnt_of(a.n_tgt, p, a.Mmax), glds);
            if (tid == 0) sh.gp = p;
        }
        double Te[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) Te[k] = sh.Te[k];
        int32_t *cbuf = r < a.nslots ? a.slots + ((size_t)p * a.nslots + r) * a.Nmax : nullptr;
        const int nch = (n + 63) >> 6;
        const int c_lo = h * nch / a.split, c_hi = (h + 1) * nch / a.split;
        int *gm = a.split > 1 ? &rs[r].misses : nullptr;
        TaskRes out;
        if constexpr (kLds)
            out = sweep_pair<kLds, RN>(a, sh, grid_lds4_view(a.grid, glds), p, n, K, Te, rs, r, cbuf, true,
                                       c_lo, c_hi, gm, h, a.split);
        else
            out = sweep_pair<kLds, RN>(a, sh, a.grid.view(p), p, n, K, Te, rs, r, cbuf, true, c_lo, c_hi,
                                       gm, h, a.split);
        // every thread's target stores have completed before the result is published
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (tid == 0) finish_task(a, rs + r, p, r, h, out, sh.lb);
    }
}

// One workgroup per pair: the sequential loop over the round's sweep results
// (exactly oracle_ransac's order of decisions), the best hypothesis' targets
// kept, and -- once the pair is finished -- its outputs.
template <bool kLds, int RN>
__global__ __launch_bounds__(kThreads) void ransac_replay_kernel(RArgs a) {
    if (round_off(a)) return;
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    Shared &sh = *reinterpret_cast<Shared *>(dsm);
    const int p = blockIdx.x, tid = threadIdx.x;
    const int n = cnt_of(a.n_src, p, a.Nmax), m = cnt_of(a.n_tgt, p, a.Mmax);
    const int K = a.n_corres ? min(max(a.n_corres[p], 0), a.Kmax) : a.Kmax;
    const bool ok = pair_ok(a, p, RN);
    if (tid == 0) {
        RState s = a.state[p];
        const bool was_active = s.active != 0 || a.b0 == 0;  // round 0 finishes invalid pairs
        int best_r = -1;
        if (was_active && s.active) {
            const double scale = fx_scale(a.thr);
            const int nt = a.ntask[p];
            const int *tk = a.tasks + (size_t)p * a.hcap;
            const TaskRes *rs = a.res + (size_t)p * a.hcap;
            for (int r = 0; r < nt; ++r) {
                const int itr = tk[r];
                if (itr >= s.est_k) break;
                const TaskRes tr = rs[r];
                if (tr.status != kDone && tr.status != kCut) {  // cannot happen: guarded
                    atomicAdd(&a.hdr->bad, 1);
                    break;
                }
                const double *T = a.hypT + ((size_t)p * a.hcap + (itr - a.b0)) * 12;
                if (apply_result(s, itr, tr, T, n, K, scale, a.conf, RN)) best_r = r;
            }
            if (best_r >= 0) s.fix = best_r < a.nslots ? 0 : 1;
        }
        const bool fin = !ok || a.b1 >= min(a.max_iter, s.est_k);
        if (was_active) {
            s.active = fin ? 0 : 1;
            a.state[p] = s;
            if (!fin) atomicAdd(&a.hdr->active_count, 1);
        }
        sh.st = s;
        sh.best_r = best_r;
        sh.done = (was_active && fin) ? 1 : 0;
        sh.chunk = 0;
        sh.misses = 0;
        sh.lb = 0;
    }
    __syncthreads();
    const int best_r = sh.best_r;
    int32_t *bb = a.bestbuf + (size_t)p * a.Nmax;
    if (best_r >= 0 && best_r < a.nslots) {  // the new best's targets leave the round's slots
        const int32_t *sl = a.slots + ((size_t)p * a.nslots + best_r) * a.Nmax;
        const int32_t *ord = a.order ? a.order + (size_t)p * a.Nmax : nullptr;
        for (int k = tid; k < n; k += kThreads) bb[ord ? ord[k] : k] = sl[k];  // slots are in sweep order
    }
    if (!sh.done) return;
    const RState &s = sh.st;
    const bool found = ok && s.best_itr >= 0;
    if (found && s.fix) {  // the best had no slot: sweep it once more for its targets
        double Te[12];
        for (int k = 0; k < 12; ++k) Te[k] = s.bestT[k];
        if constexpr (kLds) {
            const GridP4 gl = grid_to_lds4(a.grid, p, m, dsm + ((sizeof(Shared) + 15) & ~size_t(15)));
            (void)sweep_pair<kLds, RN>(a, sh, gl, p, n, K, Te, nullptr, 0, bb, false);
        } else {
            (void)sweep_pair<kLds, RN>(a, sh, a.grid.view(p), p, n, K, Te, nullptr, 0, bb, false);
        }
    }
    __syncthreads();
    // outputs.  Loop exit iteration of the sequential algorithm: first itr >=
    // est_k after the last bound update (or max_iter)
    const int iters = ok ? min(a.max_iter, max(s.last_upd + 1, s.est_k)) : 0;
    if (a.corr_tgt)
        for (int i = tid; i < a.Nmax; i += kThreads)
            a.corr_tgt[(size_t)p * a.Nmax + i] = (found && i < n) ? bb[i] : -1;
    if (a.mask)
        for (int w = tid; w < a.words; w += kThreads) {
            uint32_t bitsw = 0u;
            if (found)
                for (int b = 0; b < 32; ++b) {
                    const int i = 32 * w + b;
                    if (i < n && bb[i] >= 0) bitsw |= 1u << b;
                }
            a.mask[(size_t)p * a.words + w] = bitsw;
        }
    if (tid == 0) {
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
void val_fns(bool lds, const void **sweep, const void **replay) {
    *sweep = lds ? (const void *)ransac_sweep_kernel<true, RN> : (const void *)ransac_sweep_kernel<false, RN>;
    *replay = lds ? (const void *)ransac_replay_kernel<true, RN> : (const void *)ransac_replay_kernel<false, RN>;
}

int env_int(const char *name, int dflt) {  // test hooks (PCR_RANSAC_WGS / _SLOTS)
    const char *e = getenv(name);
    return e && *e ? atoi(e) : dflt;
}

}  // namespace

int ransac_impl(const float *src, const float *tgt, int P, int Nmax, int Mmax,
                const int32_t *n_src, const int32_t *n_tgt, const int32_t *corres,
                const int32_t *n_corres, int Kmax, const uint32_t *pair_ids,
                const pcr_ransac_params *prm, double *T_out, double *fit_out, int32_t *stats,
                int32_t *corr_tgt, uint32_t *mask, hipStream_t s, const int32_t **order_out,
                const GridBatch *grid_in, const int32_t *order_in, const float *perm_in) {
    if (order_out) *order_out = nullptr;
    PCR_REQUIRE(prm->ransac_n >= 3 && prm->ransac_n <= kMaxRansacN, PCR_ERR_ARG,
                "ransac: ransac_n=%d unsupported (3..%d)", prm->ransac_n, kMaxRansacN);
    PCR_REQUIRE(prm->max_iteration >= 0, PCR_ERR_ARG, "ransac: negative max_iteration");
    RArgs a;
    a.src = src; a.tgt = tgt; a.n_src = n_src; a.n_tgt = n_tgt; a.corres = corres;
    a.n_corres = n_corres; a.pair_ids = pair_ids; a.P = P; a.Nmax = Nmax; a.Mmax = Mmax; a.Kmax = Kmax;
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
    a.srcp = nullptr;
    const size_t nm = (size_t)(Nmax > 0 ? Nmax : 1);
    // Rounds.  Device-gated (default): [0, kRound0) and, when max_iteration is
    // larger, ONE more round [kRound0, max_iteration) launched right behind it,
    // whose kernels return at once when no pair is still running (the previous
    // round's active_count) and otherwise stop at each pair's bound -- no host
    // round trip, so the host keeps queueing the next stages (and the call can
    // be captured).  Its slots hold max_iteration - kRound0 hypotheses per pair;
    // past kAsyncSlots slots in all (huge batches) or with PCR_RANSAC_SYNC=1 the
    // host loop of kRoundN-hypothesis rounds runs instead (same results: a
    // round boundary cannot change the sequential decisions).  The round's
    // slots are capped by BYTES (kAsyncBytes; C4's 256 pairs x 98,976 slots take
    // ~3.3 GB of the 288 GB), and when their allocation fails the host loop's
    // kRoundN slots are used instead of failing (decided below, after split).
    constexpr double kAsyncBytes = 16.0 * (1 << 30);
    const int span1 = a.max_iter > kRound0 ? (a.max_iter - kRound0 + 255) / 256 * 256 : 0;
    // target slots of the first tasks of every pair (the best's are kept from
    // there; a best without one is swept again at the end): up to 32 per pair
    // within 256 MB
    const size_t per = sizeof(int32_t) * (size_t)P * nm;
    a.nslots = (int)std::min<size_t>(32, ((size_t)256 << 20) / per);
    a.nslots = std::max(0, std::min(a.nslots, env_int("PCR_RANSAC_SLOTS", a.nslots)));
    a.bestbuf = (int32_t *)workspace(21, per);
    a.state = (RState *)workspace(22, sizeof(RState) * (size_t)P);
    a.hdr = (RHeader *)workspace(25, 2 * sizeof(RHeader) + sizeof(int) * (size_t)P);
    a.slots = (int32_t *)workspace(31, a.nslots > 0 ? per * a.nslots : 16);
    PCR_REQUIRE(a.bestbuf && a.state && a.hdr && a.slots, PCR_ERR_NOMEM, "ransac: %s", pcr_last_error());
    a.ntask = (int *)(a.hdr + 2);
    a.prev_active = nullptr;
    a.grid = GridBatch{};
    a.grid.S = 1;
    a.grid.cell = 1.0;
    if (a.d > 0.0 && Mmax > 0) {
        if (grid_in) {  // built by the caller (pcr_pipeline_step: on its side stream)
            a.grid = *grid_in;
            a.order = Nmax > 0 ? order_in : nullptr;
            a.srcp = Nmax > 0 ? perm_in : nullptr;
        } else {
            int rc = build_grids(tgt, n_tgt, P, Mmax, a.d, s, 4, a.grid, 2.01, 3);
            if (rc != PCR_OK) return rc;
            if (Nmax > 0) {
                rc = spatial_order(src, n_src, P, Nmax, a.grid.cell, s, 13, &a.order, &a.srcp, 36);
                if (rc != PCR_OK) return rc;
            }
        }
        if (order_out) *order_out = a.order;
    }
    const size_t hdr = (sizeof(Shared) + 15) & ~size_t(15);
    const size_t budget = 160 * 1024 - hdr;
    const size_t gbytes = (a.d > 0.0 && Mmax > 0) ? grid_lds4_bytes(Mmax, a.grid.S, budget) : 0;
    const bool lds = gbytes > 0;
    const size_t sm = lds ? hdr + gbytes : hdr;
    const void *hfn = nullptr, *sfn = nullptr, *rfn = nullptr;
    switch (a.rn) {
#define PCR_RCASE(N)                  \
    case N:                           \
        hfn = hyp_fn<N>();            \
        val_fns<N>(lds, &sfn, &rfn);  \
        break;
        PCR_RCASE(3) PCR_RCASE(4) PCR_RCASE(5) PCR_RCASE(6) PCR_RCASE(7) PCR_RCASE(8)
#undef PCR_RCASE
        default: set_error("ransac: bad ransac_n"); return PCR_ERR_ARG;
    }
    PCR_HIP_CHECK(hipFuncSetAttribute(sfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm));
    PCR_HIP_CHECK(hipFuncSetAttribute(rfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm));
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, sfn, kThreads, sm) != hipSuccess ||
        hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
        (void)hipGetLastError();
        per_cu = 1;
        cus = 1;
    }
    const int nwg = std::max(1, env_int("PCR_RANSAC_WGS", std::max(1, per_cu) * std::max(1, cus)));
    // few pairs (multi-GPU shards, single-pair calls): up to 8 workgroups per
    // task, each a slice of the chunks -- the largest power of two with
    // split * P <= workgroups / 4 (256 CUs: 2 at 32 pairs, 8 at 8 or fewer;
    // every part loads the pair's grid, so slices are kept long)
    int split = 1;
    while (split < 8 && 2 * split * P * 4 <= nwg) split <<= 1;
    split = env_int("PCR_RANSAC_SPLIT", split);
    PCR_REQUIRE(split == 1 || split == 2 || split == 4 || split == 8, PCR_ERR_ARG,
                "ransac: PCR_RANSAC_SPLIT=%d (1, 2, 4 or 8)", split);
    a.split = split;
    // the per-hypothesis slots of a round: transforms, pass bits, task list,
    // results (+ split parts)
    const double slot_bytes = 12.0 * sizeof(double) + sizeof(unsigned long long) / 64.0 + sizeof(int) +
                              sizeof(TaskRes) + (split > 1 ? (double)split * sizeof(TaskPart) : 0.0);
    bool gated = env_int("PCR_RANSAC_SYNC", 0) == 0 &&
                 (double)P * std::max(span1, kRound0) * slot_bytes <= kAsyncBytes;
    auto alloc_slots = [&](bool g) {
        // hypotheses per round slot: the largest round that can run (kRound0 when
        // max_iteration fits the first round), a multiple of 256
        a.hcap = a.max_iter > kRound0 ? (g ? std::max(span1, kRound0) : kRoundN)
                                      : std::max(256, (std::max(a.max_iter, 1) + 255) / 256 * 256);
        a.hypT = (double *)workspace(23, sizeof(double) * 12 * (size_t)P * a.hcap);
        a.hypbits = (unsigned long long *)workspace(24, sizeof(unsigned long long) * (size_t)P * (a.hcap / 64));
        a.tasks = (int *)workspace(29, sizeof(int) * (size_t)P * a.hcap);
        a.res = (TaskRes *)workspace(30, sizeof(TaskRes) * (size_t)P * a.hcap);
        a.parts = split > 1 ? (TaskPart *)workspace(32, sizeof(TaskPart) * (size_t)split * P * a.hcap) : nullptr;
        return a.hypT && a.hypbits && a.tasks && a.res && (split == 1 || a.parts);
    };
    if (!alloc_slots(gated)) {
        PCR_REQUIRE(gated, PCR_ERR_NOMEM, "ransac: %s", pcr_last_error());
        clear_error();
        gated = false;  // the host loop's smaller rounds (same results)
        PCR_REQUIRE(alloc_slots(false), PCR_ERR_NOMEM, "ransac: %s", pcr_last_error());
    }
    const int rnarg = a.rn;
    const bool stats_env = env_int("PCR_RANSAC_STATS", 0) != 0;
    prof_begin(s, kProfRansacValidate);
    a.b0 = 0;
    a.b1 = std::min(a.max_iter, kRound0);
    a.clear_hdr = 0;
    if (gated) {
        RHeader *h0 = a.hdr;
        const int nx0 = (a.b1 - a.b0 + kHypThreads - 1) / kHypThreads;
        if (nx0 > 0) a.clear_hdr = 1;  // the first hypothesis launch clears the headers
        else PCR_HIP_CHECK(hipMemsetAsync(a.hdr, 0, 2 * sizeof(RHeader), s));
        for (int round = 0; round < (a.max_iter > kRound0 ? 2 : 1); ++round) {
            if (round == 1) {
                a.clear_hdr = 0;
                a.b0 = kRound0;
                a.b1 = a.max_iter;
                a.hdr = h0 + 1;
                a.prev_active = &h0->active_count;
            }
            void *args[] = {&a};
            const int nx = (a.b1 - a.b0 + kHypThreads - 1) / kHypThreads;
            if (nx > 0) {
                PCR_HIP_CHECK(hipLaunchKernel(hfn, dim3(round == 0 ? nx : std::min(nx, 16), P),
                                              dim3(kHypThreads), args, 0, s));
                PCR_LAUNCH_CHECK();
            }
            void *targs[] = {&a, (void *)&rnarg};
            PCR_HIP_CHECK(hipLaunchKernel((const void *)ransac_task_kernel, dim3(P), dim3(64), targs, 0, s));
            PCR_LAUNCH_CHECK();
            PCR_HIP_CHECK(hipLaunchKernel(sfn, dim3(nwg), dim3(kThreads), args, sm, s));
            PCR_LAUNCH_CHECK();
            PCR_HIP_CHECK(hipLaunchKernel(rfn, dim3(P), dim3(kThreads), args, sm, s));
            PCR_LAUNCH_CHECK();
        }
        prof_end(s, kProfRansacValidate);
        if (stats_env) {  // diagnostics only: one host read of both headers
            RHeader h[2];
            PCR_HIP_CHECK(hipMemcpyAsync(h, h0, sizeof(h), hipMemcpyDeviceToHost, s));
            PCR_HIP_CHECK(hipStreamSynchronize(s));
            for (int r = 0; r < 2; ++r)
                fprintf(stderr, "ransac gated round %d: tasks done %d cut %d skipped %d, chunks %d, active after %d, "
                        "bad %d\n", r, h[r].n_done, h[r].n_cut, h[r].n_skip, h[r].n_chunks, h[r].active_count,
                        h[r].bad);
        }
        return PCR_OK;
    }
    // host loop: [0, kRound0), then kRoundN at a time while a pair is still running
    for (;;) {
        PCR_HIP_CHECK(hipMemsetAsync(a.hdr, 0, sizeof(RHeader), s));
        const int span = a.b1 - a.b0;
        void *args[] = {&a};
        if (span > 0) {
            PCR_HIP_CHECK(hipLaunchKernel(hfn, dim3((span + kHypThreads - 1) / kHypThreads, P),
                                          dim3(kHypThreads), args, 0, s));
            PCR_LAUNCH_CHECK();
        }
        {
            void *targs[] = {&a, (void *)&rnarg};
            PCR_HIP_CHECK(hipLaunchKernel((const void *)ransac_task_kernel, dim3(P), dim3(64), targs, 0, s));
            PCR_LAUNCH_CHECK();
        }
        PCR_HIP_CHECK(hipLaunchKernel(sfn, dim3(nwg), dim3(kThreads), args, sm, s));
        PCR_LAUNCH_CHECK();
        PCR_HIP_CHECK(hipLaunchKernel(rfn, dim3(P), dim3(kThreads), args, sm, s));
        PCR_LAUNCH_CHECK();
        RHeader h;
        PCR_HIP_CHECK(hipMemcpyAsync(&h, a.hdr, sizeof(RHeader), hipMemcpyDeviceToHost, s));
        PCR_HIP_CHECK(hipStreamSynchronize(s));
        PCR_REQUIRE(h.bad == 0, PCR_ERR_HIP, "ransac: %d pairs met an unswept task", h.bad);
        if (stats_env)
            fprintf(stderr, "ransac round [%d,%d): tasks done %d cut %d skipped %d, chunks %d (%.2f full sweeps)\n",
                    a.b0, a.b1, h.n_done, h.n_cut, h.n_skip, h.n_chunks,
                    h.n_chunks / (double)std::max(1, (Nmax + 63) / 64));
        if (a.b1 >= a.max_iter || h.active_count == 0) break;
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
                            pcr::as_stream(stream), nullptr, nullptr, nullptr, nullptr);
}
