// a8: batched point-to-point ICP (Open3D 0.13 RegistrationICP as called from
// DataPreparation/RANSAC.py:61-63 and dip/preprocess_correspondences.py:48,83).
// Contract: oracle_icp (pcr_oracle.c).
//
// MI355X design: the whole ICP loop of a pair runs inside one launch (no host
// round trips), on one 1024-thread workgroup per pair -- or on G workgroups per
// pair meeting at a per-pair barrier (cooperative launch, coop.h) when the batch
// has fewer pairs than the chip has CUs.  Each workgroup holds the pair's target
// hash grid in LDS.
//  * The f64 working copy (transformed in place every iteration, as Open3D's
//    Transform does) is stored by POSITION in the spatial (Morton-of-cell)
//    order, and the sweep takes 64-query chunks of that order from a counter:
//    a chunk's loads and stores are one contiguous 1.5 KB run (stored by source
//    index, every lane touched a line of its own through the order).
//  * Per iteration ONE sweep: every point is transformed by the last update,
//    queried in the grid (radius-limited 1-NN), and -- if it has a
//    correspondence -- its Umeyama terms are added to the thread's sums right
//    there: s - c0, t - c0 and their 9 products, each truncated to a multiple of
//    a per-pair quantum 2^-k small enough that every partial sum is an integer
//    multiple of 2^-k below 2^52 (oracle_icp_quantum).  The f64 additions are
//    then exact, so any split over threads, waves and workgroups gives the same
//    bits; the means and the cross-covariance (C = Sst - ms' St^T) come out of
//    the sweep and one reduction, with no correspondence array written or
//    re-read (the sums are kept in quanta and scaled by 2^-k once).  Horn's
//    quaternion solve and the T <- U*T update run redundantly in every
//    workgroup on the same totals.
#include "pcr_internal.h"
#include "coop.h"
#include "geom.h"
#include "grid.h"
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

namespace pcr {
namespace {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;
constexpr int kQ = 15;  // exact sums: s' (3), t' (3), s'_a t'_b (9)

// one workgroup's partial of a reduction (G > 1): HBM slot per (pair, parity, g)
struct XPart {
    double s[kQ];
    unsigned long long acc;
    int cnt, pad;
};

struct IArgs {
    const float *src, *tgt;
    const int32_t *n_src, *n_tgt;
    int Nmax, Mmax;
    const double *init;  // P x 16
    double d, thr, rel_fit, rel_rmse;
    int max_iter;
    GridBatch grid;
    double *P3;          // P x Nmax x 3 working copy by position in the order
    int4 *cst;           // P x Nmax correspondence state by position (see CorrState)
    const float *srcp;   // (P, Nmax, 3) the source points in that order, or null
    double *T_out, *fit_out;
    int32_t *stats;
    int32_t *corr_tgt;   // optional (P, Nmax): final correspondence per source point
    const int32_t *order;  // (P, Nmax) spatial order of the source points, or null
    int G;               // workgroups per pair (phase 2: computed on the device)
    // tail rebalancing (phase 1 / 2; phase 0 = one launch as before): phase 1 runs
    // every pair on one workgroup and, once at most thr_active pairs are still
    // iterating, the rest save their state and list themselves; phase 2 spreads
    // the listed pairs over all CUs (G = grid / listed) and finishes them
    int phase, thr_active, gmax2;
    int *ctl;            // [0] pairs still iterating in phase 1, [1] listed pairs
    int *list;           // (P) listed pairs
    double *save;        // (P, kSave) the listed pairs' state
    XPart *part;         // (P, 2, G) when G > 1
    // when G > 1: per pair 4 words at bar + 4 p, the pair barrier (arrivals,
    // generation)
    unsigned *bar;
    unsigned long long *timing;  // debug (PCR_ICP_TIMING): per pair, phase clocks
};

// The working copy when a pair has G > 1 workgroups: each pair barrier's
// release fence writes back the XCD L2's dirty lines, and a sweep dirtied ~48 KB
// of working copy per workgroup (2,048 points x 24 B at 32 pairs, G = 4).
// Stored write-through (sc1: the line leaves L2 clean) there is nothing of it to
// write back; visibility is still the barrier's release / acquire.
__device__ __forceinline__ void put3(double *q, double x, double y, double z, bool wt) {
    if (wt) {
        __hip_atomic_store(q, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(q + 1, y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(q + 2, z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        q[0] = x; q[1] = y; q[2] = z;
    }
}

// Correspondence reuse.  A point's grid walk also reports the two smallest
// distances it computed and a lower bound rho on the distance to any target it
// did not examine (grid.h kClear), which give a clearance c: every target other
// than the winner w lies at least c = min(second smallest, rho) from the point
// (with no correspondence: every target at least min(smallest, rho)).  Moved
// since by at most D (the summed step lengths), the point is still strictly
// nearest to w -- the walk would return w, with the same d2 bits -- while
// |p - w| < c - D and d2 < thr; without one it still has none while c - D >
// sqrt(thr).  Such a point skips the walk.  Per position, int4 {w's grid slot
// or -1, c (f32, rounded down), D (f32, rounded up), unused}; rewritten by every
// walk (D = 0).
__device__ __forceinline__ void put_state(int4 *q, int4 v, bool wt) {
    if (wt) {
        int *w = reinterpret_cast<int *>(q);
        __hip_atomic_store(w, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(w + 1, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(w + 2, v.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        *q = v;
    }
}
__device__ __forceinline__ void put_step(int4 *q, int z, bool wt) {
    int *w = reinterpret_cast<int *>(q) + 2;
    if (wt) __hip_atomic_store(w, z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *w = z;
}

// a listed pair's state: T (16), C (9), ms (3), mt (3), fit, rmse, count, it
constexpr int kSave = 36;

__device__ __forceinline__ int cnt_of(const int32_t *n, int p, int mx) {
    return n ? min(max(n[p], 0), mx) : mx;
}

struct IShared {  // LDS header; the grid copy (if any) follows
    double ws[kWaves][kQ];
    unsigned long long wacc[kWaves];
    int wcnt[kWaves];
    double tot[kQ];
    double C[9];      // cross-covariance of the current correspondences
    double c0[3];     // the pair's reference point (first target point)
    double ms[3], mt[3];  // Umeyama means of the current correspondences
    double sk, isk;   // 2^k, 2^-k: the quantum of the exact sums
    double bt[kWaves];
    unsigned long long acc;
    int cnt;
    double T[16];     // the running transformation (init, then U * T per iteration)
    double U[12];     // this iteration's update
    int nred;         // reductions done (parity of the HBM partial slots)
    int chunk[2];     // next 64-position chunk of this workgroup's range, by sweep parity
    int handoff;      // phase 1: this pair is listed for phase 2
    int pend[kWaves][128];  // per wave: positions waiting for a grid walk (a stack)
    int nwalk;        // debug (PCR_ICP_PHASES): walks done by this workgroup
};

// wave-level sums of the kQ exact f64 values (integer multiples of the quantum:
// the additions are exact, so the tree shape is free), parked in
// sh.ws[wave][0..kQ).  A reduce-scatter butterfly: at each of the offsets 32,
// 16, 8, 4 a lane keeps half of its values and adds its partner's copy of that
// half (8 + 4 + 2 + 1 shuffles instead of 6 per value), then offsets 2, 1 finish
// the one value left -- lane l ends with value (l >> 2) summed over the wave.
__device__ __forceinline__ void wave_park(IShared &sh, const double *v) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double w[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) w[q] = q < kQ ? v[q] : 0.0;
    auto step = [&](auto hc) {
        constexpr int h = decltype(hc)::value, o = 4 * h;
        const bool up = (lane & o) != 0;  // keeps the upper half
#pragma unroll
        for (int i = 0; i < h; ++i) {
            const double keep = up ? w[i + h] : w[i], send = up ? w[i] : w[i + h];
            w[i] = keep + __shfl_xor(send, o, 64);
        }
    };
    step(std::integral_constant<int, 8>{});
    step(std::integral_constant<int, 4>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 1>{});
    double t = w[0];
    t += __shfl_xor(t, 2, 64);
    t += __shfl_xor(t, 1, 64);
    // lane bits 5..2 picked the half at offsets 32..4: lane l holds value
    // (l >> 5 & 1) * 8 + (l >> 4 & 1) * 4 + (l >> 3 & 1) * 2 + (l >> 2 & 1)
    const int q = lane >> 2;
    if ((lane & 3) == 0 && q < kQ) sh.ws[wid][q] = t;
}

// sum the NV parked values + (cnt, acc) over the pair's workgroups; result in
// sh.tot / sh.cnt / sh.acc (all threads call; ends with a barrier)
// mk(ph): debug phase clocks (PCR_ICP_PHASES): 5 = the workgroup's waves
// joined, 6 = the pair barrier passed
template <int NV, typename Mark>
__device__ void pair_reduce(const IArgs &a, IShared &sh, int p, int g, int G, int cnt,
                            unsigned long long acc, Mark mk) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        cnt += __shfl_xor(cnt, o, 64);
        acc += __shfl_xor(acc, o, 64);
    }
    if (lane == 0) {
        sh.wcnt[wid] = cnt;
        sh.wacc[wid] = acc;
    }
    __syncthreads();
    mk(5);
    if (tid < NV + 2) {  // thread q sums quantity q (NV: count, NV+1: error sum)
        double s = 0.0;
        unsigned long long A = 0;
        int C = 0;
        for (int w = 0; w < kWaves; ++w) {
            if (tid < NV) s += sh.ws[w][tid];
            else if (tid == NV) C += sh.wcnt[w];
            else A += sh.wacc[w];
        }
        if (G > 1) {
            XPart &me = a.part[((size_t)p * 2 + (sh.nred & 1)) * G + g];
            if (tid < NV) me.s[tid] = s;
            else if (tid == NV) me.cnt = C;
            else me.acc = A;
        } else {
            if (tid < NV) sh.tot[tid] = s;
            else if (tid == NV) sh.cnt = C;
            else sh.acc = A;
        }
    }
    if (G > 1) {
        pair_barrier(a.bar + 4 * (size_t)p, G);
        mk(6);
        if (tid < NV + 2) {
            const XPart *all = a.part + ((size_t)p * 2 + (sh.nred & 1)) * G;
            double s = 0.0;
            unsigned long long A = 0;
            int C = 0;
            for (int h = 0; h < G; ++h) {
                if (tid < NV) s += all[h].s[tid];
                else if (tid == NV) C += all[h].cnt;
                else A += all[h].acc;
            }
            if (tid < NV) sh.tot[tid] = s;
            else if (tid == NV) sh.cnt = C;
            else sh.acc = A;
        }
    }
    __syncthreads();
    if (tid == 0) sh.nred += 1;  // read only by threads < NV + 2 after the next barrier
}

template <bool kLds>
__global__ __launch_bounds__(kThreads) void icp_kernel(IArgs a) {
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    IShared &sh = *reinterpret_cast<IShared *>(dsm);
    int G = a.G, p, g;
    if (a.phase == 2) {
        // the listed pairs over the whole grid (uniform in every workgroup)
        const int R = __hip_atomic_load(&a.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (R <= 0) return;
        G = max(1, min(a.gmax2, (int)gridDim.x / R));
        if ((int)blockIdx.x >= R * G) return;  // whole workgroup, before any barrier
        p = a.list[blockIdx.x / G];
        g = blockIdx.x - (blockIdx.x / G) * G;
    } else {
        p = blockIdx.x / G;
        g = blockIdx.x - p * G;
    }
    const bool resume = a.phase == 2;
    const int n = cnt_of(a.n_src, p, a.Nmax);
    const int m = cnt_of(a.n_tgt, p, a.Mmax);
    const int tid = threadIdx.x, lane = tid & 63;
    const float *S = a.src + (size_t)p * a.Nmax * 3;
    const int32_t *ord = a.order ? a.order + (size_t)p * a.Nmax : nullptr;
    // working copy (f64 xyz) by source INDEX, AoS
    double *P3 = a.P3 + (size_t)p * a.Nmax * 3;
    int4 *cst = a.cst + (size_t)p * a.Nmax;
    const bool wt = G > 1;  // working copy / state stores write-through (put3)
    int32_t *CT = a.corr_tgt ? a.corr_tgt + (size_t)p * a.Nmax : nullptr;
    const double *sv = resume ? a.save + (size_t)p * kSave : nullptr;
    if (tid < 16) sh.T[tid] = resume ? sv[tid] : a.init[(size_t)p * 16 + tid];
    if (tid == 0) { sh.nred = 0; sh.chunk[0] = 0; sh.chunk[1] = 0; sh.handoff = 0; sh.nwalk = 0; }
    __syncthreads();
    const bool valid = a.d > 0.0 && n > 0 && m > 0;
    bool ident = true;
    for (int k = 0; k < 16; ++k) ident = ident && (sh.T[k] == ((k % 5 == 0) ? 1.0 : 0.0));
    const int stride = G * kThreads, base = g * kThreads + tid;
    // the workgroup's share of the sweep order: 64-position chunks [c_lo, c_hi),
    // the same in every sweep (its waves take them from an LDS counter), so a
    // position's working copy and state are only ever touched by one workgroup
    const int nch = (n + 63) >> 6;
    const int c_lo = (int)((long long)nch * g / G), c_hi = (int)((long long)nch * (g + 1) / G);
    // the pair's reference point and quantum of the exact Umeyama sums
    // (oracle_icp_quantum): c0 = the first target point, 2^k from the largest
    // |t - c0| (every workgroup computes the same values)
    if (valid) {
        const float *Tg = a.tgt + (size_t)p * a.Mmax * 3;
        const double c0x = (double)Tg[0], c0y = (double)Tg[1], c0z = (double)Tg[2];
        double bt = 0.0;
        for (int j = tid; j < m; j += kThreads)
            bt = fmax(bt, fmax(fabs((double)Tg[3 * j] - c0x),
                               fmax(fabs((double)Tg[3 * j + 1] - c0y), fabs((double)Tg[3 * j + 2] - c0z))));
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) bt = fmax(bt, __shfl_xor(bt, o, 64));
        if (lane == 0) sh.bt[tid >> 6] = bt;
        if (tid == 0) { sh.c0[0] = c0x; sh.c0[1] = c0y; sh.c0[2] = c0z; }
        __syncthreads();
        bt = sh.bt[0];
        for (int w = 1; w < kWaves; ++w) bt = fmax(bt, sh.bt[w]);
        const double B = bt + 2.0 * a.d;
        int eb = 0;
        (void)frexp(B, &eb);
        const int emax = eb > 2 * eb ? eb : 2 * eb;
        int en = 0;
        while ((1LL << en) < (long long)(n > 1 ? n : 1)) ++en;
        const int k = min(200, max(-200, 52 - en - emax));
        if (tid == 0) { sh.sk = ldexp(1.0, k); sh.isk = ldexp(1.0, -k); }
    }
    if (valid && !resume) {  // working copy = init applied to the f32 input (Open3D's Transform)
        double T0[12];
        for (int q = 0; q < 12; ++q) T0[q] = sh.T[q];
        const float *Sp = (a.srcp && ord) ? a.srcp + (size_t)p * a.Nmax * 3 : nullptr;
        for (int k = 64 * c_lo + tid; k < min(n, 64 * c_hi); k += kThreads) {
            const float *q = Sp ? Sp + 3 * k : S + 3 * (ord ? ord[k] : k);
            double x = (double)q[0], y = (double)q[1], z = (double)q[2];
            if (!ident) {
                double ox, oy, oz;
                xform12(T0, x, y, z, ox, oy, oz);
                x = ox; y = oy; z = oz;
            }
            put3(P3 + 3 * k, x, y, z, wt);
        }
    }
    GridP4 gl{};
    GridView gg{};
    if (valid) {
        if constexpr (kLds) gl = grid_to_lds4(a.grid, p, m, dsm + ((sizeof(IShared) + 15) & ~size_t(15)));
        else gg = a.grid.view(p);
    }
    __syncthreads();
    const double scale = fx_scale(a.thr);
    const int wid = tid >> 6;
    // debug phase clocks (s_memtime) of workgroup 0's thread 0: only in a build
    // with -DPCR_ICP_PHASES (the registers they hold cost the normal build)
#ifdef PCR_ICP_PHASES
    const bool tmg = a.timing != nullptr && g == 0 && tid == 0;
#else
    const bool tmg = false;
#endif
    unsigned long long tph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tlast = tmg ? __builtin_readcyclecounter() : 0ull;
    const unsigned long long t00 = tlast;
    auto mark = [&](int ph) {
        if (tmg) {
            const unsigned long long t = __builtin_readcyclecounter();
            tph[ph] += t - tlast;
            tlast = t;
        }
    };
    auto sync_pair = [&]() {
        if (G > 1) pair_barrier(a.bar + 4 * (size_t)p, G);
        else __syncthreads();
    };
    double fit = 0.0, rmse = 0.0;
    int count = 0;
    // correspondences of the current points, their count / error sum and the
    // Umeyama means
    // with_u: this iteration's update U is applied to the working copy inside
    // the sweep (each point read, transformed, written back and queried by the
    // same thread), which saves the separate transform pass and a pair barrier
    int nsweep = 0;  // sweeps done: parity of the chunk counters
    auto evaluate = [&](bool with_u) {
        unsigned long long acc = 0;
        int cnt = 0;
        double v[kQ];
#pragma unroll
        for (int q = 0; q < kQ; ++q) v[q] = 0.0;
        {  // 64-query chunks of the spatial order taken from a counter (dense and
           // sparse regions cost different time); the counter of this sweep's
           // parity was re-armed after the previous sweep's reduction
            int *ctr = &sh.chunk[nsweep & 1];
            const double c0x = sh.c0[0], c0y = sh.c0[1], c0z = sh.c0[2];
            // the exact Umeyama terms of a correspondence, in quanta: trunc(s'_a
            // 2^k), trunc(t'_b 2^k), trunc(s'_a t'_b 2^k) -- the scaling by 2^k is
            // exact, so (s'_a 2^k) t'_b rounds to the same value as (s'_a t'_b)
            // 2^k; the sums (integers below 2^52) are scaled back by 2^-k after
            // the reduction
            auto add_corr = [&](double *vv, int &cn, unsigned long long &ac, double x, double y, double z,
                                float qx, float qy, float qz, double d2) {
                ++cn;
                ac += (unsigned long long)(d2 * scale);
                const volatile double *skv = &sh.sk;
                const double sk = skv[0];
                const double sps[3] = {(x - c0x) * sk, (y - c0y) * sk, (z - c0z) * sk};
                const double tp[3] = {(double)qx - c0x, (double)qy - c0y, (double)qz - c0z};
#pragma unroll
                for (int cc = 0; cc < 3; ++cc) {
                    vv[cc] = vv[cc] + __builtin_trunc(sps[cc]);
                    vv[3 + cc] = vv[3 + cc] + __builtin_trunc(tp[cc] * sk);
#pragma unroll
                    for (int e = 0; e < 3; ++e)
                        vv[6 + 3 * cc + e] = vv[6 + 3 * cc + e] + __builtin_trunc(sps[cc] * tp[e]);
                }
            };
            // the grid walk of position k (its point already transformed): the
            // correspondence, and the state that lets later sweeps reuse it
            auto walk = [&](int k) {
#ifdef PCR_ICP_PHASES
                atomicAdd(&sh.nwalk, 1);
#endif
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // this wave's P3 stores
                const double x = P3[3 * k], y = P3[3 * k + 1], z = P3[3 * k + 2];
                double d2, e12[3];
                int q, sl;
                float qx = 0.f, qy = 0.f, qz = 0.f, qw;
                if constexpr (kLds) {
                    q = grid_query_exact<GridP4, true, 2, true>(gl, a.d, a.thr, x, y, z, d2, &sl, e12);
                    if (q >= 0) gl.load(sl, qx, qy, qz, qw);
                } else {
                    q = grid_query_exact<GridView, true, 2, true>(gg, a.d, a.thr, x, y, z, d2, &sl, e12);
                    if (q >= 0) gg.load(sl, qx, qy, qz, qw);
                }
                if (CT) CT[ord ? ord[k] : k] = q;
                // the clearance: to every target other than the winner (a
                // correspondence), or to every target (none within d)
                const float cf = (float)(__builtin_sqrt(__builtin_fmin(q >= 0 ? e12[1] : e12[0], e12[2])) *
                                         (1.0 - 2e-6));
                put_state(cst + k, make_int4(q >= 0 ? sl : -1, __float_as_int(cf), 0, 0), wt);
                if (q >= 0) add_corr(v, cnt, acc, x, y, z, qx, qy, qz, d2);
            };
            int np = 0;  // positions on this wave's stack
            for (;;) {
                int c = 0;
                if (lane == 0) c = atomicAdd(ctr, 1);
                c = __shfl(c, 0, 64) + c_lo;
                if (c >= c_hi) break;
                const int k = (c << 6) + lane;
                // phase A: transform; reuse the correspondence when certified
                bool need = false;
                if (k < n) {
                    double x = P3[3 * k], y = P3[3 * k + 1], z = P3[3 * k + 2];
                    if (!with_u) {
                        need = true;
                    } else {  // U from LDS per chunk (volatile: not held across the query)
                        const volatile double *Uv = sh.U;
                        double U[12];
#pragma unroll
                        for (int q = 0; q < 12; ++q) U[q] = Uv[q];
                        double ox, oy, oz;
                        xform12(U, x, y, z, ox, oy, oz);
                        put3(P3 + 3 * k, ox, oy, oz, wt);
                        const int4 st = cst[k];
                        // D += this step's length (rounded up)
                        const double dx = ox - x, dy = oy - y, dz = oz - z;
                        const double Dn = (double)__int_as_float(st.z) +
                                          __builtin_sqrt((dx * dx + dy * dy) + dz * dz) * (1.0 + 1e-9);
                        const double room = ((double)__int_as_float(st.y) - Dn) * (1.0 - 1e-12);
                        need = true;
                        if (st.x < 0) {
                            // no target within d at the walk: still none while every
                            // target stays farther than sqrt(thr) (the walk would find
                            // d2 >= thr for each)
                            if (room > __builtin_sqrt(a.thr) * (1.0 + 1e-9)) {
                                need = false;
                                put_step(cst + k, __float_as_int((float)(Dn * (1.0 + 1e-6) + 1e-30)), wt);
                                if (CT) CT[ord ? ord[k] : k] = -1;
                            }
                        } else {
                            float qx, qy, qz, qw;
                            if constexpr (kLds) gl.load(st.x, qx, qy, qz, qw);
                            else gg.load(st.x, qx, qy, qz, qw);
                            const double d2 = dist2(ox, oy, oz, (double)qx, (double)qy, (double)qz);
                            if (d2 < a.thr && __builtin_sqrt(d2) * (1.0 + 1e-9) < room) {
                                need = false;
                                put_step(cst + k, __float_as_int((float)(Dn * (1.0 + 1e-6) + 1e-30)), wt);
                                if (CT) CT[ord ? ord[k] : k] = __float_as_int(qw);
                                add_corr(v, cnt, acc, ox, oy, oz, qx, qy, qz, d2);
                            }
                        }
                    }
                }
                // phase B: the positions needing a walk wait on the wave's stack and
                // are walked 64 at a time (full waves)
                const unsigned long long need_m = __ballot(need);
                if (need) sh.pend[wid][np + __builtin_amdgcn_mbcnt_hi((unsigned)(need_m >> 32),
                                             __builtin_amdgcn_mbcnt_lo((unsigned)need_m, 0u))] = k;
                np += __popcll(need_m);
                if (np >= 64) {
                    np -= 64;
                    walk(sh.pend[wid][np + lane]);
                }
            }
            mark(7);
            if (lane < np) walk(sh.pend[wid][lane]);  // the rest of the stack
        }
        mark(0);
        wave_park(sh, v);
        mark(4);
        pair_reduce<kQ>(a, sh, p, g, G, cnt, acc, mark);
        // every workgroup has left this sweep (pair_reduce's barrier): re-arm its
        // counter for the sweep after next (the next sweep uses the other one,
        // re-armed one reduction ago)
        if (tid == 0) sh.chunk[nsweep & 1] = 0;
        ++nsweep;
        mark(1);
        count = sh.cnt;
        if (count > 0) {
            fit = (double)count / (double)n;
            rmse = __builtin_sqrt(((double)sh.acc / scale) / (double)count);
            const double inv = 1.0 / (double)count;
            if (tid == 0) {
                double tot[kQ], msp[3];
                for (int q = 0; q < kQ; ++q) tot[q] = sh.tot[q] * sh.isk;  // quanta -> values (exact)
                for (int c = 0; c < 3; ++c) {
                    msp[c] = tot[c] * inv;
                    sh.ms[c] = msp[c] + sh.c0[c];
                    sh.mt[c] = tot[3 + c] * inv + sh.c0[c];
                }
                for (int c = 0; c < 3; ++c)
                    for (int e = 0; e < 3; ++e) sh.C[3 * c + e] = tot[6 + 3 * c + e] - msp[c] * tot[3 + e];
            }
        } else {
            fit = 0.0;
            rmse = 0.0;
        }
        __syncthreads();  // sh.tot is rewritten by the next reduction
    };
    int it = 0;
    bool handed = false;
    if (valid) {
        if (resume) {  // the state phase 1 left: the last sweep's sums, fit, rmse
            if (tid < 9) sh.C[tid] = sv[16 + tid];
            if (tid < 3) { sh.ms[tid] = sv[25 + tid]; sh.mt[tid] = sv[28 + tid]; }
            fit = sv[31];
            rmse = sv[32];
            count = (int)sv[33];
            it = (int)sv[34];
            __syncthreads();
        } else {
            evaluate(false);
        }
        for (; it < a.max_iter;) {
            if (count == 0) break;
            mark(2);
            if (tid == 0) {
                double Sm[9], R[9], U[12];
                for (int k = 0; k < 9; ++k) Sm[k] = sh.C[k];
                horn_rotation(Sm, R);
                double ms[3], mt[3];
                for (int c = 0; c < 3; ++c) { ms[c] = sh.ms[c]; mt[c] = sh.mt[c]; }
                compose_rt(R, ms, mt, U);
                double Tn[16];
                for (int r = 0; r < 4; ++r)
                    for (int c = 0; c < 4; ++c) {
                        const double u0 = r < 3 ? U[4 * r + 0] : 0.0, u1 = r < 3 ? U[4 * r + 1] : 0.0,
                                     u2 = r < 3 ? U[4 * r + 2] : 0.0, u3 = r < 3 ? U[4 * r + 3] : 1.0;
                        Tn[4 * r + c] =
                            ((u0 * sh.T[c] + u1 * sh.T[4 + c]) + u2 * sh.T[8 + c]) + u3 * sh.T[12 + c];
                    }
                for (int k = 0; k < 16; ++k) sh.T[k] = Tn[k];
                for (int k = 0; k < 12; ++k) sh.U[k] = U[k];
            }
            __syncthreads();
            mark(3);
            // (the points are transformed in place by the next sweep)
            const double pf = fit, pr = rmse;
            evaluate(true);
            ++it;
            if (__builtin_fabs(pf - fit) < a.rel_fit && __builtin_fabs(pr - rmse) < a.rel_rmse) break;
            if (a.phase == 1 && it < a.max_iter && count > 0) {
                // few pairs still iterating: hand this one to phase 2 (G = 1 here)
                if (tid == 0)
                    sh.handoff = __hip_atomic_load(&a.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <=
                                 a.thr_active;
                __syncthreads();
                if (sh.handoff) {
                    if (tid == 0) {
                        double *o = a.save + (size_t)p * kSave;
                        for (int k = 0; k < 16; ++k) o[k] = sh.T[k];
                        for (int k = 0; k < 9; ++k) o[16 + k] = sh.C[k];
                        for (int k = 0; k < 3; ++k) { o[25 + k] = sh.ms[k]; o[28 + k] = sh.mt[k]; }
                        o[31] = fit;
                        o[32] = rmse;
                        o[33] = (double)count;
                        o[34] = (double)it;
                        a.list[atomicAdd(&a.ctl[1], 1)] = p;
                    }
                    handed = true;
                    break;
                }
            }
        }
    }
    if (a.phase == 1 && !handed && tid == 0)  // this pair is done: one fewer iterating
        __hip_atomic_fetch_add(&a.ctl[0], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (handed) return;  // phase 2 writes its outputs
    if (CT) {  // the last sweep wrote CT[0, n) when valid
        for (int i = valid ? n + base : base; i < a.Nmax; i += stride) CT[i] = -1;
    }
    if (g == 0 && tid == 0) {
        for (int k = 0; k < 16; ++k) a.T_out[(size_t)p * 16 + k] = sh.T[k];
        a.fit_out[2 * p] = valid ? fit : 0.0;
        a.fit_out[2 * p + 1] = valid ? rmse : 0.0;
        a.stats[2 * p] = it;
        a.stats[2 * p + 1] = valid ? count : 0;
        if (tmg) {
            unsigned long long *tt = a.timing + (size_t)p * 12;
            for (int k = 0; k < 8; ++k) tt[k] = tph[k];
            tt[8] = __builtin_readcyclecounter() - t00;
            tt[9] = (unsigned long long)it;
            tt[10] = (unsigned long long)sh.nwalk;
        }
    }
}


const void *icp_fn(bool lds) {
    return lds ? (const void *)icp_kernel<true> : (const void *)icp_kernel<false>;
}

}  // namespace

int icp_impl(const float *src, const float *tgt, int P, int Nmax, int Mmax, const int32_t *n_src,
             const int32_t *n_tgt, const double *init, const pcr_icp_params *prm, double *T_out,
             double *fit_out, int32_t *stats, int32_t *corr_tgt, hipStream_t s, const int32_t *order_in,
             const GridBatch *grid_in, const float *perm_in) {
    IArgs a;
    a.src = src; a.tgt = tgt; a.n_src = n_src; a.n_tgt = n_tgt; a.Nmax = Nmax; a.Mmax = Mmax;
    a.init = init;
    a.order = nullptr;
    a.d = prm->max_correspondence_distance;
    a.thr = radius_thr(a.d);
    a.rel_fit = prm->relative_fitness;
    a.rel_rmse = prm->relative_rmse;
    a.max_iter = prm->max_iteration;
    a.P3 = nullptr;
    a.cst = nullptr;
    a.srcp = nullptr;
    if (a.d > 0.0) {
        int rc = PCR_OK;
        if (grid_in) a.grid = *grid_in;  // built by the caller (pcr_pipeline_step's side stream)
        else rc = build_grids(tgt, n_tgt, P, Mmax, a.d, s, 7, a.grid);
        if (rc != PCR_OK) return rc;
        if (Nmax > 0) {
            // any spatial order serves (it only groups a wave's queries): the
            // pipeline hands over RANSAC's, sorted by its coarser cells
            if (order_in) {
                a.order = order_in;
                a.srcp = perm_in;
            } else {
                rc = spatial_order(src, n_src, P, Nmax, a.grid.cell, s, 14, &a.order, &a.srcp, 35);
                if (rc != PCR_OK) return rc;
            }
        }
    } else {
        a.grid = GridBatch{};
        a.grid.S = 1;
        a.grid.cell = 1.0;
    }
    a.T_out = T_out; a.fit_out = fit_out; a.stats = stats; a.corr_tgt = corr_tgt;
    const size_t hdr = (sizeof(IShared) + 15) & ~size_t(15);
    const size_t gbytes = (a.d > 0.0 && Mmax > 0) ? grid_lds4_bytes(Mmax, a.grid.S, 160 * 1024 - hdr) : 0;
    const bool lds = gbytes > 0;
    const size_t sm = lds ? hdr + gbytes : hdr;
    const void *fn = icp_fn(lds);
    PCR_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm));
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kThreads, sm) != hipSuccess) {
        (void)hipGetLastError();
        per_cu = 0;
    }
    // at most 4: an ICP iteration meets at four pair barriers, and past 4
    // workgroups their cost outgrows the split sweep (32-pair shard: G = 4
    // 0.80 ms, G = 8 0.97 ms; RANSAC, two barriers per sweep, is best at 8)
    a.G = coop_groups(P, per_cu, 4);
    a.phase = 0;
    a.thr_active = 0;
    a.gmax2 = 8;
    a.ctl = nullptr;
    a.list = nullptr;
    a.save = nullptr;
    // tail rebalancing: a batch that fills the chip with one workgroup per pair
    // (G = 1) ends on a few slow pairs -- C4: 4.6 iterations per pair on average,
    // 8 at most, so ~40 % of the CU-time of the launch sat idle.  Phase 1 hands
    // the last thr_active pairs still iterating to a second, cooperative launch
    // that gives each of them G = CUs / listed workgroups (PCR_ICP_TAIL=0: one
    // launch).  The sums are exact, so G changes no bit.
    const char *tail_env = getenv("PCR_ICP_TAIL");
    const bool tail_on = !(tail_env && atoi(tail_env) == 0);
    // phase 2 is sized like coop_groups' grids: this launch's share of the chip
    // when pcr_set_concurrency(k) lets k launches run at once, so concurrent
    // phase-2 grids are all resident together (their pair barriers spin)
    const int grid2 = coop_capacity(per_cu);
    const bool two_phase = tail_on && a.G == 1 && a.d > 0.0 && Nmax > 0 && grid2 >= 4 && P >= grid2 / 2;
    if (two_phase) a.thr_active = grid2 / 4;  // phase 2: >= 4 workgroups per listed pair
    // working copy, by position
    const size_t nm = (size_t)(Nmax > 0 ? Nmax : 1);
    char *ws = (char *)workspace(8, sizeof(double) * 3 * (size_t)P * nm + 64);
    PCR_REQUIRE(ws, PCR_ERR_NOMEM, "icp: %s", pcr_last_error());
    a.P3 = (double *)ws;
    a.cst = (int4 *)workspace(38, sizeof(int4) * (size_t)P * nm + 64);
    PCR_REQUIRE(a.cst, PCR_ERR_NOMEM, "icp: %s", pcr_last_error());
    bool *icp_dirty = nullptr;
    if (a.G > 1 || two_phase) {
        const int gp = two_phase ? a.gmax2 : a.G;  // partial slots per pair
        char *cw = (char *)workspace(10, sizeof(XPart) * 2 * (size_t)gp * (size_t)P + 64);
        PCR_REQUIRE(cw, PCR_ERR_NOMEM, "icp: %s", pcr_last_error());
        a.part = (XPart *)cw;
        // barriers in a slot of their own, zeroed when allocated: every launch
        // leaves the arrivals zero (a barrier resets them) and the barrier
        // works from any generation, so no memset per call; the
        // (pair, 4) layout does not move with P, and a power-of-two size either
        // fits the zeroed range or outgrows the slot's headroom (fresh, zeroed)
        size_t nb = 16384;
        while (nb < 4 * (size_t)P) nb <<= 1;
        // A launch that failed after some of its workgroups arrived could leave
        // arrivals behind: the call after any failed one in this (device,
        // context) re-zeroes.
        bool fresh = false;
        a.bar = (unsigned *)workspace(39, sizeof(unsigned) * nb, &fresh);
        PCR_REQUIRE(a.bar, PCR_ERR_NOMEM, "icp: %s", pcr_last_error());
        // the slot's dirty flag (per device and workspace context, as the slot
        // itself) is set while a call's launches are being issued: a call that
        // returned an error in between leaves it set for the next one here
        icp_dirty = workspace_dirty(39);
        PCR_REQUIRE(icp_dirty, PCR_ERR_ARG, "icp: no workspace slot");
        if (fresh || *icp_dirty) PCR_HIP_CHECK(hipMemsetAsync(a.bar, 0, sizeof(unsigned) * nb, s));
        *icp_dirty = false;
    } else {
        a.part = nullptr;
        a.bar = nullptr;
    }
    a.timing = nullptr;
    const bool want_timing = getenv("PCR_ICP_TIMING") != nullptr;
    if (want_timing) {
        a.timing = (unsigned long long *)workspace(12, sizeof(unsigned long long) * 12 * (size_t)P);
        PCR_REQUIRE(a.timing, PCR_ERR_NOMEM, "icp timing: %s", pcr_last_error());
        PCR_HIP_CHECK(hipMemsetAsync(a.timing, 0, sizeof(unsigned long long) * 12 * (size_t)P, s));
    }
    if (two_phase) {
        char *tw = (char *)workspace(37, sizeof(int) * (2 + (size_t)P) + sizeof(double) * kSave * (size_t)P + 64);
        PCR_REQUIRE(tw, PCR_ERR_NOMEM, "icp: %s", pcr_last_error());
        a.save = (double *)tw;
        a.ctl = (int *)(a.save + kSave * (size_t)P);
        a.list = a.ctl + 2;
        PCR_HIP_CHECK(hipMemsetD32Async(a.ctl, P, 1, s));       // pairs iterating
        PCR_HIP_CHECK(hipMemsetAsync(a.ctl + 1, 0, sizeof(int), s));  // none listed
    }
    prof_begin(s, kProfIcp);
    if (icp_dirty) *icp_dirty = true;  // until every launch below went in
    if (!two_phase) {
        void *args[] = {&a};
        PCR_HIP_CHECK(coop_launch(fn, P, a.G, kThreads, args, sm, s));
        PCR_LAUNCH_CHECK();
    } else {
        a.phase = 1;
        {
            void *args[] = {&a};
            PCR_HIP_CHECK(coop_launch(fn, P, 1, kThreads, args, sm, s));  // one workgroup per pair
            PCR_LAUNCH_CHECK();
        }
        a.phase = 2;
        a.G = 0;  // from the listed count, on the device
        void *args[] = {&a};
        PCR_HIP_CHECK(hipLaunchCooperativeKernel(fn, dim3(grid2), dim3(kThreads), args, (unsigned)sm, s));
        PCR_LAUNCH_CHECK();
    }
    if (icp_dirty) *icp_dirty = false;
    prof_end(s, kProfIcp);
    if (want_timing) {  // debug: phase split in shader clocks, mean over pairs, to stderr
        std::vector<unsigned long long> h(12 * (size_t)P);
        PCR_HIP_CHECK(hipMemcpyAsync(h.data(), a.timing, h.size() * 8, hipMemcpyDeviceToHost, s));
        PCR_HIP_CHECK(hipStreamSynchronize(s));
        double m[11] = {};
        for (int q = 0; q < P; ++q)
            for (int k = 0; k < 11; ++k) m[k] += (double)h[12 * q + k] / P;
        fprintf(stderr, "icp timing (clocks, mean over %d pairs, G=%d): chunks %.0f drain %.0f park %.0f join %.0f "
                "pair-barrier %.0f partials %.0f means %.0f horn %.0f total %.0f iters %.2f walks (workgroup 0) %.0f\n",
                P, a.G, m[7], m[0], m[4], m[5], m[6], m[1], m[2], m[3], m[8], m[9], m[10]);
    }
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
                         fitness_rmse, stats, corr_tgt, pcr::as_stream(stream), nullptr, nullptr, nullptr);
}
