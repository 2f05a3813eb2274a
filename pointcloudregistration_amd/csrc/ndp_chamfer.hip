// f4: the Chamfer pass of an NDP level iteration (registration.py:231-244 on
// pytorch3d's knn_points; the nnd drop-in's contract, a1/a2) with its
// gradient, specialised for the level loop:
//
//   * the target does not move during the optimisation: its grid is built once
//     (pcr_ndp_chamfer_prepare) and every iteration only rebuilds the grid of
//     the warped subset xs, with a cell fixed per level (the cell size only
//     changes the work, never the answer);
//   * the subset grid is a three-launch counting sort over all CUs (count,
//     scan, scatter; a single-pair cloud in one workgroup took 35-63 us);
//   * queries of both directions in one launch, LPQ lanes per query, the ring
//     walk of nng.h; a query not certified within kmax rings is listed and
//     answered by nc_fallback, an exact scan of the other cloud spread over
//     the whole chip (blocks of 64 listed queries x 2,048-candidate slices,
//     16 queries per wave against each LDS-staged candidate, the slices' (d, j)
//     minima combined by 64-bit atomicMin on (d bits, j): d >= 0, so that is
//     the lexicographic minimum) -- the far target points of a partially
//     overlapping pair (36 % of the C5 target) had made every wave of the
//     general kernel run a whole-cloud scan (428 us per C5 iteration);
//   * the gradient dL/dxs is accumulated in the same epilogue: query i of the
//     subset adds 2 gd1 (x_i - y_j), query k of the target subtracts
//     2 gd2 (y_k - x_i) at its answer i, each taken exactly to a two-word fixed
//     point and added with integer atomics (exact and order-free: the same bits
//     on every replay), gd = 1/K, 1/M where d < trunc (else 0) as
//     pcr_ndp_chamfer_glue.  The scale follows the data (round 4): per
//     iteration, from the subset's and the target's largest finite |coordinate|
//     A_s, A_t, every finite term is at most T = 2 max(gd) (A_s + A_t), and an
//     entry sums at most M + 1 of them, so with 2^s <= 2^60 / ((M + 2) T) no
//     integer sum can overflow; a term v goes in as hi = rint(v 2^s) plus
//     lo = rint((v 2^s - hi) 2^40), i.e. with a quantum 2^-(s+40) (~1e-29 at
//     the C5 level's s = 57) -- relative precision for any term that matters,
//     at unit or millimetre scale alike.  Only a non-finite term sets the flag
//     (the gradient is then NaN, as the reference's would be);
//     pcr_ndp_train_backward reads the sums.  This replaces the five-launch
//     deterministic bucket backward of pcr_nnd_backward (~110 us per C5
//     iteration).  Distances and indices are those of pcr_nnd_forward bit for
//     bit; the gradient differs from the CPU-order f32 sums of
//     pcr_nnd_backward by its rounding (f32 contributions, exact sums).
//
// Non-finite or out-of-range points (no integer cell coordinates) switch the
// iteration to the reference loop (seed with candidate 0, strict <) as
// nnd_grid.hip does.
//
// Round 4, the default (PCR_NC_BOX=1): the grid path above is replaced by a
// box path -- each cloud in a spatial order fixed at prepare, 32-point leaves
// and 1024-point groups with their bounding boxes; per iteration one launch
// rewrites the subset's points and boxes (nc_leaves) and one answers both
// directions (nc_bquery), each query's search bounded by the distance to its
// previous answer (the level loop moves points a little per iteration, and the
// level's first iteration starts from the previous level's answers).  A box
// bound is d2f's own roundings on the axis gaps, so it is a true lower bound of
// every computed distance inside (monotone rounding): a box above the bound
// cannot hold the answer or a tie, and the result is the exact lexicographic
// (d, j) minimum -- the same bits as the grid path and pcr_nnd_forward -- from
// any starting index.  Four launches and the far-query list (count / scan /
// scatter, walk, fallback, emit) become two.
constexpr bool kNcSkip = false;  // ring_walk's per-cell bounds (nng.h): off for the level Chamfer (measured equal)
#include "pcr_internal.h"
#include "nng.h"
#include "scan.h"
#include <algorithm>
#include <cstdlib>

namespace pcr {
namespace {

using nng::ccoord;
using nng::d2f;
using nng::nhash;
using nng::take;

constexpr int kRep = PCR_NDP_GACC_REPLICAS;     // gradient sum replicas (query index mod kRep)
constexpr int kFbQW = 16;                       // nc_fallback: listed queries per wave (8 packed pairs)
constexpr int kFbQ = 4 * kFbQW, kFbSlice = 1024;  // work item: listed queries x candidates
constexpr int kFbBlocks = 2048;                 // nc_fallback: persistent 256-thread blocks

struct NcHdr {
    float cell_t, cell_s;
    int tflag;      // target non-finite / out of cell range: reference loop for the level
    int sflag;      // subset non-finite / out of range this iteration (nc_count)
    int mode;       // sflag | tflag as nc_scan saw it (read by the queries)
    int fb_cnt[2];  // listed (uncertified) queries per direction
    int pad;
    unsigned amax_t;  // the target's largest finite |coordinate| (f32 bits), prepare
    unsigned amax_s;  // the subset's, this iteration (nc_count; nc_scan consumes and clears)
    int shift;        // this iteration's fixed-point exponent s (nc_scan)
    int pad2;
    long long reserved0;  // (layout kept: the diagnostics below sit at byte 64)
    unsigned reserved1;
    int pad3;
    unsigned long long st[3];  // box path diagnostics (PCR_NC_STATS=1): queries, groups, leaves scanned
    unsigned samax[32];        // box path: per subset group, its largest finite |coordinate| (nc_leaves)
    int sbad[32];              //   and whether it holds a non-finite coordinate
};

// ---- the box path (default; PCR_NC_BOX=0 selects the grid path above) ------
// Each cloud in a fixed spatial (Morton) order, cut into leaves of kLeaf
// consecutive points and groups of kGrp leaves, each with its f32 bounding box.
// The target's order and boxes are built once (prepare); the subset keeps the
// order of its level's starting positions and only its points and boxes are
// rewritten per iteration (nc_leaves: one launch instead of count / scan /
// scatter).  A box moving with its points stays exact -- it is recomputed from
// the current coordinates -- only its tightness depends on the order.
constexpr int kLeaf = 32, kGrp = 32;  // points per leaf, leaves per group (= one 1024-thread block)
constexpr int kOrdBits5 = 5, kOrdN = 1 << (3 * kOrdBits5);  // 32^3 Morton buckets of the bounding box

struct NcBox {
    float4 lo, hi;  // .w unused
};

struct NcTree {
    int n, L, G;      // points, leaves, groups
    int *ord;         // position -> original index (prepare)
    float4 *pts;      // n points in that order: (x, y, z, index bits)
    NcBox *leaf;      // L
    NcBox *grp;       // G
};

// one cloud's hashed grid (nng.h)
struct NcCloud {
    int S;
    int *start;   // S + 1
    float4 *pts;  // n: (x, y, z, index bits) sorted by slot
};

struct NcArgs {
    const float *xs, *tgt;  // (K, 3), (M, 3)
    int K, M, St, Ss, kmax;
    NcCloud ct, cs;         // target, subset
    float trunc, g1, g2;    // g1 = 1/K, g2 = 1/M (as the glue)
    float *d1, *d2;
    int32_t *i1, *i2;
    long long *gacc;        // [0]: bit 0 non-finite term, bits 8..: s + 2048; [1 + 3 (r K + k) + c]:
                            // replica r of dL/dxs[k][c] hi words (2^-s), [1 + 3 K R + ...] lo words
                            // (2^-(s+40)) (pcr_ndp_train_backward sums the replicas)
    NcHdr *hdr;
    int fshift;             // diagnostics (PCR_NDP_FIXSHIFT): a fixed exponent, hi words only
                            // (round 3's 2^-44 quantum at 44); -1: the data-scaled two words
    int *cnt;               // counting-sort counts, zero between builds
    int *fb;                // K + M: listed queries (dir 0 at 0, dir 1 at K)
    unsigned long long *fbkey;  // K + M: their (d bits, j) minima
    const double *gate;
    bool box;               // the box path (PCR_NC_BOX, default on)
    bool stats;             // PCR_NC_STATS: count the groups / leaves the queries scan
    NcTree bt, bs;          // its target / subset trees
};

__device__ __forceinline__ bool cell_ok(float x, float y, float z, double ic) {
    return __builtin_isfinite(x) && __builtin_isfinite(y) && __builtin_isfinite(z) &&
           fabs((double)x * ic) < 1e9 && fabs((double)y * ic) < 1e9 && fabs((double)z * ic) < 1e9;
}

// cell = 0.6 cbrt(bbox volume / n) of one cloud (nng_bbox's rule); flag on a
// non-finite point.  One workgroup.
__global__ __launch_bounds__(1024) void nc_bbox(const float *P, int n, float *cell, int *flag,
                                                unsigned *amax) {
    const int t = threadIdx.x;
    float lo[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
    float hi[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    int bad = 0;
    float am = 0.0f;  // largest finite |coordinate|
    for (int i = t; i < n; i += 1024)
        for (int c = 0; c < 3; ++c) {
            const float v = P[3 * i + c];
            bad |= !__builtin_isfinite(v);
            lo[c] = fminf(lo[c], v);
            hi[c] = fmaxf(hi[c], v);
            if (__builtin_isfinite(v)) am = fmaxf(am, fabsf(v));
        }
    if (amax) {
        for (int o = 32; o; o >>= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
        if ((t & 63) == 0) atomicMax(amax, __float_as_uint(am));  // >= 0: bits order as values
    }
    __shared__ float sl[3][16], sh[3][16];
    __shared__ int sb[16];
    for (int c = 0; c < 3; ++c)
        for (int o = 32; o; o >>= 1) {
            lo[c] = fminf(lo[c], __shfl_xor(lo[c], o, 64));
            hi[c] = fmaxf(hi[c], __shfl_xor(hi[c], o, 64));
        }
    for (int o = 32; o; o >>= 1) bad |= __shfl_xor(bad, o, 64);
    if ((t & 63) == 0) {
        for (int c = 0; c < 3; ++c) { sl[c][t >> 6] = lo[c]; sh[c][t >> 6] = hi[c]; }
        sb[t >> 6] = bad;
    }
    __syncthreads();
    if (t != 0) return;
    double e[3], m = 0.0;
    for (int c = 0; c < 3; ++c) {
        float l = sl[c][0], h = sh[c][0];
        for (int w = 1; w < 16; ++w) { l = fminf(l, sl[c][w]); h = fmaxf(h, sh[c][w]); }
        e[c] = (double)h - (double)l;
        m = fmax(m, e[c]);
    }
    bad = 0;
    for (int w = 0; w < 16; ++w) bad |= sb[w];
    double cl = 1.0;
    if (m > 0.0 && m < 1e300) {
        double v = 1.0;
        for (int c = 0; c < 3; ++c) v *= fmax(e[c], 1e-3 * m);
        cl = 0.6 * cbrt(v / (double)(n > 0 ? n : 1));
    }
    *cell = (float)cl;
    if (flag && bad) *flag = 1;
}

// counting sort of one cloud by hash slot: count (optionally zeroing the
// gradient sums of the subset), scan, scatter.  cnt is all-zero before count
// and after scatter (scatter counts down).
__global__ void nc_count(const float *P, int n, const float *cellp, NcCloud g, int *cnt, int *flag,
                         long long *gacc, unsigned *amax, const double *gate) {
    if (gated_off(gate)) return;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float am = 0.0f;
    bool ok = false;
    float x = 0.f, y = 0.f, z = 0.f;
    double ic = 1.0;
    if (i < n) {
        if (gacc)
#pragma unroll
            for (int r = 0; r < kRep; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    gacc[1 + 3 * ((size_t)r * n + i) + c] = 0;                      // hi words
                    gacc[1 + 3 * ((size_t)kRep * n + (size_t)r * n + i) + c] = 0;   // lo words
                }
        x = P[3 * i]; y = P[3 * i + 1]; z = P[3 * i + 2];
        ic = 1.0 / (double)*cellp;
        ok = cell_ok(x, y, z, ic);
        if (!ok) atomicOr(flag, 1);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float v = c == 0 ? x : (c == 1 ? y : z);
            if (__builtin_isfinite(v)) am = fmaxf(am, fabsf(v));
        }
    }
    if (amax) {  // the subset's largest finite |coordinate|, one atomic per wave
        for (int o = 32; o; o >>= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
        if ((threadIdx.x & 63) == 0 && am > 0.0f) atomicMax(amax, __float_as_uint(am));
    }
    if (ok) atomicAdd(cnt + nhash(ccoord(x, ic), ccoord(y, ic), ccoord(z, ic), g.S), 1);
}

// one workgroup: starts of the subset (or target) grid; the per-iteration
// resets (mode, listed counts, the gradient's non-finite flag) ride along
// (the counts are staged through LDS with coalesced loads: the span scan's
// strided global reads took ~19 us for 16K slots)
constexpr int kScanLds = 32768;

// the fixed-point exponent of this iteration (header comment): every finite
// term <= T = 2 gmax (A_s + A_t), an entry sums <= M + 1 of them
__device__ inline int nc_shift_of(float amax_s, float amax_t, float gmax, int Mq, int fshift) {
    const double T = 2.0 * (double)gmax * ((double)amax_s + (double)amax_t) * (1.0 + 0x1p-20);
    const double B = (double)(Mq + 2) * T;
    int sh = 60;
    if (B > 0.0 && __builtin_isfinite(B)) sh = 59 - ilogb(B);  // B < 2^(ilogb+1): B 2^s < 2^60
    sh = sh < -900 ? -900 : (sh > 900 ? 900 : sh);
    if (fshift >= 0) sh = 1000 + fshift;  // marks "hi words only" for fix_add
    return sh;
}

__device__ inline int nc_shift(const NcHdr *h, float gmax, int Mq, int fshift) {
    return nc_shift_of(__uint_as_float(h->amax_s), __uint_as_float(h->amax_t), gmax, Mq, fshift);
}

__global__ __launch_bounds__(1024) void nc_scan(const int *cnt, NcCloud g, NcHdr *h, long long *gacc,
                                                float gmax, int Mq, int fshift, const double *gate) {
    if (gated_off(gate)) return;
    // LDS index i + i / 16: thread t's span [t per, (t+1) per) starts 17 t words
    // apart at per = 16 (no bank conflicts; the plain layout was 16-way)
    extern __shared__ int lds[];  // (S + 1) * 17 / 16
    __shared__ int wtot[16];
    auto P = [](int i) { return i + (i >> 4); };
    const int S = g.S, t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (int i = t; i < S; i += 1024) lds[P(i)] = cnt[i];
    __syncthreads();
    const int per = (S + 1023) >> 10;
    const int b0 = min(S, t * per), b1 = min(S, b0 + per);
    int v = 0;
    for (int i = b0; i < b1; ++i) v += lds[P(i)];
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wtot[w] = x;
    __syncthreads();
    if (t == 0) {
        int acc = 0;
        for (int k = 0; k < 16; ++k) { const int c = wtot[k]; wtot[k] = acc; acc += c; }
        lds[P(S)] = acc;
    }
    __syncthreads();
    int run = wtot[w] + x - v;
    for (int i = b0; i < b1; ++i) { const int c = lds[P(i)]; lds[P(i)] = run; run += c; }
    __syncthreads();
    for (int i = t; i <= S; i += 1024) g.start[i] = lds[P(i)];
    if (threadIdx.x == 0 && gacc) {
        h->mode = h->sflag | h->tflag;
        h->sflag = 0;
        h->fb_cnt[0] = 0;
        h->fb_cnt[1] = 0;
        // the fixed-point exponent of this iteration (header comment): every
        // finite term <= T = 2 gmax (A_s + A_t), an entry sums <= M + 1 of them
        const int sh = nc_shift(h, gmax, Mq, fshift);
        h->shift = sh;
        h->amax_s = 0u;
        gacc[0] = (long long)(sh + 2048) << 8;
    }
}

__global__ void nc_scatter(const float *P, int n, const float *cellp, NcCloud g, int *cnt, const double *gate) {
    if (gated_off(gate)) return;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = P[3 * i], y = P[3 * i + 1], z = P[3 * i + 2];
    const double ic = 1.0 / (double)*cellp;
    if (!cell_ok(x, y, z, ic)) return;
    const unsigned hs = nhash(ccoord(x, ic), ccoord(y, ic), ccoord(z, ic), g.S);
    g.pts[g.start[hs] + atomicSub(cnt + hs, 1) - 1] = make_float4(x, y, z, __int_as_float(i));
}

// v exactly into the two words (hi at 2^-s, lo at 2^-(s+40)): t = v 2^s is exact
// (a power-of-two scale of an f32), hi = rint(t), t - hi is exact (|t - hi| <=
// 1/2), lo = rint((t - hi) 2^40); |hi| < 2^60 / (M + 2) by the choice of s
__device__ __forceinline__ void fix_add(long long *hi, long long *lo, float v, int sh, long long *flag) {
    if (!__builtin_isfinite(v)) {
        __hip_atomic_fetch_or(flag, 1LL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const bool hi_only = sh >= 1000;  // diagnostics: round 3's single word
    if (hi_only) sh -= 1000;
    const double t = __builtin_ldexp((double)v, sh);
    const double h = __builtin_rint(t);
    const double l = hi_only ? 0.0 : __builtin_rint((t - h) * 0x1p40);
    if (h != 0.0)
        __hip_atomic_fetch_add(hi, (long long)h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (l != 0.0)
        __hip_atomic_fetch_add(lo, (long long)l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the answer (best, bj) of query q in direction dir: outputs and gradient
// (pcr_nnd_backward's terms: g = gd * 2, grad1 += g (x - y), grad1[i] -= g (y - x)).
// The far target points of a partial overlap share a few boundary answers (up to
// ~350 terms on one subset point in C5): the terms go to replica q mod kRep, so
// same-address atomics stay short (integer sums: the replica split changes no bit)
__device__ __forceinline__ void emit(const NcArgs &a, int dir, int q, float best, int bj, int sh, long long *flag) {
    long long *rep = a.gacc + 1 + (size_t)(q & (kRep - 1)) * 3 * a.K;
    const size_t lo = (size_t)3 * kRep * a.K;  // lo words after all hi words
    if (dir == 0) {
        a.d1[q] = best;
        a.i1[q] = bj;
        const float g = (!(best >= a.trunc) ? a.g1 : 0.0f) * 2;
        if (bj < 0 || bj >= a.M) return;
        for (int c = 0; c < 3; ++c)
            fix_add(rep + 3 * q + c, rep + lo + 3 * q + c, g * (a.xs[3 * q + c] - a.tgt[3 * bj + c]), sh, flag);
    } else {
        a.d2[q] = best;
        a.i2[q] = bj;
        const float g = (!(best >= a.trunc) ? a.g2 : 0.0f) * 2;
        if (bj < 0 || bj >= a.K) return;
        for (int c = 0; c < 3; ++c)
            fix_add(rep + 3 * bj + c, rep + lo + 3 * bj + c, -(g * (a.tgt[3 * q + c] - a.xs[3 * bj + c])), sh,
                    flag);
    }
}

// both directions: blocks [0, nb0) query the subset against the target grid,
// the rest the target against the subset grid; queries in their own grid's
// slot order (lanes of a wave walk neighbouring cells)
template <int LPQ>
__global__ __launch_bounds__(256) void nc_query(NcArgs a, int nb0) {
    if (gated_off(a.gate)) return;
    constexpr int QPB = 256 / LPQ;
    const int dir = blockIdx.x < nb0 ? 0 : 1;
    const int qslot = (blockIdx.x - (dir ? nb0 : 0)) * QPB + threadIdx.x / LPQ;
    const int sub = threadIdx.x % LPQ;
    const int nq = dir ? a.M : a.K, nc = dir ? a.K : a.M;
    if (qslot >= nq) return;  // a query's lanes leave together
    const bool brute = a.hdr->mode != 0;
    const int sh = a.hdr->shift;
    const float *Q = dir ? a.tgt : a.xs;
    const float *C = dir ? a.xs : a.tgt;
    int qi = qslot;
    float qx, qy, qz;
    if (brute) {
        qx = Q[3 * qi]; qy = Q[3 * qi + 1]; qz = Q[3 * qi + 2];
    } else {
        const float4 qp = (dir ? a.ct.pts : a.cs.pts)[qslot];
        qx = qp.x; qy = qp.y; qz = qp.z;
        qi = __float_as_int(qp.w);
    }
    float best = __builtin_inff();
    int bj = 0x7fffffff;
    if (brute) {
        // the reference loop: seed with candidate 0, strict < (my_lib.cpp:11-20)
        if (sub != 0) return;
        best = d2f(C[0], C[1], C[2], qx, qy, qz);
        bj = 0;
        for (int j = 1; j < nc; ++j) {
            const float d = d2f(C[3 * j], C[3 * j + 1], C[3 * j + 2], qx, qy, qz);
            if (d < best) { best = d; bj = j; }
        }
        emit(a, dir, qi, best, bj, sh, a.gacc);
        return;
    }
    const nng::View v = dir ? nng::View{a.hdr->cell_s, a.cs.S, a.cs.start, a.cs.pts}
                            : nng::View{a.hdr->cell_t, a.ct.S, a.ct.start, a.ct.pts};
    const bool done = nng::ring_walk<LPQ, kNcSkip>(v, qx, qy, qz, sub, a.kmax, best, bj);
    // listed queries appended with one atomic per wave (thousands of far
    // queries on one counter serialised at the L2); a wave holds one direction
    const bool list = !done && sub == 0;
    const unsigned long long bal = __ballot(list);
    if (bal) {
        const int lane = threadIdx.x & 63;
        int base = 0;
        if (lane == __ffsll((long long)bal) - 1) base = atomicAdd(&a.hdr->fb_cnt[dir], __popcll(bal));
        base = __shfl(base, __ffsll((long long)bal) - 1, 64);
        if (list) {
            const int e = (dir ? a.K : 0) + base + __popcll(bal & ((1ULL << lane) - 1));
            a.fb[e] = qi;
            a.fbkey[e] = ~0ULL;
        }
    }
    if (sub == 0 && done) emit(a, dir, qi, best, bj, sh, a.gacc);
}

// the listed queries: work item = (64 listed queries of one direction, a
// 1,024-candidate slice of the other cloud in index order), persistent blocks
// over all items.  The slice is staged in LDS; wave w holds queries
// 16w..16w+15 as eight packed pairs, lane l takes candidates l, l + 64, ...
// in increasing index, so a strict < keeps the lowest index of a tie (one
// compare and two selects per query, no mask arithmetic); the lanes merge
// lexicographically and each query's (d, j) minimum over the slice goes to
// its key by atomicMin.
typedef float f2v __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void nc_fallback(NcArgs a) {
    if (gated_off(a.gate)) return;
    __shared__ float4 tile[kFbSlice];
    const int c0 = a.hdr->fb_cnt[0], c1 = a.hdr->fb_cnt[1];
    const int g0 = (c0 + kFbQ - 1) / kFbQ, g1 = (c1 + kFbQ - 1) / kFbQ;
    const int s0 = (a.M + kFbSlice - 1) / kFbSlice, s1 = (a.K + kFbSlice - 1) / kFbSlice;
    const int n0 = g0 * s0, total = n0 + g1 * s1;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr int H = kFbQW / 2;
    for (int it = blockIdx.x; it < total; it += gridDim.x) {
        const int dir = it < n0 ? 0 : 1;
        const int r = dir ? it - n0 : it, ns = dir ? s1 : s0;
        const int grp = r / ns, sl = r - grp * ns;
        const int cnt = dir ? c1 : c0, nc = dir ? a.K : a.M;
        const float *Q = dir ? a.tgt : a.xs;
        const float *C = dir ? a.xs : a.tgt;
        const int lbase = (dir ? a.K : 0) + grp * kFbQ;
        const int qn = min(kFbQ, cnt - grp * kFbQ);
        const int t0 = sl * kFbSlice, tn = min(kFbSlice, nc - t0);
        __syncthreads();  // the previous item's tile is consumed
        for (int c = threadIdx.x; c < tn; c += 256) {
            const float *cp = C + 3 * (size_t)(t0 + c);
            tile[c] = make_float4(cp[0], cp[1], cp[2], 0.0f);
        }
        __syncthreads();
        if (wv * kFbQW >= qn) continue;  // no listed query for this wave (barriers are above)
        f2v qx[H], qy[H], qz[H], best[H];
        int bj[kFbQW];
#pragma unroll
        for (int u = 0; u < kFbQW; ++u) {
            const int e = wv * kFbQW + u;
            const int q = e < qn ? a.fb[lbase + e] : a.fb[lbase];
            qx[u >> 1][u & 1] = Q[3 * q];
            qy[u >> 1][u & 1] = Q[3 * q + 1];
            qz[u >> 1][u & 1] = Q[3 * q + 2];
            best[u >> 1][u & 1] = __builtin_inff();
            bj[u] = 0x7fffffff;
        }
        // the lane's first candidate seeds its minima (so a d = inf still names an index)
        if (lane < tn) {
            const float4 p = tile[lane];
            const f2v px = {p.x, p.x}, py = {p.y, p.y}, pz = {p.z, p.z};
#pragma unroll
            for (int h = 0; h < H; ++h) {
                const f2v dx = px - qx[h], dy = py - qy[h], dz = pz - qz[h];
                best[h] = (dx * dx + dy * dy) + dz * dz;
                bj[2 * h] = bj[2 * h + 1] = t0 + lane;
            }
        }
#pragma unroll 2
        for (int c = lane + 64; c < tn; c += 64) {
            const float4 p = tile[c];
            const int j = t0 + c;
            const f2v px = {p.x, p.x}, py = {p.y, p.y}, pz = {p.z, p.z};
#pragma unroll
            for (int h = 0; h < H; ++h) {
                const f2v dx = px - qx[h], dy = py - qy[h], dz = pz - qz[h];
                const f2v d = (dx * dx + dy * dy) + dz * dz;  // d2f's roundings, two queries at once
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    const bool lt = d[b] < best[h][b];
                    best[h][b] = lt ? d[b] : best[h][b];
                    bj[2 * h + b] = lt ? j : bj[2 * h + b];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kFbQW; ++u) {
            float bb = best[u >> 1][u & 1];
            int jj = bj[u];
#pragma unroll
            for (int o = 32; o; o >>= 1) {
                const float ob = __shfl_xor(bb, o, 64);
                const int oj = __shfl_xor(jj, o, 64);
                nng::take_sel(ob, oj, bb, jj);
            }
            const int e = wv * kFbQW + u;
            if (lane == u && e < qn && jj != 0x7fffffff)
                atomicMin(a.fbkey + lbase + e, ((unsigned long long)__float_as_uint(bb) << 32) | (unsigned)jj);
        }
    }
}

// the listed queries' answers from their keys
__global__ __launch_bounds__(256) void nc_fallback_emit(NcArgs a) {
    if (gated_off(a.gate)) return;
    const int c0 = a.hdr->fb_cnt[0], c1 = a.hdr->fb_cnt[1];
    const int w = blockIdx.x * 256 + threadIdx.x;
    if (w >= c0 + c1) return;
    const int dir = w < c0 ? 0 : 1;
    const int e = dir ? a.K + (w - c0) : w;
    const unsigned long long k = a.fbkey[e];
    emit(a, dir, a.fb[e], __uint_as_float((unsigned)(k >> 32)), (int)(unsigned)(k & 0xffffffffu),
         a.hdr->shift, a.gacc);
}

// ---- box path kernels --------------------------------------------------------
__device__ __forceinline__ unsigned spread5(unsigned v) {  // 5 bits -> every third bit
    v &= 31u;
    v = (v | (v << 8)) & 0x0000F00Fu;
    v = (v | (v << 4)) & 0x000C30C3u;
    v = (v | (v << 2)) & 0x00249249u;
    return v;
}

// prepare: a spatial order of one cloud (one 1024-thread workgroup): Morton
// code of the point's bucket in a 32^3 division of the finite bounding box,
// counting sort in LDS (order inside a bucket: atomic order -- it only changes
// how tight the boxes are, never an answer)
__global__ __launch_bounds__(1024) void nc_order(const float *P, int n, int *ord) {
    extern __shared__ int bk[];  // kOrdN + 1
    __shared__ float sl[3][16], sh[3][16];
    __shared__ float lo_s[3], sc_s[3];
    const int t = threadIdx.x;
    float lo[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
    float hi[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    for (int i = t; i < n; i += 1024)
        for (int c = 0; c < 3; ++c) {
            const float v = P[3 * i + c];
            if (__builtin_isfinite(v)) { lo[c] = fminf(lo[c], v); hi[c] = fmaxf(hi[c], v); }
        }
    for (int c = 0; c < 3; ++c) {
        for (int o = 32; o; o >>= 1) {
            lo[c] = fminf(lo[c], __shfl_xor(lo[c], o, 64));
            hi[c] = fmaxf(hi[c], __shfl_xor(hi[c], o, 64));
        }
        if ((t & 63) == 0) { sl[c][t >> 6] = lo[c]; sh[c][t >> 6] = hi[c]; }
    }
    for (int i = t; i < kOrdN; i += 1024) bk[i] = 0;
    __syncthreads();
    if (t < 3) {
        float l = sl[t][0], h = sh[t][0];
        for (int w = 1; w < 16; ++w) { l = fminf(l, sl[t][w]); h = fmaxf(h, sh[t][w]); }
        const double e = (double)h - (double)l;
        lo_s[t] = l;
        sc_s[t] = (e > 0.0 && e < 1e300) ? (float)(32.0 / e) : 0.0f;
    }
    __syncthreads();
    auto key = [&](int i) -> unsigned {
        unsigned k = 0;
        for (int c = 0; c < 3; ++c) {
            const float v = (P[3 * i + c] - lo_s[c]) * sc_s[c];  // NaN / inf -> bucket 0 / 31
            const int q = v > 0.0f ? (v < 31.0f ? (int)v : 31) : 0;
            k |= spread5((unsigned)q) << c;
        }
        return k;
    };
    for (int i = t; i < n; i += 1024) atomicAdd(&bk[key(i)], 1);
    __syncthreads();
    block_exclusive_scan_1024(bk, bk, kOrdN, false);
    for (int i = t; i < n; i += 1024) ord[atomicAdd(&bk[key(i)], 1)] = i;
}

// one group per 1024-thread block: position k's point (original index ord[k])
// into pts[k], the boxes of its leaf (half a wave) and of its group; for the
// subset also the per-iteration duties of nc_count (zero the gradient words,
// the non-finite flag, the largest finite |coordinate|)
__global__ __launch_bounds__(1024) void nc_leaves(const float *P, NcTree g, int *flag, long long *gacc,
                                                  unsigned *amax, const double *gate) {
    if (gated_off(gate)) return;
    __shared__ NcBox lb[kGrp];
    __shared__ unsigned s_am[16];
    __shared__ int s_bad[16];
    const int t = threadIdx.x, k = blockIdx.x * 1024 + t;
    if (gacc) {  // the header word and the 6 kRep n gradient words, spread over every block
        const size_t nw = (size_t)6 * kRep * g.n + 1;
        for (size_t e = (size_t)k; e < nw; e += (size_t)gridDim.x * 1024) gacc[e] = 0;
    }
    if ((int)blockIdx.x >= g.G) return;  // zeroing-only blocks
    const bool v = k < g.n;
    float x = 0.f, y = 0.f, z = 0.f, am = 0.0f;
    float lo[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
    float hi[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    bool bad = false;
    if (v) {
        const int i = g.ord[k];
        x = P[3 * i]; y = P[3 * i + 1]; z = P[3 * i + 2];
        g.pts[k] = make_float4(x, y, z, __int_as_float(i));
        const float q[3] = {x, y, z};
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            if (__builtin_isfinite(q[c])) {
                am = fmaxf(am, fabsf(q[c]));
                lo[c] = q[c];
                hi[c] = q[c];
            } else {
                bad = true;
            }
        }
    }
    // per group: its largest finite |coordinate| and a non-finite flag, plain
    // stores into flag[b] / amax[b] (the query kernel reduces the G of them: no
    // atomics, nothing to reset between iterations)
    if (amax || flag) {
        for (int o = 32; o; o >>= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
        const bool wbad = __ballot(bad) != 0ull;
        if ((t & 63) == 0) { s_am[t >> 6] = __float_as_uint(am); s_bad[t >> 6] = wbad ? 1 : 0; }
    }
#pragma unroll
    for (int o = 16; o; o >>= 1)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            lo[c] = fminf(lo[c], __shfl_xor(lo[c], o, 64));
            hi[c] = fmaxf(hi[c], __shfl_xor(hi[c], o, 64));
        }
    const int leaf = k >> 5;
    if ((t & 31) == 0) {
        const NcBox b{make_float4(lo[0], lo[1], lo[2], 0.f), make_float4(hi[0], hi[1], hi[2], 0.f)};
        lb[t >> 5] = b;
        if (leaf < g.L) g.leaf[leaf] = b;
    }
    __syncthreads();
    if (t < 32) {
        const NcBox b = lb[t];
        float l[3] = {b.lo.x, b.lo.y, b.lo.z}, h[3] = {b.hi.x, b.hi.y, b.hi.z};
#pragma unroll
        for (int o = 16; o; o >>= 1)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                l[c] = fminf(l[c], __shfl_xor(l[c], o, 64));
                h[c] = fmaxf(h[c], __shfl_xor(h[c], o, 64));
            }
        if (t == 0) g.grp[blockIdx.x] = NcBox{make_float4(l[0], l[1], l[2], 0.f), make_float4(h[0], h[1], h[2], 0.f)};
        if (t == 0 && (amax || flag)) {
            unsigned m = 0u;
            int b = 0;
            for (int w = 0; w < 16; ++w) { m = max(m, s_am[w]); b |= s_bad[w]; }  // >= 0: bits order as values
            if (amax) amax[blockIdx.x] = m;
            if (flag) flag[blockIdx.x] = b;
        }
    }
}

// lower bound of d2f over a box: the same roundings as d2f on the per-axis gap
// (rounding is monotone, so every point c of the box has fl(c - q)^2 terms at
// least these, and its computed distance is >= the bound; exact, no margin)
__device__ __forceinline__ float box_lb(const NcBox &b, float qx, float qy, float qz) {
    const float gx = fmaxf(fmaxf(b.lo.x - qx, qx - b.hi.x), 0.0f);
    const float gy = fmaxf(fmaxf(b.lo.y - qy, qy - b.hi.y), 0.0f);
    const float gz = fmaxf(fmaxf(b.lo.z - qz, qz - b.hi.z), 0.0f);
    return (gx * gx + gy * gy) + gz * gz;
}

// LPQ lanes per query, 64 / LPQ queries per wave, both directions (blocks
// [0, nb0): the subset against the target, the rest the target against the
// subset), queries in their cloud's spatial order.  U = the distance to the
// query's answer of the previous call (i1 / i2: any index in range is a valid
// start, so the first call of a level is exact too, only slower) bounds the
// answer: a group, then a leaf, whose box bound exceeds U is skipped (its
// points cannot win or tie).  The query's lanes split the groups, OR their
// selections, split each selected group's leaves, and scan their selected
// leaves' points themselves; the lanes' (d, j) minima are merged
// lexicographically.  Nothing is reset between iterations: the subset's extent
// and non-finite flag arrive as nc_leaves' per-group partials (every block
// reduces them alike), nc_leaves zeroes the gradient header word, block 0 ORs
// the exponent into it and a non-finite term ORs bit 0.
template <int LPQ>
__global__ __launch_bounds__(256) void nc_bquery(NcArgs a, int nb0) {
    if (gated_off(a.gate)) return;
    constexpr int QPB = 256 / LPQ;
    // the candidate tree's group and leaf boxes, staged once per block (<= 33 KiB):
    // the box tests read LDS, so a query's chain of dependent global loads is its
    // start point and its leaves' points only
    extern __shared__ NcBox sbox[];  // [0, 32): groups, [32, 32 + L): leaves
    const int sub = threadIdx.x % LPQ;
    const int dir = blockIdx.x < nb0 ? 0 : 1;
    {
        const NcTree &Ct = dir ? a.bs : a.bt;
        const float4 *gsrc = reinterpret_cast<const float4 *>(Ct.grp);
        const float4 *lsrc = reinterpret_cast<const float4 *>(Ct.leaf);
        float4 *dst = reinterpret_cast<float4 *>(sbox);
        for (int i = threadIdx.x; i < 2 * Ct.G; i += 256) dst[i] = gsrc[i];
        for (int i = threadIdx.x; i < 2 * Ct.L; i += 256) dst[2 * kGrp + i] = lsrc[i];
        __syncthreads();
    }
    const int k = (blockIdx.x - (dir ? nb0 : 0)) * QPB + (int)threadIdx.x / LPQ;
    const int nq = dir ? a.M : a.K, nc = dir ? a.K : a.M;
    const NcHdr *h = a.hdr;
    // the subset's extent and non-finite flag from nc_leaves' per-group partials
    // (every block reduces the same values in the same order)
    unsigned amx = 0u;
    int sbad = 0;
    for (int b = 0; b < a.bs.G; ++b) { amx = max(amx, h->samax[b]); sbad |= h->sbad[b]; }
    const int sh = nc_shift_of(__uint_as_float(amx), __uint_as_float(h->amax_t), a.g1 > a.g2 ? a.g1 : a.g2, a.M,
                               a.fshift);
    // the gradient header word (nc_leaves zeroed it): the exponent, once; a
    // non-finite term ORs bit 0 into the same word (fix_add)
    if (blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_fetch_or(a.gacc, (long long)(sh + 2048) << 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float *C = dir ? a.xs : a.tgt;
    if (k < nq) {
        if ((sbad | h->tflag) != 0) {
            // the reference loop: seed with candidate 0, strict < (my_lib.cpp:11-20)
            if (sub == 0) {
                const float *Q = dir ? a.tgt : a.xs;
                const float qx = Q[3 * k], qy = Q[3 * k + 1], qz = Q[3 * k + 2];
                float best = d2f(C[0], C[1], C[2], qx, qy, qz);
                int bj = 0;
                for (int j = 1; j < nc; ++j) {
                    const float d = d2f(C[3 * j], C[3 * j + 1], C[3 * j + 2], qx, qy, qz);
                    if (d < best) { best = d; bj = j; }
                }
                emit(a, dir, k, best, bj, sh, a.gacc);
            }
        } else {
            const NcTree &Qt = dir ? a.bt : a.bs;
            const NcTree &Ct = dir ? a.bs : a.bt;
            const float4 qp = Qt.pts[k];
            const float qx = qp.x, qy = qp.y, qz = qp.z;
            const int qi = __float_as_int(qp.w);
            int jp = dir ? a.i2[qi] : a.i1[qi];
            jp = (jp >= 0 && jp < nc) ? jp : 0;
            const float U = d2f(C[3 * jp], C[3 * jp + 1], C[3 * jp + 2], qx, qy, qz);
            float best = U;
            int bj = jp;
            // The query's LPQ lanes share one list: lane sub tests groups (then the
            // leaves of two selected groups) sub, sub + LPQ, ...; the lanes OR their
            // bits, then take every selected leaf two at a time, lane sub loading its
            // points sub, sub + LPQ, ... of both (one round trip per two leaves)
            constexpr int PL = kGrp / LPQ;
            auto orq = [](unsigned m) {
#pragma unroll
                for (int o = 1; o < LPQ; o <<= 1) m |= __shfl_xor(m, o, 64);
                return m;
            };
            unsigned gm = 0;
#pragma unroll
            for (int t = 0; t < PL; ++t) {
                const int g = sub + LPQ * t;
                if (g < Ct.G && box_lb(sbox[g], qx, qy, qz) <= U) gm |= 1u << g;
            }
            gm = orq(gm);
            if (a.stats && sub == 0) {
                atomicAdd(&a.hdr->st[0], 1ull);
                atomicAdd(&a.hdr->st[1], (unsigned long long)__popc(gm));
            }
            while (gm) {
                const int ga = __ffs((int)gm) - 1;
                gm &= gm - 1;
                int gb = -1;
                if (gm) {
                    gb = __ffs((int)gm) - 1;
                    gm &= gm - 1;
                }
                unsigned la = 0, lb = 0;
#pragma unroll
                for (int t = 0; t < PL; ++t) {
                    const int i = sub + LPQ * t;
                    const int fa = ga * kGrp + i, fb = gb * kGrp + i;
                    if (fa < Ct.L && box_lb(sbox[kGrp + fa], qx, qy, qz) <= U) la |= 1u << i;
                    if (gb >= 0 && fb < Ct.L && box_lb(sbox[kGrp + fb], qx, qy, qz) <= U) lb |= 1u << i;
                }
                unsigned long long lm = (unsigned long long)orq(la) | ((unsigned long long)orq(lb) << 32);
                if (a.stats && sub == 0) atomicAdd(&a.hdr->st[2], (unsigned long long)__popcll(lm));
                while (lm) {
                    const int b0 = __ffsll((long long)lm) - 1;
                    lm &= lm - 1;
                    int b1 = -1;
                    if (lm) {
                        b1 = __ffsll((long long)lm) - 1;
                        lm &= lm - 1;
                    }
                    const int l0 = (b0 < 32 ? ga : gb) * kGrp + (b0 & 31);
                    const int l1 = b1 < 0 ? -1 : (b1 < 32 ? ga : gb) * kGrp + (b1 & 31);
                    float4 p[2 * PL];
                    bool ok[2 * PL];
#pragma unroll
                    for (int v = 0; v < 2 * PL; ++v) {
                        const int lf = v < PL ? l0 : l1;
                        const int pos = lf * kLeaf + sub + LPQ * (v % PL);
                        ok[v] = lf >= 0 && pos < Ct.n;
                        if (ok[v]) p[v] = Ct.pts[pos];
                    }
#pragma unroll
                    for (int v = 0; v < 2 * PL; ++v)
                        if (ok[v]) take(d2f(p[v].x, p[v].y, p[v].z, qx, qy, qz), __float_as_int(p[v].w), best, bj);
                }
            }
#pragma unroll
            for (int o = 1; o < LPQ; o <<= 1) {
                const float ob = __shfl_xor(best, o, 64);
                const int oj = __shfl_xor(bj, o, 64);
                take(ob, oj, best, bj);
            }
            if (sub == 0) emit(a, dir, qi, best, bj, sh, a.gacc);
        }
    }
}

// the scan's dynamic LDS limit, set once outside any stream capture (prepare
// runs eagerly before a level graph is captured)
hipError_t nc_scan_attr() {
    static const hipError_t e = hipFuncSetAttribute((const void *)nc_scan, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                    (int)(sizeof(int) * (kScanLds + 2 + kScanLds / 16)));
    return e;
}

hipError_t nc_order_attr() {
    static const hipError_t e = hipFuncSetAttribute((const void *)nc_order, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                    (int)(sizeof(int) * (kOrdN + 1)));
    return e;
}

struct NcLayout {
    size_t hdr, cnt, fb, fbkey, total;
    size_t start[2], pts[2];  // [0] target, [1] subset
    int S[2];
    size_t ord[2], bpts[2], leaf[2], grp[2];  // the box path's trees
    int L[2], G[2];
};

inline int pow2_at_least(int n, int lo) {
    int S = lo;
    while (S < n) S <<= 1;
    return S;
}

inline size_t up256(size_t x) { return (x + 255) & ~(size_t)255; }

NcLayout nc_layout(int K, int M) {
    NcLayout L;
    const int n[2] = {M, K};
    size_t o = 0;
    L.hdr = o; o = up256(o + sizeof(NcHdr));
    for (int c = 0; c < 2; ++c) {
        L.S[c] = pow2_at_least(n[c], 256);
        L.start[c] = o; o = up256(o + sizeof(int) * ((size_t)L.S[c] + 1));
        L.pts[c] = o; o = up256(o + sizeof(float4) * (size_t)n[c]);
    }
    for (int c = 0; c < 2; ++c) {
        L.L[c] = (n[c] + kLeaf - 1) / kLeaf;
        L.G[c] = (L.L[c] + kGrp - 1) / kGrp;
        L.ord[c] = o; o = up256(o + sizeof(int) * (size_t)n[c]);
        L.bpts[c] = o; o = up256(o + sizeof(float4) * (size_t)n[c]);
        L.leaf[c] = o; o = up256(o + sizeof(NcBox) * (size_t)L.L[c]);
        L.grp[c] = o; o = up256(o + sizeof(NcBox) * (size_t)L.G[c]);
    }
    L.cnt = o; o = up256(o + sizeof(int) * (size_t)std::max(L.S[0], L.S[1]));
    L.fb = o; o = up256(o + sizeof(int) * ((size_t)K + M));
    L.fbkey = o; o = up256(o + sizeof(unsigned long long) * ((size_t)K + M));
    L.total = o;
    return L;
}

int nc_args(const pcr_ndp_chamfer *c, NcArgs &a) {
    PCR_REQUIRE(c, PCR_ERR_ARG, "ndp_chamfer: null descriptor");
    PCR_REQUIRE(c->K >= 1 && c->M >= 1, PCR_ERR_ARG, "ndp_chamfer: K=%d, M=%d (both >= 1)", c->K, c->M);
    PCR_REQUIRE(c->K <= kScanLds && c->M <= kScanLds, PCR_ERR_ARG,
                "ndp_chamfer: K=%d, M=%d (at most %d each)", c->K, c->M, kScanLds);
    PCR_REQUIRE(c->xs && c->tgt && c->d1 && c->d2 && c->i1 && c->i2 && c->gacc && c->scratch, PCR_ERR_ARG,
                "ndp_chamfer: null buffer");
    PCR_REQUIRE(((uintptr_t)c->scratch & 255) == 0, PCR_ERR_ARG, "ndp_chamfer: scratch not 256-byte aligned");
    const NcLayout L = nc_layout(c->K, c->M);
    char *s = (char *)c->scratch;
    a.xs = c->xs; a.tgt = c->tgt; a.K = c->K; a.M = c->M; a.St = L.S[0]; a.Ss = L.S[1];
    for (int k = 0; k < 2; ++k) {
        NcCloud &g = k ? a.cs : a.ct;
        g.S = L.S[k];
        g.start = (int *)(s + L.start[k]);
        g.pts = (float4 *)(s + L.pts[k]);
    }
    for (int k = 0; k < 2; ++k) {
        NcTree &t = k ? a.bs : a.bt;
        t.n = k ? c->K : c->M;
        t.L = L.L[k];
        t.G = L.G[k];
        t.ord = (int *)(s + L.ord[k]);
        t.pts = (float4 *)(s + L.bpts[k]);
        t.leaf = (NcBox *)(s + L.leaf[k]);
        t.grp = (NcBox *)(s + L.grp[k]);
    }
    a.box = true;
    if (const char *e = getenv("PCR_NC_BOX")) a.box = atoi(e) != 0;
    a.stats = false;
    if (const char *e = getenv("PCR_NC_STATS")) a.stats = atoi(e) != 0;
    a.kmax = 1;
    if (const char *e = getenv("PCR_NDP_CHAMFER_RINGS")) {  // test / tuning hook: 0..3
        const int v = atoi(e);
        if (v >= 0 && v <= 3) a.kmax = v;
    }
    a.trunc = (float)c->trunc;
    a.g1 = (float)(1.0 / (double)c->K);
    a.g2 = (float)(1.0 / (double)c->M);
    a.d1 = c->d1; a.d2 = c->d2; a.i1 = c->i1; a.i2 = c->i2;
    a.gacc = (long long *)c->gacc;
    a.hdr = (NcHdr *)(s + L.hdr);
    a.cnt = (int *)(s + L.cnt);
    a.fb = (int *)(s + L.fb);
    a.fbkey = (unsigned long long *)(s + L.fbkey);
    a.gate = current_gate();
    a.fshift = -1;  // (a fixed exponent, hi words only: the round-3 form, kept for diagnostics)
    return PCR_OK;
}

}  // namespace
}  // namespace pcr

extern "C" int64_t pcr_ndp_chamfer_scratch_bytes(int32_t K, int32_t M) {
    if (K < 1 || M < 1) return 0;
    return (int64_t)pcr::nc_layout(K, M).total;
}

extern "C" int64_t pcr_ndp_chamfer_gacc_words(int32_t K) {
    return K < 1 ? 0 : 1 + 6 * (int64_t)K * PCR_NDP_GACC_REPLICAS;
}

extern "C" int32_t pcr_ndp_chamfer_max_points(void) { return pcr::kScanLds; }

namespace pcr {
namespace {
// count, scan, scatter and the coarse boxes of one cloud (cell from the header)
int nc_build(const NcArgs &a, const float *P, int n, const float *cellp, const NcCloud &g, int *flag,
             long long *gacc, const double *gate, hipStream_t s) {
    const int nb = (n + 255) / 256;
    // the subset build (gacc given) also measures the subset's extent for the
    // gradient's fixed-point exponent
    hipLaunchKernelGGL(nc_count, dim3(nb), dim3(256), 0, s, P, n, cellp, g, a.cnt, flag, gacc,
                       gacc ? &a.hdr->amax_s : (unsigned *)nullptr, gate);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(nc_scan, dim3(1), dim3(1024), sizeof(int) * ((size_t)g.S + 1 + (g.S >> 4) + 1), s, (const int *)a.cnt, g,
                       a.hdr, gacc, a.g1 > a.g2 ? a.g1 : a.g2, a.M, a.fshift, gate);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(nc_scatter, dim3(nb), dim3(256), 0, s, P, n, cellp, g, a.cnt, gate);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}
}  // namespace
}  // namespace pcr

extern "C" int pcr_ndp_chamfer_prepare(const pcr_ndp_chamfer *c, const float *xs0, pcr_stream_t stream) {
    pcr::clear_error();
    pcr::NcArgs a;
    int rc = pcr::nc_args(c, a);
    if (rc != PCR_OK) return rc;
    PCR_REQUIRE(xs0, PCR_ERR_ARG, "ndp_chamfer_prepare: null xs0");
    hipStream_t s = pcr::as_stream(stream);
    PCR_HIP_CHECK(pcr::nc_scan_attr());
    PCR_HIP_CHECK(hipMemsetAsync(a.hdr, 0, sizeof(pcr::NcHdr), s));
    PCR_HIP_CHECK(hipMemsetAsync(a.cnt, 0, sizeof(int) * (size_t)(a.St > a.Ss ? a.St : a.Ss), s));
    hipLaunchKernelGGL(pcr::nc_bbox, dim3(1), dim3(1024), 0, s, a.tgt, a.M, &a.hdr->cell_t, &a.hdr->tflag,
                       &a.hdr->amax_t);
    PCR_LAUNCH_CHECK();
    if (a.box) {
        // both clouds' spatial orders (the subset's from its starting positions xs0),
        // the target's tree once
        PCR_HIP_CHECK(pcr::nc_order_attr());
        const size_t lds = sizeof(int) * (pcr::kOrdN + 1);
        hipLaunchKernelGGL(pcr::nc_order, dim3(1), dim3(1024), lds, s, a.tgt, a.M, a.bt.ord);
        PCR_LAUNCH_CHECK();
        hipLaunchKernelGGL(pcr::nc_order, dim3(1), dim3(1024), lds, s, xs0, a.K, a.bs.ord);
        PCR_LAUNCH_CHECK();
        hipLaunchKernelGGL(pcr::nc_leaves, dim3(a.bt.G), dim3(1024), 0, s, a.tgt, a.bt, (int *)nullptr,
                           (long long *)nullptr, (unsigned *)nullptr, (const double *)nullptr);
        PCR_LAUNCH_CHECK();
        return PCR_OK;
    }
    hipLaunchKernelGGL(pcr::nc_bbox, dim3(1), dim3(1024), 0, s, xs0, a.K, &a.hdr->cell_s, (int *)nullptr,
                       (unsigned *)nullptr);
    PCR_LAUNCH_CHECK();
    // the target grids, once (ungated: prepare runs outside the level graph)
    return pcr::nc_build(a, a.tgt, a.M, &a.hdr->cell_t, a.ct, &a.hdr->tflag, nullptr, nullptr, s);
}

extern "C" int pcr_ndp_chamfer_step(const pcr_ndp_chamfer *c, pcr_stream_t stream) {
    pcr::clear_error();
    pcr::NcArgs a;
    int rc = pcr::nc_args(c, a);
    if (rc != PCR_OK) return rc;
    hipStream_t s = pcr::as_stream(stream);
    if (a.box) {
        // the leaf blocks, and enough more that each thread zeroes <= 16 gradient words
        const long long zw = 6LL * pcr::kRep * a.K;
        const int nbz = (int)std::max<long long>(a.bs.G, (zw + 16 * 1024 - 1) / (16 * 1024));
        hipLaunchKernelGGL(pcr::nc_leaves, dim3(nbz), dim3(1024), 0, s, a.xs, a.bs, a.hdr->sbad, a.gacc,
                           a.hdr->samax, a.gate);
        PCR_LAUNCH_CHECK();
        const int lpq = 8;  // lanes per box query (4 / 8 / 16 measured, round 4)
        const int qpb = 256 / lpq;
        const int nb0 = (a.K + qpb - 1) / qpb, nb1 = (a.M + qpb - 1) / qpb;
        const size_t lds = sizeof(pcr::NcBox) * (size_t)(pcr::kGrp + std::max(a.bt.L, a.bs.L));  // <= 33 KiB
        prof_begin(s, pcr::kProfNndGrid);
        switch (lpq) {
            case 4: hipLaunchKernelGGL(pcr::nc_bquery<4>, dim3(nb0 + nb1), dim3(256), lds, s, a, nb0); break;
            case 16: hipLaunchKernelGGL(pcr::nc_bquery<16>, dim3(nb0 + nb1), dim3(256), lds, s, a, nb0); break;
            default: hipLaunchKernelGGL(pcr::nc_bquery<8>, dim3(nb0 + nb1), dim3(256), lds, s, a, nb0); break;
        }
        PCR_LAUNCH_CHECK();
        prof_end(s, pcr::kProfNndGrid);
        return PCR_OK;
    }
    rc = pcr::nc_build(a, a.xs, a.K, &a.hdr->cell_s, a.cs, &a.hdr->sflag, a.gacc, a.gate, s);
    if (rc != PCR_OK) return rc;
    // lanes per query (C5, 30K queries: 4 lanes and a ring cap of 1 measured best,
    // tools/ndp_sweep.sh)
    const long long nq = (long long)a.K + a.M;
    int lpq = nq >= (1LL << 18) ? 1 : nq >= (1LL << 14) ? 4 : 8;
    if (const char *e = getenv("PCR_NND_LPQ")) {
        const int v = atoi(e);
        if (v == 1 || v == 2 || v == 4 || v == 8) lpq = v;
    }
    const int qpb = 256 / lpq;
    const int nb0 = (a.K + qpb - 1) / qpb, nb1 = (a.M + qpb - 1) / qpb;
    prof_begin(s, pcr::kProfNndGrid);
    switch (lpq) {
        case 1: hipLaunchKernelGGL(pcr::nc_query<1>, dim3(nb0 + nb1), dim3(256), 0, s, a, nb0); break;
        case 2: hipLaunchKernelGGL(pcr::nc_query<2>, dim3(nb0 + nb1), dim3(256), 0, s, a, nb0); break;
        case 4: hipLaunchKernelGGL(pcr::nc_query<4>, dim3(nb0 + nb1), dim3(256), 0, s, a, nb0); break;
        default: hipLaunchKernelGGL(pcr::nc_query<8>, dim3(nb0 + nb1), dim3(256), 0, s, a, nb0); break;
    }
    PCR_LAUNCH_CHECK();
    prof_end(s, pcr::kProfNndGrid);
    hipLaunchKernelGGL(pcr::nc_fallback, dim3(pcr::kFbBlocks), dim3(256), 0, s, a);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(pcr::nc_fallback_emit, dim3((a.K + a.M + 255) / 256), dim3(256), 0, s, a);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}
