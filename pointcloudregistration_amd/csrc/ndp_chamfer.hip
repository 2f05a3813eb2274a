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
//     answered by nc_fallback, a tiled exact scan (one wave per 4 listed
//     queries, 1,024 candidates per LDS tile) -- the far target points of a
//     partially overlapping pair (36 % of the C5 target) had made every wave
//     of the general kernel run a whole-cloud scan;
//   * the gradient dL/dxs is accumulated in the same epilogue: query i of the
//     subset adds 2 gd1 (x_i - y_j), query k of the target subtracts
//     2 gd2 (y_k - x_i) at its answer i, each rounded to 2^-44 fixed point and
//     added with integer atomics (exact and order-free: the same bits on every
//     replay), gd = 1/K, 1/M where d < trunc (else 0) as pcr_ndp_chamfer_glue;
//     pcr_ndp_train_backward reads the sums.  This replaces the five-launch
//     deterministic bucket backward of pcr_nnd_backward (~110 us per C5
//     iteration).  Distances and indices are those of pcr_nnd_forward bit for
//     bit; the gradient differs from the CPU-order f32 sums of
//     pcr_nnd_backward by its rounding (f32 contributions, exact sums).
//
// Non-finite or out-of-range points (no integer cell coordinates) switch the
// iteration to the reference loop (seed with candidate 0, strict <) as
// nnd_grid.hip does.
#include "pcr_internal.h"
#include "nng.h"
#include "scan.h"

namespace pcr {
namespace {

using nng::ccoord;
using nng::d2f;
using nng::nhash;
using nng::take;

constexpr double kFixScale = 17592186044416.0;  // 2^44
constexpr int kTile = 1024;                     // candidates per LDS tile of nc_fallback
constexpr int kFbWaves = 8, kFbQ = 4;           // nc_fallback: waves per block, queries per wave

struct NcHdr {
    float cell_t, cell_s;
    int tflag;      // target non-finite / out of cell range: reference loop for the level
    int sflag;      // subset non-finite / out of range this iteration (nc_count)
    int mode;       // sflag | tflag as nc_scan saw it (read by the queries)
    int fb_cnt[2];  // listed (uncertified) queries per direction
    int pad;
};

struct NcArgs {
    const float *xs, *tgt;  // (K, 3), (M, 3)
    int K, M, St, Ss, kmax;
    float trunc, g1, g2;    // g1 = 1/K, g2 = 1/M (as the glue)
    float *d1, *d2;
    int32_t *i1, *i2;
    long long *gacc;        // [0]: non-finite contribution flag; [1 + 3k + c]: dL/dxs fixed point
    NcHdr *hdr;
    int *cnt;               // max(Ss, St): counting-sort counts, zero between builds
    int *start_t, *start_s; // St + 1, Ss + 1
    float4 *pts_t, *pts_s;  // M, K: (x, y, z, index bits) sorted by slot
    int *fb;                // K + M: listed queries (dir 0 at 0, dir 1 at K)
    const double *gate;
};

__device__ __forceinline__ bool cell_ok(float x, float y, float z, double ic) {
    return __builtin_isfinite(x) && __builtin_isfinite(y) && __builtin_isfinite(z) &&
           fabs((double)x * ic) < 1e9 && fabs((double)y * ic) < 1e9 && fabs((double)z * ic) < 1e9;
}

// cell = 0.6 cbrt(bbox volume / n) of one cloud (nng_bbox's rule); flag on a
// non-finite point.  One workgroup.
__global__ __launch_bounds__(1024) void nc_bbox(const float *P, int n, float *cell, int *flag) {
    const int t = threadIdx.x;
    float lo[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
    float hi[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    int bad = 0;
    for (int i = t; i < n; i += 1024)
        for (int c = 0; c < 3; ++c) {
            const float v = P[3 * i + c];
            bad |= !__builtin_isfinite(v);
            lo[c] = fminf(lo[c], v);
            hi[c] = fmaxf(hi[c], v);
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
__global__ void nc_count(const float *P, int n, const float *cellp, int S, int *cnt, int *flag,
                         long long *gacc, const double *gate) {
    if (gated_off(gate)) return;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (gacc) {
        gacc[1 + 3 * i] = 0; gacc[2 + 3 * i] = 0; gacc[3 + 3 * i] = 0;
    }
    const float x = P[3 * i], y = P[3 * i + 1], z = P[3 * i + 2];
    const double ic = 1.0 / (double)*cellp;
    if (!cell_ok(x, y, z, ic)) { atomicOr(flag, 1); return; }
    atomicAdd(cnt + nhash(ccoord(x, ic), ccoord(y, ic), ccoord(z, ic), S), 1);
}

// one workgroup: starts of the subset (or target) grid; the per-iteration
// resets (mode, listed counts, the gradient's non-finite flag) ride along
__global__ __launch_bounds__(1024) void nc_scan(int *cnt, int *start, int S, NcHdr *h, long long *gacc,
                                                const double *gate) {
    if (gated_off(gate)) return;
    block_exclusive_scan_1024(cnt, start, S, false);
    if (threadIdx.x == 0 && gacc) {
        h->mode = h->sflag | h->tflag;
        h->sflag = 0;
        h->fb_cnt[0] = 0;
        h->fb_cnt[1] = 0;
        gacc[0] = 0;
    }
}

__global__ void nc_scatter(const float *P, int n, const float *cellp, int S, int *cnt, const int *start,
                           float4 *pts, const double *gate) {
    if (gated_off(gate)) return;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = P[3 * i], y = P[3 * i + 1], z = P[3 * i + 2];
    const double ic = 1.0 / (double)*cellp;
    if (!cell_ok(x, y, z, ic)) return;
    const unsigned hs = nhash(ccoord(x, ic), ccoord(y, ic), ccoord(z, ic), S);
    const int pos = start[hs] + atomicSub(cnt + hs, 1) - 1;
    pts[pos] = make_float4(x, y, z, __int_as_float(i));
}

__device__ __forceinline__ void fix_add(long long *dst, float v, long long *flag) {
    if (!__builtin_isfinite(v) || fabs((double)v) >= 4096.0) {  // |v| 2^12: sums stay below 2^63
        __hip_atomic_fetch_or(flag, 1LL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    __hip_atomic_fetch_add(dst, (long long)__builtin_rint((double)v * kFixScale), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// the answer (best, bj) of query q in direction dir: outputs and gradient
// (pcr_nnd_backward's terms: g = gd * 2, grad1 += g (x - y), grad1[i] -= g (y - x))
__device__ __forceinline__ void emit(const NcArgs &a, int dir, int q, float best, int bj) {
    if (dir == 0) {
        a.d1[q] = best;
        a.i1[q] = bj;
        const float g = (!(best >= a.trunc) ? a.g1 : 0.0f) * 2;
        if (bj < 0 || bj >= a.M) return;
        for (int c = 0; c < 3; ++c)
            fix_add(a.gacc + 1 + 3 * q + c, g * (a.xs[3 * q + c] - a.tgt[3 * bj + c]), a.gacc);
    } else {
        a.d2[q] = best;
        a.i2[q] = bj;
        const float g = (!(best >= a.trunc) ? a.g2 : 0.0f) * 2;
        if (bj < 0 || bj >= a.K) return;
        for (int c = 0; c < 3; ++c)
            fix_add(a.gacc + 1 + 3 * bj + c, -(g * (a.tgt[3 * q + c] - a.xs[3 * bj + c])), a.gacc);
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
    const float *Q = dir ? a.tgt : a.xs;
    const float *C = dir ? a.xs : a.tgt;
    int qi = qslot;
    float qx, qy, qz;
    if (brute) {
        qx = Q[3 * qi]; qy = Q[3 * qi + 1]; qz = Q[3 * qi + 2];
    } else {
        const float4 qp = (dir ? a.pts_t : a.pts_s)[qslot];
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
        emit(a, dir, qi, best, bj);
        return;
    }
    const nng::View v = dir ? nng::View{a.hdr->cell_s, a.Ss, a.start_s, a.pts_s}
                            : nng::View{a.hdr->cell_t, a.St, a.start_t, a.pts_t};
    const bool done = nng::ring_walk<LPQ>(v, qx, qy, qz, sub, a.kmax, best, bj);
    if (sub != 0) return;
    if (done) {
        emit(a, dir, qi, best, bj);
    } else {
        const int pos = atomicAdd(&a.hdr->fb_cnt[dir], 1);
        a.fb[(dir ? a.K : 0) + pos] = qi;
    }
}

// the listed queries: exact scan of every candidate, kTile at a time through
// LDS; wave w holds queries 4w..4w+3 of the block's 32 in registers, lane l
// takes candidates l, l + 64, ... of each tile
__global__ __launch_bounds__(64 * kFbWaves) void nc_fallback(NcArgs a) {
    if (gated_off(a.gate)) return;
    const int dir = blockIdx.y;
    const int cnt = a.hdr->fb_cnt[dir];
    const int base = blockIdx.x * (kFbWaves * kFbQ);
    if (base >= cnt) return;  // uniform over the block
    __shared__ float4 tile[kTile];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const float *Q = dir ? a.tgt : a.xs;
    const float4 *cand = dir ? a.pts_s : a.pts_t;
    const int nc = dir ? a.K : a.M;
    const int *list = a.fb + (dir ? a.K : 0);
    float qx[kFbQ], qy[kFbQ], qz[kFbQ], best[kFbQ];
    int qi[kFbQ], bj[kFbQ];
#pragma unroll
    for (int u = 0; u < kFbQ; ++u) {
        const int e = base + wv * kFbQ + u;
        qi[u] = e < cnt ? list[e] : -1;
        const int q = qi[u] >= 0 ? qi[u] : 0;
        qx[u] = Q[3 * q]; qy[u] = Q[3 * q + 1]; qz[u] = Q[3 * q + 2];
        best[u] = __builtin_inff();
        bj[u] = 0x7fffffff;
    }
    for (int t0 = 0; t0 < nc; t0 += kTile) {
        const int tn = min(kTile, nc - t0);
        __syncthreads();
        for (int c = threadIdx.x; c < tn; c += 64 * kFbWaves) tile[c] = cand[t0 + c];
        __syncthreads();
        for (int c = lane; c < tn; c += 64) {
            const float4 p = tile[c];
            const int j = __float_as_int(p.w);
#pragma unroll
            for (int u = 0; u < kFbQ; ++u) take(d2f(p.x, p.y, p.z, qx[u], qy[u], qz[u]), j, best[u], bj[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < kFbQ; ++u)
#pragma unroll
        for (int o = 32; o; o >>= 1) {
            const float ob = __shfl_xor(best[u], o, 64);
            const int oj = __shfl_xor(bj[u], o, 64);
            take(ob, oj, best[u], bj[u]);
        }
#pragma unroll
    for (int u = 0; u < kFbQ; ++u)
        if (lane == u && qi[u] >= 0) emit(a, dir, qi[u], best[u], bj[u]);
}

struct NcLayout {
    size_t hdr, cnt, start_t, start_s, pts_t, pts_s, fb, total;
    int St, Ss;
};

inline int pow2_at_least(int n) {
    int S = 256;
    while (S < n) S <<= 1;
    return S;
}

inline size_t up256(size_t x) { return (x + 255) & ~(size_t)255; }

NcLayout nc_layout(int K, int M) {
    NcLayout L;
    L.St = pow2_at_least(M);
    L.Ss = pow2_at_least(K);
    size_t o = 0;
    L.hdr = o; o = up256(o + sizeof(NcHdr));
    L.cnt = o; o = up256(o + sizeof(int) * (size_t)(L.St > L.Ss ? L.St : L.Ss));
    L.start_t = o; o = up256(o + sizeof(int) * ((size_t)L.St + 1));
    L.start_s = o; o = up256(o + sizeof(int) * ((size_t)L.Ss + 1));
    L.pts_t = o; o = up256(o + sizeof(float4) * (size_t)M);
    L.pts_s = o; o = up256(o + sizeof(float4) * (size_t)K);
    L.fb = o; o = up256(o + sizeof(int) * ((size_t)K + M));
    L.total = o;
    return L;
}

int nc_args(const pcr_ndp_chamfer *c, NcArgs &a) {
    PCR_REQUIRE(c, PCR_ERR_ARG, "ndp_chamfer: null descriptor");
    PCR_REQUIRE(c->K >= 1 && c->M >= 1, PCR_ERR_ARG, "ndp_chamfer: K=%d, M=%d (both >= 1)", c->K, c->M);
    PCR_REQUIRE(c->xs && c->tgt && c->d1 && c->d2 && c->i1 && c->i2 && c->gacc && c->scratch, PCR_ERR_ARG,
                "ndp_chamfer: null buffer");
    PCR_REQUIRE(((uintptr_t)c->scratch & 255) == 0, PCR_ERR_ARG, "ndp_chamfer: scratch not 256-byte aligned");
    const NcLayout L = nc_layout(c->K, c->M);
    char *s = (char *)c->scratch;
    a.xs = c->xs; a.tgt = c->tgt; a.K = c->K; a.M = c->M; a.St = L.St; a.Ss = L.Ss;
    a.kmax = 2;
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
    a.start_t = (int *)(s + L.start_t);
    a.start_s = (int *)(s + L.start_s);
    a.pts_t = (float4 *)(s + L.pts_t);
    a.pts_s = (float4 *)(s + L.pts_s);
    a.fb = (int *)(s + L.fb);
    a.gate = current_gate();
    return PCR_OK;
}

}  // namespace
}  // namespace pcr

extern "C" int64_t pcr_ndp_chamfer_scratch_bytes(int32_t K, int32_t M) {
    if (K < 1 || M < 1) return 0;
    return (int64_t)pcr::nc_layout(K, M).total;
}

extern "C" int pcr_ndp_chamfer_prepare(const pcr_ndp_chamfer *c, const float *xs0, pcr_stream_t stream) {
    pcr::clear_error();
    pcr::NcArgs a;
    int rc = pcr::nc_args(c, a);
    if (rc != PCR_OK) return rc;
    PCR_REQUIRE(xs0, PCR_ERR_ARG, "ndp_chamfer_prepare: null xs0");
    hipStream_t s = pcr::as_stream(stream);
    PCR_HIP_CHECK(hipMemsetAsync(a.hdr, 0, sizeof(pcr::NcHdr), s));
    PCR_HIP_CHECK(hipMemsetAsync(a.cnt, 0, sizeof(int) * (size_t)(a.St > a.Ss ? a.St : a.Ss), s));
    hipLaunchKernelGGL(pcr::nc_bbox, dim3(1), dim3(1024), 0, s, a.tgt, a.M, &a.hdr->cell_t, &a.hdr->tflag);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(pcr::nc_bbox, dim3(1), dim3(1024), 0, s, xs0, a.K, &a.hdr->cell_s, (int *)nullptr);
    PCR_LAUNCH_CHECK();
    // the target grid, once (ungated: prepare runs outside the level graph)
    const int nb = (a.M + 255) / 256;
    hipLaunchKernelGGL(pcr::nc_count, dim3(nb), dim3(256), 0, s, a.tgt, a.M, &a.hdr->cell_t, a.St, a.cnt,
                       &a.hdr->tflag, (long long *)nullptr, (const double *)nullptr);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(pcr::nc_scan, dim3(1), dim3(1024), 0, s, a.cnt, a.start_t, a.St, a.hdr,
                       (long long *)nullptr, (const double *)nullptr);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(pcr::nc_scatter, dim3(nb), dim3(256), 0, s, a.tgt, a.M, &a.hdr->cell_t, a.St, a.cnt,
                       (const int *)a.start_t, a.pts_t, (const double *)nullptr);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

extern "C" int pcr_ndp_chamfer_step(const pcr_ndp_chamfer *c, pcr_stream_t stream) {
    pcr::clear_error();
    pcr::NcArgs a;
    int rc = pcr::nc_args(c, a);
    if (rc != PCR_OK) return rc;
    hipStream_t s = pcr::as_stream(stream);
    const int nbk = (a.K + 255) / 256;
    hipLaunchKernelGGL(pcr::nc_count, dim3(nbk), dim3(256), 0, s, a.xs, a.K, &a.hdr->cell_s, a.Ss, a.cnt,
                       &a.hdr->sflag, a.gacc, a.gate);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(pcr::nc_scan, dim3(1), dim3(1024), 0, s, a.cnt, a.start_s, a.Ss, a.hdr, a.gacc, a.gate);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(pcr::nc_scatter, dim3(nbk), dim3(256), 0, s, a.xs, a.K, &a.hdr->cell_s, a.Ss, a.cnt,
                       (const int *)a.start_s, a.pts_s, a.gate);
    PCR_LAUNCH_CHECK();
    // lanes per query as pcr_nnd_forward's grid search (8 below 64K queries)
    const long long nq = (long long)a.K + a.M;
    int lpq = nq >= (1LL << 18) ? 1 : nq >= (1LL << 16) ? 4 : 8;
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
    const int per = pcr::kFbWaves * pcr::kFbQ;
    const int nmax = a.K > a.M ? a.K : a.M;
    hipLaunchKernelGGL(pcr::nc_fallback, dim3((nmax + per - 1) / per, 2), dim3(64 * pcr::kFbWaves), 0, s, a);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}
