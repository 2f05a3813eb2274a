// a1 (large clouds): exact nearest neighbour by certified grid search.
//
// Same contract as the brute-force kernel (nnd.hip, my_lib.cpp:3-25): for each
// query q the result is the candidate j minimising d_j = (dx*dx + dy*dy) +
// dz*dz in f32 (dx = c_j - q, no FMA), lowest index on ties.  For finite
// inputs that is the lexicographic minimum of (d_j, j), which a search over any
// superset of the winners returns unchanged; clouds holding a NaN/Inf (where
// the reference's seed rule matters) or too far from the origin for integer
// cell coordinates are answered by the reference loop itself.
//
// Per cloud a hashed uniform grid (cell = 0.6 * cbrt(bbox volume / n),
// degenerate boxes widened) stores float4 (x, y, z, index) sorted by slot.
// A query scans the Chebyshev rings k = 0, 1, ... of cells around its own;
// after ring k, every unvisited point is at least g = (distance from q to the
// faces of the (2k+1)^3 block) away, and its computed f32 distance at least
// g^2 (1 - 8 * 2^-24) (each of the 5 f32 roundings is relative); once that
// exceeds the best distance (strictly) the answer is final.  Rings are capped
// at kMaxRing, then the query scans every point (same exact rule).
//
// One thread (or LPQ lanes) per query, 256-thread blocks over all pairs and both directions,
// ordered per XCD (xcd_slot) so each grid (160 KB per 8192-point cloud) is
// served from one XCD's L2.
#include "pcr_internal.h"
#include "scan.h"
#include "nng.h"
#include "geom.h"
#include <cstdlib>

namespace pcr {
namespace {

constexpr int kMaxRing = 3;

struct NgArgs {
    const float *xyz[2];  // set 0: xyz1 (B, n0, 3), set 1: xyz2 (B, n1, 3)
    int n[2];
    int B, S, nmax;
    float cf;             // cell factor (0.6)
    float *cell;          // [2][B]
    int *flag;            // [2][B]: set s of pair b holds a NaN/Inf or is too far out (both: the reference loop)
    int *hcnt;            // [2][B][S]
    int *start;           // [2][B][S+1]
    float4 *pts;          // [2][B][nmax]
    float *dist[2];       // dist[0] = dist1: queries of set 0 against the grid of set 1
    int32_t *idx[2];
    const double *gate;   // f4 early stop (pcr_internal.h), or null
    // set 0 as T (x) src, written to xyz[0] by the box pass (nnd_forward_grid_xf;
    // null: set 0 is read as given)
    const float *xsrc;
    const double *xT;
    float *xout;
};

// the pair's clouds go to the reference loop (either set flagged by nng_bbox)
__device__ __forceinline__ bool ref_loop(const NgArgs &a, int b) { return (a.flag[b] | a.flag[a.B + b]) != 0; }

using nng::ccoord;
using nng::d2f;
using nng::nhash;

// one cloud's box -> its cell size and flag (thread 0 writes both, to global
// and to *cell_out / *bad_out in LDS); every thread of the block calls it
__device__ __forceinline__ void bbox_block(const NgArgs &a, float *cell_out, int *bad_out) {
    const int s = blockIdx.x, b = blockIdx.y, t = threadIdx.x, n = a.n[s];
    const float *P = a.xyz[s] + (size_t)b * n * 3;
    float lo[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
    float hi[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    int bad = 0;
    const bool xf = a.xsrc && s == 0;
#pragma unroll 4
    for (int i = t; i < n; i += 1024) {
        float v[3];
        if (xf) {  // transform_kernel's rounding (procrustes.hip): f64 xform12, then f32
            const float *q = a.xsrc + ((size_t)b * n + i) * 3;
            double x, y, z;
            xform12(a.xT + (size_t)b * 16, (double)q[0], (double)q[1], (double)q[2], x, y, z);
            v[0] = (float)x; v[1] = (float)y; v[2] = (float)z;
            float *o = a.xout + ((size_t)b * n + i) * 3;
            o[0] = v[0]; o[1] = v[1]; o[2] = v[2];
        } else {
            v[0] = P[3 * i]; v[1] = P[3 * i + 1]; v[2] = P[3 * i + 2];
        }
        for (int c = 0; c < 3; ++c) {
            bad |= !__builtin_isfinite(v[c]);
            lo[c] = fminf(lo[c], v[c]);
            hi[c] = fmaxf(hi[c], v[c]);
        }
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
    if (t != 0) return;  // (the callers synchronise after the call)
    double e[3], m = 0.0, amax = 0.0;
    for (int c = 0; c < 3; ++c) {
        float l = sl[c][0], h = sh[c][0];
        for (int w = 1; w < 16; ++w) { l = fminf(l, sl[c][w]); h = fmaxf(h, sh[c][w]); }
        e[c] = (double)h - (double)l;
        m = fmax(m, e[c]);
        amax = fmax(amax, fmax(fabs((double)l), fabs((double)h)));
    }
    bad = 0;
    for (int w = 0; w < 16; ++w) bad |= sb[w];
    double cell = 1.0;
    if (m > 0.0) {
        double v = 1.0;
        for (int c = 0; c < 3; ++c) v *= fmax(e[c], 1e-3 * m);
        cell = (double)a.cf * cbrt(v / (double)(n > 0 ? n : 1));
    }
    // integer cell coordinates must stay far from int overflow
    if (!(amax / cell < 1e9)) bad = 1;
    a.cell[s * a.B + b] = (float)cell;
    a.flag[s * a.B + b] = bad ? 1 : 0;  // every launch writes both sets' flags: no clearing
    *cell_out = (float)cell;
    *bad_out = bad;
}

__global__ __launch_bounds__(1024) void nng_bbox(NgArgs a) {
    if (gated_off(a.gate)) return;
    __shared__ float sc;
    __shared__ int sbad;
    bbox_block(a, &sc, &sbad);
}

__global__ void nng_count(NgArgs a) {
    if (gated_off(a.gate)) return;
    const int s = blockIdx.z, b = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n[s] || ref_loop(a, b)) return;
    const float *p = a.xyz[s] + ((size_t)b * a.n[s] + i) * 3;
    const double ic = 1.0 / (double)a.cell[s * a.B + b];
    const unsigned h = nhash(ccoord(p[0], ic), ccoord(p[1], ic), ccoord(p[2], ic), a.S);
    atomicAdd(a.hcnt + ((size_t)s * a.B + b) * a.S + h, 1);
}

__global__ __launch_bounds__(1024) void nng_scan(NgArgs a) {
    if (gated_off(a.gate)) return;
    const int s = blockIdx.y, b = blockIdx.x;
    if (ref_loop(a, b)) return;
    const size_t g = (size_t)s * a.B + b;
    block_exclusive_scan_1024(a.hcnt + g * a.S, a.start + g * (a.S + 1), a.S, true);
}

__global__ void nng_scatter(NgArgs a) {
    if (gated_off(a.gate)) return;
    const int s = blockIdx.z, b = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n[s] || ref_loop(a, b)) return;
    const float *p = a.xyz[s] + ((size_t)b * a.n[s] + i) * 3;
    const size_t g = (size_t)s * a.B + b;
    const double ic = 1.0 / (double)a.cell[g];
    const unsigned h = nhash(ccoord(p[0], ic), ccoord(p[1], ic), ccoord(p[2], ic), a.S);
    const int pos = a.start[g * (a.S + 1) + h] + atomicAdd(a.hcnt + g * a.S + h, 1);
    a.pts[g * a.nmax + pos] = make_float4(p[0], p[1], p[2], __int_as_float(i));
}

// count, scan and scatter of one cloud's grid in one workgroup, the slot
// counters in LDS (S <= kLdsSlots): the per-point atomics stay on the CU (the
// global count / scatter passes took ~0.35 ms per C4 Chamfer).  Order within a
// cell is atomic order, as before; the (d, j) minimum does not depend on it.
constexpr int kLdsSlots = 32768;

__device__ __forceinline__ void build_block(const NgArgs &a, float cell) {
    extern __shared__ int cnt[];  // S + 1: counts -> exclusive starts -> cursors
    const int s = blockIdx.x, b = blockIdx.y, S = a.S, n = a.n[s];
    const size_t g = (size_t)s * a.B + b;
    const float *P = a.xyz[s] + (size_t)b * n * 3;
    const double ic = 1.0 / (double)cell;
    for (int i = threadIdx.x; i < S; i += 1024) cnt[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += 1024)
        atomicAdd(&cnt[nhash(ccoord(P[3 * i], ic), ccoord(P[3 * i + 1], ic), ccoord(P[3 * i + 2], ic), S)], 1);
    __syncthreads();
    block_exclusive_scan_1024(cnt, cnt, S, false);
    int *st = a.start + g * (S + 1);
    for (int i = threadIdx.x; i <= S; i += 1024) st[i] = cnt[i];
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += 1024) {
        const float x = P[3 * i], y = P[3 * i + 1], z = P[3 * i + 2];
        const unsigned h = nhash(ccoord(x, ic), ccoord(y, ic), ccoord(z, ic), S);
        a.pts[g * a.nmax + atomicAdd(&cnt[h], 1)] = make_float4(x, y, z, __int_as_float(i));
    }
}

// the box and the grid of one cloud in one workgroup (one launch fewer per
// call).  A cloud flagged by its own box is not built; one flagged only by the
// other set's box is built and never read (nng_query, launched after both,
// tests both flags).
__global__ __launch_bounds__(1024) void nng_bbox_build(NgArgs a) {
    if (gated_off(a.gate)) return;
    __shared__ float sc;
    __shared__ int sbad;
    bbox_block(a, &sc, &sbad);
    __syncthreads();
    if (sbad) return;
    build_block(a, sc);
}

// XCD-aware block order: the hardware deals linear block ids round-robin over
// the 8 XCDs; the k-th block an XCD receives takes the k-th slot of that XCD's
// contiguous range of (direction, pair, chunk) work, so every grid is read by
// one XCD at a time and stays in its L2 while its 32 chunks run (row-major
// order spread each grid over all 8 L2s: 5.3 GB of fabric reads per C4 launch).
__device__ __forceinline__ int xcd_slot(int L, int total) {
    const int xcd = L & 7, k = L >> 3, per = total >> 3, rem = total & 7;
    return (xcd < rem ? xcd * (per + 1) : rem * (per + 1) + (xcd - rem) * per) + k;
}

// LPQ lanes per query.  A batch fills the chip with one thread per query; a
// single pair (the NDP Chamfer, quality metrics: ~25K queries) does not, and its
// per-query cell walks are long dependent load chains.  With LPQ > 1 the lanes
// of a query split each ring's (dx, dy) columns (and the fallback scan) and
// merge their (d, j) minima before the certification test; the minimum of
// (d, j) pairs does not depend on the merge order, so every LPQ gives the same
// answer.
template <int LPQ>
__global__ __launch_bounds__(256) void nng_query(NgArgs a, int nchunk) {
    if (gated_off(a.gate)) return;
    constexpr int QPB = 256 / LPQ;
    const int w = xcd_slot(blockIdx.x, gridDim.x);
    const int grp = w / nchunk, chunk = w - grp * nchunk;
    const int dir = grp / a.B, b = grp - dir * a.B;
    const int sub = threadIdx.x % LPQ, qslot = chunk * QPB + threadIdx.x / LPQ;
    const int qs = dir, gs = 1 - dir;  // queries from set dir, candidates from the other set
    if (qslot >= a.n[qs]) return;  // a query's lanes leave together
    // queries in the slot order of their own cloud's grid (cell-sorted): the
    // lanes of a wave walk neighbouring cells (less divergence, shared lines);
    // the reference-loop clouds (flag) have no grid and go in index order
    int qi = qslot;
    float qx, qy, qz;
    const bool refl = ref_loop(a, b);
    if (refl) {
        const float *q = a.xyz[qs] + ((size_t)b * a.n[qs] + qi) * 3;
        qx = q[0]; qy = q[1]; qz = q[2];
    } else {
        const float4 qp = a.pts[((size_t)qs * a.B + b) * a.nmax + qslot];
        qx = qp.x; qy = qp.y; qz = qp.z;
        qi = __float_as_int(qp.w);
    }
    const int m = a.n[gs];
    const float *C = a.xyz[gs] + (size_t)b * m * 3;
    float best = __builtin_inff();
    int bj = 0x7fffffff;
    bool done = false;
    auto merge = [&]() {
#pragma unroll
        for (int o = 1; o < LPQ; o <<= 1) {
            const float ob = __shfl_xor(best, o, 64);
            const int oj = __shfl_xor(bj, o, 64);
            if (ob < best || (ob == best && oj < bj)) { best = ob; bj = oj; }
        }
    };
    if (refl) {
        // the reference loop: seed with candidate 0, strict < (my_lib.cpp:11-20)
        if (sub == 0) {
            best = d2f(C[0], C[1], C[2], qx, qy, qz);
            bj = 0;
            for (int j = 1; j < m; ++j) {
                const float d = d2f(C[3 * j], C[3 * j + 1], C[3 * j + 2], qx, qy, qz);
                if (d < best) { best = d; bj = j; }
            }
        }
        done = true;
    }
    if (!done) {
        const size_t g = (size_t)gs * a.B + b;
        const nng::View v{a.cell[g], a.S, a.start + g * (a.S + 1), a.pts + g * a.nmax};
        const float4 *pts = v.pts;
        done = nng::ring_walk<LPQ>(v, qx, qy, qz, sub, kMaxRing, best, bj);
        if (!done) {  // not certified within kMaxRing rings: every candidate, read
                      // as the grid's float4 (x, y, z, index) copy (one 16-B load each)
#pragma unroll 4
            for (int s = sub; s < m; s += LPQ) {
                const float4 p = pts[s];
                const float d = d2f(p.x, p.y, p.z, qx, qy, qz);
                const int j = __float_as_int(p.w);
                if (d < best || (d == best && j < bj)) { best = d; bj = j; }
            }
            merge();
        }
    }
    if (sub == 0) {
        a.dist[dir][(size_t)b * a.n[qs] + qi] = best;
        a.idx[dir][(size_t)b * a.n[qs] + qi] = bj;
    }
}

}  // namespace

int nnd_forward_grid(const float *xyz1, const float *xyz2, int b, int n, int m, float *dist1,
                     float *dist2, int32_t *idx1, int32_t *idx2, hipStream_t s) {
    return nnd_forward_grid_xf(xyz1, nullptr, nullptr, xyz2, b, n, m, dist1, dist2, idx1, idx2, s);
}

int nnd_forward_grid_xf(const float *xyz1, const float *src, const double *T, const float *xyz2, int b, int n,
                        int m, float *dist1, float *dist2, int32_t *idx1, int32_t *idx2, hipStream_t s) {
    NgArgs a;
    a.xyz[0] = xyz1; a.xyz[1] = xyz2; a.n[0] = n; a.n[1] = m; a.B = b;
    a.xsrc = src; a.xT = T; a.xout = src ? const_cast<float *>(xyz1) : nullptr;
    a.nmax = n > m ? n : m;
    int S = 256;
    while (S < a.nmax) S <<= 1;
    a.S = S;
    const size_t cells = 2 * (size_t)b, hc = cells * S, stc = cells * (S + 1), pc = cells * a.nmax;
    char *ws = (char *)workspace(15, 4 * (cells + 2 * (size_t)b + hc + stc) + 16 * pc + 256);
    PCR_REQUIRE(ws, PCR_ERR_NOMEM, "nnd_forward (grid): %s", pcr_last_error());
    a.pts = (float4 *)ws;
    a.cell = (float *)(a.pts + pc);
    a.flag = (int *)(a.cell + cells);
    a.hcnt = a.flag + 2 * (size_t)b;
    a.start = a.hcnt + hc;
    a.dist[0] = dist1; a.dist[1] = dist2; a.idx[0] = idx1; a.idx[1] = idx2;
    a.gate = current_gate();
    a.cf = 0.6f;  // 0.4 / 0.5 / 0.6 / 0.8 / 1.0 x cbrt(V / n) measured
    const bool lds_build = S <= kLdsSlots;
    PCR_REQUIRE(lds_build || !src, PCR_ERR_ARG, "nnd_forward (grid): fused transform needs the LDS build");
    if (!lds_build) PCR_HIP_CHECK(hipMemsetAsync(a.hcnt, 0, sizeof(int) * hc, s));
    if (lds_build) {
        // the attribute is set once, outside any stream capture (the NDP level
        // graphs capture this call after an eager warm-up step)
        static const hipError_t attr = hipFuncSetAttribute((const void *)nng_bbox_build,
                                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                                           (int)(sizeof(int) * (kLdsSlots + 1)));
        PCR_HIP_CHECK(attr);
        hipLaunchKernelGGL(nng_bbox_build, dim3(2, b), dim3(1024), sizeof(int) * (size_t)(S + 1), s, a);
        PCR_LAUNCH_CHECK();
    } else {
        hipLaunchKernelGGL(nng_bbox, dim3(2, b), dim3(1024), 0, s, a);
        PCR_LAUNCH_CHECK();
        const dim3 pg((a.nmax + 255) / 256, b, 2);
        hipLaunchKernelGGL(nng_count, pg, dim3(256), 0, s, a);
        PCR_LAUNCH_CHECK();
        hipLaunchKernelGGL(nng_scan, dim3(b, 2), dim3(1024), 0, s, a);
        PCR_LAUNCH_CHECK();
        PCR_HIP_CHECK(hipMemsetAsync(a.hcnt, 0, sizeof(int) * hc, s));
        hipLaunchKernelGGL(nng_scatter, pg, dim3(256), 0, s, a);
        PCR_LAUNCH_CHECK();
    }
    prof_begin(s, kProfNndGrid);
    // lanes per query: one thread per query once the launch fills the chip
    // (PCR_NND_LPQ = 1|2|4|8|16 overrides)
    const long long nq = (long long)b * (n + m);
    int lpq = nq >= (1LL << 18) ? 1 : nq >= (1LL << 16) ? 4 : 8;
    if (const char *e = getenv("PCR_NND_LPQ")) {
        const int v = atoi(e);
        if (v == 1 || v == 2 || v == 4 || v == 8 || v == 16) lpq = v;
    }
    const int nchunk = (a.nmax + 256 / lpq - 1) / (256 / lpq);
    const dim3 qg(2 * b * nchunk), qb(256);
    switch (lpq) {
        case 1: hipLaunchKernelGGL(nng_query<1>, qg, qb, 0, s, a, nchunk); break;
        case 2: hipLaunchKernelGGL(nng_query<2>, qg, qb, 0, s, a, nchunk); break;
        case 4: hipLaunchKernelGGL(nng_query<4>, qg, qb, 0, s, a, nchunk); break;
        case 8: hipLaunchKernelGGL(nng_query<8>, qg, qb, 0, s, a, nchunk); break;
        default: hipLaunchKernelGGL(nng_query<16>, qg, qb, 0, s, a, nchunk); break;
    }
    PCR_LAUNCH_CHECK();
    prof_end(s, kProfNndGrid);
    return PCR_OK;
}

}  // namespace pcr
