// f2: the KPConv input pyramid helpers of ngenet,
// c2p-net/ngenet/cpp_wrappers:
//   * batch grid subsampling  (cpp_subsampling/grid_subsampling/grid_subsampling.cpp
//     grid_subsampling :3-106, batch_grid_subsampling :109-211; wrapper.cpp :59-330)
//   * batch radius neighbours (cpp_neighbors/neighbors/neighbors.cpp
//     batch_nanoflann_neighbors :211-332; wrapper.cpp :63-230)
// as called by ngenet/data/dataloader.py batch_grid_subsampling :28-66 and
// batch_neighbors :12-25 (the collate_fn pyramid :116-160).
//
// Grid subsampling.  The reference accumulates each voxel's point / feature sums
// in float, in input order, inside an unordered_map<size_t, SampledData> keyed by
// mapIdx = iX + NX*iY + NX*NY*iZ (size_t arithmetic), then emits the voxels in
// the map's iteration order.  Here the per-point keys, a stable radix sort by
// (batch, key), the voxel runs and the float sums (each voxel summed sequentially
// in input order -> the same roundings) run on the GPU.  The emission order is a
// property of libstdc++'s hashtable (bucket count growth and node splicing), so
// the host replays it: it inserts the distinct keys, in first-occurrence order,
// into a std::unordered_map<size_t, int> -- the same insertion sequence the
// reference performs, hence the same iteration order -- and the GPU then writes
// barycentres and mean features straight to their output slots.
//
// Radius neighbours.  Supports go into a hashed uniform grid (cell = |radius|
// (1 + 1e-6), key = (batch, cell)); a query visits the 27 cells around its own
// (de-duplicated hash slots), keeps supports of its batch with f32
// d = (dx*dx + dy*dy) + dz*dz < r2 (nanoflann L2_Simple_Adaptor::evalMetric,
// RadiusResultSet::addPoint: strict), counts them (pass 1), writes
// (d bits, index) keys (pass 2) that a segmented radix sort orders by
// ascending distance, and the rows are padded with supports.size().
// Equal distances come out of the reference in nanoflann's leaf-visit order as
// permuted by std::sort (not stable), and its float box-distance pruning could
// drop a point within ulps of the radius: the GPU flags rows holding a distance
// tie or a near-radius distance, and the host recomputes exactly those rows with
// the reference's tree (kdreplay.cpp).  Every other row is decided by distance
// alone, so the (distance, index) sort gives the reference's order.
#include "pcr_internal.h"

#include <cstring>

#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <iterator>
#include <unordered_map>
#include <vector>

namespace pcr {

// kdreplay.cpp
void kd_replay_rows(const float *q, const float *s, const int *soff, const std::vector<int> &rows,
                    const std::vector<int> &qbatch, float r2, std::vector<std::vector<int>> &res);

namespace {

typedef unsigned long long u64;

// ---------------------------------------------------------------------------
// grid subsampling
// ---------------------------------------------------------------------------

// (size_t)f as g++ emits it on x86-64 (values below 2^63 through the signed
// cvttss2si, so -1.0f -> 2^64 - 1): the reference's iX for a point a rounding
// below its origin corner.
__device__ __forceinline__ u64 f2size(float f) {
    if (f >= 9.223372036854775808e18f) return (u64)(long long)(f - 9.223372036854775808e18f) ^ (1ull << 63);
    return (u64)(long long)f;
}

struct GsArgs {
    const float *pts, *feat;
    int n, fdim, nb;
    const int *off;   // [nb+1] batch offsets
    float dl;
    float *origin;    // [nb][3]
    u64 *nxy;         // [nb][2]
    u64 *maxkey;
    int *bad;
    u64 *key;         // [n] raw mapIdx
    int *bat;         // [n] batch of point
};

__device__ __forceinline__ int batch_of(const int *off, int nb, int i) {
    int lo = 0, hi = nb - 1;  // largest b with off[b] <= i
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= i) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// one block per batch: min/max corners (cloud.cpp min_point/max_point :27-68),
// origin corner and grid extents (grid_subsampling.cpp :23-31)
__global__ __launch_bounds__(256) void gs_bbox(GsArgs a) {
    const int b = blockIdx.x, t = threadIdx.x;
    const int i0 = a.off[b], i1 = a.off[b + 1];
    float lo[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
    float hi[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    int bad = 0;
    for (int i = i0 + t; i < i1; i += 256)
        for (int c = 0; c < 3; ++c) {
            const float v = a.pts[3 * (size_t)i + c];
            bad |= !__builtin_isfinite(v);
            lo[c] = fminf(lo[c], v);
            hi[c] = fmaxf(hi[c], v);
        }
    __shared__ float sl[3][4], sh[3][4];
    __shared__ int sb[4];
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
    if (sb[0] | sb[1] | sb[2] | sb[3]) atomicOr(a.bad, 1);
    if (i1 <= i0) return;
    const float inv = __fdiv_rn(1.0f, a.dl);  // (1/sampleDl): int / float
    float org[3], mx[3];
    for (int c = 0; c < 3; ++c) {
        float l = sl[c][0], h = sh[c][0];
        for (int w = 1; w < 4; ++w) { l = fminf(l, sl[c][w]); h = fmaxf(h, sh[c][w]); }
        org[c] = __fmul_rn(floorf(__fmul_rn(l, inv)), a.dl);
        mx[c] = h;
        a.origin[3 * b + c] = org[c];
    }
    a.nxy[2 * b] = f2size(floorf(__fdiv_rn(__fsub_rn(mx[0], org[0]), a.dl))) + 1ull;
    a.nxy[2 * b + 1] = f2size(floorf(__fdiv_rn(__fsub_rn(mx[1], org[1]), a.dl))) + 1ull;
}

// grid_subsampling.cpp :50-54
__global__ void gs_key(GsArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.off[a.nb]) return;
    const int b = batch_of(a.off, a.nb, i);
    const float *p = a.pts + 3 * (size_t)i;
    const float *o = a.origin + 3 * b;
    const u64 ix = f2size(floorf(__fdiv_rn(__fsub_rn(p[0], o[0]), a.dl)));
    const u64 iy = f2size(floorf(__fdiv_rn(__fsub_rn(p[1], o[1]), a.dl)));
    const u64 iz = f2size(floorf(__fdiv_rn(__fsub_rn(p[2], o[2]), a.dl)));
    const u64 nx = a.nxy[2 * b], ny = a.nxy[2 * b + 1];
    const u64 k = (ix + nx * iy) + (nx * ny) * iz;
    a.key[i] = k;
    a.bat[i] = b;
    atomicMax(a.maxkey, k);
}

__global__ void gs_compose(const u64 *key, const int *bat, int n, int kbits, u64 *ck, int *iota) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    ck[i] = kbits < 64 ? (((u64)bat[i] << kbits) | key[i]) : key[i];
    iota[i] = i;
}

__global__ void gs_batch_key(const int *bat, const int *v, int n, u64 *ck) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ck[i] = (u64)bat[v[i]];
}

// run heads of the (batch, key)-sorted points
__global__ void gs_heads(const u64 *key, const int *bat, const int *v, int n, unsigned char *head) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int a = v[i];
    head[i] = (i == 0) || bat[a] != bat[v[i - 1]] || key[a] != key[v[i - 1]];
}

// mark[first point of voxel] = voxel id (the sort is stable: a run's first
// entry is its lowest input index)
__global__ void gs_mark(const int *start, const int *v, int V, int *mark) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < V) mark[v[start[r]]] = r;
}

struct NonNeg {
    __device__ bool operator()(int x) const { return x >= 0; }
};

__global__ void gs_okey(const int *list, const int *start, const int *v, const u64 *key,
                        const int *bat, int V, u64 *okey, int *obat) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= V) return;
    const int first = v[start[list[r]]];
    okey[r] = key[first];
    obat[r] = bat[first];
}

// barycentres and mean features, written to their output slot: sums in input
// order from zero (SampledData::update_* :41-79), then point * (float)(1.0 /
// count) and f / (float)count (grid_subsampling.cpp :86-95)
__global__ void gs_emit(GsArgs a, const int *outr, int total, const int *list, const int *start,
                        const int *v, float *out_pts, float *out_feat) {
    const int pos = blockIdx.x * blockDim.x + threadIdx.x;
    if (pos >= total) return;
    const int vox = list[outr[pos]];
    const int s0 = start[vox], s1 = start[vox + 1];
    float sx = 0.0f, sy = 0.0f, sz = 0.0f;
    for (int s = s0; s < s1; ++s) {
        const float *p = a.pts + 3 * (size_t)v[s];
        sx = __fadd_rn(sx, p[0]);
        sy = __fadd_rn(sy, p[1]);
        sz = __fadd_rn(sz, p[2]);
    }
    const int cnt = s1 - s0;
    const float sc = (float)(1.0 / (double)cnt);
    out_pts[3 * (size_t)pos] = __fmul_rn(sx, sc);
    out_pts[3 * (size_t)pos + 1] = __fmul_rn(sy, sc);
    out_pts[3 * (size_t)pos + 2] = __fmul_rn(sz, sc);
    if (a.feat && out_feat) {
        const float fc = (float)cnt;
        for (int d = 0; d < a.fdim; ++d) {
            float f = 0.0f;
            for (int s = s0; s < s1; ++s) f = __fadd_rn(f, a.feat[(size_t)v[s] * a.fdim + d]);
            out_feat[(size_t)pos * a.fdim + d] = __fdiv_rn(f, fc);
        }
    }
}

inline unsigned nbits(u64 x) { return x ? 64u - (unsigned)__builtin_clzll(x) : 0u; }

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// carve a workspace slot into aligned sub-buffers
struct Carver {
    size_t used = 0;
    template <class T> size_t take(size_t count) {
        const size_t at = used;
        used = align256(used + sizeof(T) * (count > 0 ? count : 1));
        return at;
    }
};

// ---------------------------------------------------------------------------
// radius neighbours
// ---------------------------------------------------------------------------

struct RnArgs {
    const float *q, *s;
    int nq, ns, nb;
    const int *qoff, *soff;  // [nb+1]
    float r2;
    double ic;               // 1 / cell, 0 = no grid (radius 0 / NaN)
    int S;
    int *bad;                // some finite support is too far out for int cell coords
    int *hcnt, *start;       // [S], [S+1]
    float4 *cell_pts;        // [ns] (x, y, z, global support index)
    int *counts;             // [nq]
    int *maxcnt;
    u64 *total;              // sum of counts
    const unsigned *offs;    // [nq+1] exclusive scan of counts
    u64 *keys;               // [total]
    int ibits;
    float r2lo;              // d in [r2lo, r2): near-radius row, replayed on the host
    int *bcnt, *blist;       // near-radius rows (pass 1)
    int *tcnt, *tlist;       // rows with an equal-distance pair (after the sort)
};

constexpr double kCoordLimit = 1073741824.0;  // 2^30

__device__ __forceinline__ unsigned rhash(int b, int x, int y, int z, int S) {
    return (((unsigned)x * 73856093u) ^ ((unsigned)y * 19349663u) ^ ((unsigned)z * 83492791u) ^
            ((unsigned)b * 2654435761u)) & (unsigned)(S - 1);
}

__device__ __forceinline__ bool cell_of(const float *p, double ic, int &x, int &y, int &z) {
    const double u = (double)p[0] * ic, v = (double)p[1] * ic, w = (double)p[2] * ic;
    if (!(fabs(u) < kCoordLimit && fabs(v) < kCoordLimit && fabs(w) < kCoordLimit)) return false;
    x = (int)floor(u); y = (int)floor(v); z = (int)floor(w);
    return true;
}

__device__ __forceinline__ bool finite3(const float *p) {
    return __builtin_isfinite(p[0]) && __builtin_isfinite(p[1]) && __builtin_isfinite(p[2]);
}

template <bool SCATTER>
__global__ void rn_grid(RnArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.soff[a.nb]) return;
    const float *p = a.s + 3 * (size_t)i;
    if (!finite3(p)) return;  // d is NaN / inf against every query: never a neighbour
    int x, y, z;
    if (!cell_of(p, a.ic, x, y, z)) {
        if (!SCATTER) atomicOr(a.bad, 1);
        return;
    }
    const unsigned h = rhash(batch_of(a.soff, a.nb, i), x, y, z, a.S);
    if (!SCATTER) {
        atomicAdd(a.hcnt + h, 1);
    } else {
        const int pos = a.start[h] + atomicAdd(a.hcnt + h, 1);
        a.cell_pts[pos] = make_float4(p[0], p[1], p[2], __int_as_float(i));
    }
}

// neighbors.cpp / nanoflann L2_Simple_Adaptor::evalMetric: diff = q - s, f32
__device__ __forceinline__ float rdist(float qx, float qy, float qz, float sx, float sy, float sz) {
    const float dx = __fsub_rn(qx, sx), dy = __fsub_rn(qy, sy), dz = __fsub_rn(qz, sz);
    return __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
}

template <bool FILL>
__global__ __launch_bounds__(256) void rn_query(RnArgs a) {
    const int qi0 = blockIdx.x * blockDim.x + threadIdx.x;
    if (FILL && qi0 >= a.nq) return;
    const bool live = qi0 < a.nq;
    const int qi = live ? qi0 : a.nq - 1;  // idle lanes join the count reduction with 0
    const int b = batch_of(a.qoff, a.nb, qi);
    const int s0 = a.soff[b], s1 = a.soff[b + 1];
    const float *qp = a.q + 3 * (size_t)qi;
    const float qx = qp[0], qy = qp[1], qz = qp[2];
    int cnt = 0;
    bool edge = false;
    u64 *out = nullptr;
    if (FILL) out = a.keys + a.offs[qi];
    auto take = [&](float d, int j) {
        if (live && d < a.r2) {
            if (FILL) out[cnt] = ((u64)__float_as_uint(d) << a.ibits) | (u64)(unsigned)j;
            ++cnt;
            edge |= d >= a.r2lo;
        }
    };
    int cx, cy, cz;
    const bool grid = a.ic > 0.0 && !*a.bad && cell_of(qp, a.ic, cx, cy, cz);
    if (a.ic > 0.0 && !grid && finite3(qp)) {
        // far outside the integer cell range: every support of the batch
        for (int j = s0; j < s1; ++j) {
            const float *sp = a.s + 3 * (size_t)j;
            take(rdist(qx, qy, qz, sp[0], sp[1], sp[2]), j);
        }
    } else if (grid) {
        unsigned h[27];
#pragma unroll
        for (int k = 0; k < 27; ++k) h[k] = rhash(b, cx + k % 3 - 1, cy + (k / 3) % 3 - 1, cz + k / 9 - 1, a.S);
#pragma unroll
        for (int k = 0; k < 27; ++k) {
            bool dup = false;
#pragma unroll
            for (int j = 0; j < k; ++j) dup |= h[j] == h[k];
            if (dup) continue;
            const int e = a.start[h[k] + 1];
            for (int t = a.start[h[k]]; t < e; ++t) {
                const float4 p = a.cell_pts[t];
                const int j = __float_as_int(p.w);
                if (j < s0 || j >= s1) continue;  // another batch hashed into the slot
                take(rdist(qx, qy, qz, p.x, p.y, p.z), j);
            }
        }
    }
    if (!FILL) {
        if (live && edge) a.blist[atomicAdd(a.bcnt, 1)] = qi;
        if (live) a.counts[qi] = cnt;
        atomicMax(a.maxcnt, cnt);
        u64 t = (u64)cnt;
        for (int o = 32; o; o >>= 1) t += __shfl_xor(t, o, 64);
        if ((threadIdx.x & 63) == 0) atomicAdd(a.total, t);
    }
}

// rows whose sorted keys hold two equal distances (d > 0: the reference's own
// order decides them)
__global__ void rn_ties(const u64 *keys, const unsigned *offs, const int *counts, int nq, int ibits,
                        int *tcnt, int *tlist) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const u64 *k = keys + offs[q];
    const int c = counts[q];
    for (int j = 1; j < c; ++j)
        if ((k[j] >> ibits) == (k[j - 1] >> ibits)) {
            tlist[atomicAdd(tcnt, 1)] = q;
            return;
        }
}

__global__ void rn_emit(const u64 *keys, const unsigned *offs, const int *counts, int nq, int width,
                        int ns, unsigned lowmask, int32_t *out) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)nq * width) return;
    const int q = (int)(t / (unsigned)width), j = (int)(t - (size_t)q * width);
    out[t] = j < counts[q] ? (int32_t)(keys[offs[q] + j] & lowmask) : ns;
}

// The reference's batch walk (neighbors.cpp :268-286) advances at most one batch
// per query, so a query batch of length 0 other than the first or trailing ones
// leaves the following queries on the wrong batch.  Returns false there and
// when the lengths do not sum to nq.
bool query_offsets(const int32_t *qb, int nb, int nq, std::vector<int> &qoff) {
    qoff.assign(nb + 1, 0);
    for (int b = 0; b < nb; ++b) qoff[b + 1] = qoff[b] + qb[b];
    if (qoff[nb] != nq) return false;
    int b = 0, i0 = 0;
    while (i0 < nq) {
        if (i0 == qoff[b] + qb[b]) ++b;  // the single advance per query
        if (b >= nb || qoff[b + 1] <= i0) return false;
        i0 = qoff[b + 1];
    }
    return true;
}

struct RnPlan {
    RnArgs a;
    std::vector<int> qoff, soff;
    void *tmp;
    size_t tmp_bytes;
};

// validation, grid build (count -> scan -> scatter), pass 1 (counts, max, total)
int rn_prepare(const float *q, int nq, const float *s, int ns, const int32_t *qb, const int32_t *sb,
               int nb, float radius, hipStream_t st, RnPlan &P) {
    PCR_REQUIRE(nq >= 0 && ns >= 0 && nb >= 1, PCR_ERR_ARG, "radius_neighbors: bad sizes");
    PCR_REQUIRE(qb && sb, PCR_ERR_ARG, "radius_neighbors: null batch lengths");
    PCR_REQUIRE((q || nq == 0) && (s || ns == 0), PCR_ERR_ARG, "radius_neighbors: null points");
    for (int b = 0; b < nb; ++b)
        PCR_REQUIRE(qb[b] >= 0 && sb[b] >= 0, PCR_ERR_ARG, "radius_neighbors: negative batch length");
    PCR_REQUIRE(query_offsets(qb, nb, nq, P.qoff), PCR_ERR_ARG,
                "radius_neighbors: query batches must sum to the query count, with empty batches "
                "only first or last (the reference's batch walk, neighbors.cpp:268-286, "
                "misassigns queries otherwise)");
    P.soff.assign(nb + 1, 0);
    for (int b = 0; b < nb; ++b) P.soff[b + 1] = P.soff[b] + sb[b];
    PCR_REQUIRE(P.soff[nb] <= ns, PCR_ERR_ARG,
                "radius_neighbors: support batches sum to %d > %d supports", P.soff[nb], ns);
    RnArgs &a = P.a;
    a = RnArgs{};
    a.q = q; a.s = s; a.nq = nq; a.ns = ns; a.nb = nb;
    a.r2 = radius * radius;  // neighbors.cpp :226, f32
    a.r2lo = (float)((double)a.r2 * (1.0 - 1.0 / 131072.0));
    const double cell = fabs((double)radius) * (1.0 + 1e-6);
    a.ic = (a.r2 > 0.0f && cell < 1e300) ? 1.0 / cell : 0.0;
    int S = 1024;
    while (S < 2 * ns) S <<= 1;
    a.S = S;
    a.ibits = (int)nbits((u64)(ns > 0 ? ns : 1));
    Carver c;
    const size_t o_off = c.take<int>(2 * (nb + 1)), o_hdr = c.take<u64>(3), o_h = c.take<int>(S + 1),
                 o_st = c.take<int>(S + 1), o_pts = c.take<float4>(ns), o_cnt = c.take<int>(nq),
                 o_offs = c.take<unsigned>(nq + 1), o_bl = c.take<int>(nq), o_tl = c.take<int>(nq);
    char *ws = (char *)workspace(18, c.used);
    PCR_REQUIRE(ws, PCR_ERR_NOMEM, "radius_neighbors: %s", pcr_last_error());
    int *dev_off = (int *)(ws + o_off);
    a.qoff = dev_off; a.soff = dev_off + nb + 1;
    a.total = (u64 *)(ws + o_hdr);
    a.bad = (int *)(a.total + 1); a.maxcnt = a.bad + 1;
    a.bcnt = (int *)(a.total + 2); a.tcnt = a.bcnt + 1;
    a.blist = (int *)(ws + o_bl); a.tlist = (int *)(ws + o_tl);
    a.hcnt = (int *)(ws + o_h); a.start = (int *)(ws + o_st);
    a.cell_pts = (float4 *)(ws + o_pts);
    a.counts = (int *)(ws + o_cnt);
    a.offs = (const unsigned *)(ws + o_offs);
    std::vector<int> offs(P.qoff);
    offs.insert(offs.end(), P.soff.begin(), P.soff.end());
    PCR_HIP_CHECK(hipMemcpyAsync(dev_off, offs.data(), sizeof(int) * offs.size(), hipMemcpyHostToDevice, st));
    PCR_HIP_CHECK(hipMemsetAsync(a.total, 0, 3 * sizeof(u64), st));
    size_t tb = 0, tb2 = 0;
    PCR_HIP_CHECK(rocprim::exclusive_scan(nullptr, tb, a.hcnt, a.start, 0, (size_t)S + 1,
                                          rocprim::plus<int>(), st));
    PCR_HIP_CHECK(rocprim::exclusive_scan(nullptr, tb2, (const int *)a.counts, (unsigned *)a.offs, 0u,
                                          (size_t)nq + 1, rocprim::plus<unsigned>(), st));
    tb = tb > tb2 ? tb : tb2;
    P.tmp = workspace(19, tb);
    P.tmp_bytes = tb;
    PCR_REQUIRE(P.tmp, PCR_ERR_NOMEM, "radius_neighbors: %s", pcr_last_error());
    if (a.ic > 0.0 && ns > 0) {
        PCR_HIP_CHECK(hipMemsetAsync(a.hcnt, 0, sizeof(int) * (S + 1), st));
        const int gs = (P.soff[nb] + 255) / 256;
        if (gs > 0) hipLaunchKernelGGL(rn_grid<false>, dim3(gs), dim3(256), 0, st, a);
        PCR_LAUNCH_CHECK();
        size_t t = tb;
        PCR_HIP_CHECK(rocprim::exclusive_scan(P.tmp, t, a.hcnt, a.start, 0, (size_t)S + 1,
                                              rocprim::plus<int>(), st));
        PCR_HIP_CHECK(hipMemsetAsync(a.hcnt, 0, sizeof(int) * S, st));
        if (gs > 0) hipLaunchKernelGGL(rn_grid<true>, dim3(gs), dim3(256), 0, st, a);
        PCR_LAUNCH_CHECK();
    }
    if (nq > 0) {
        hipLaunchKernelGGL(rn_query<false>, dim3((nq + 255) / 256), dim3(256), 0, st, a);
        PCR_LAUNCH_CHECK();
    }
    return PCR_OK;
}

// host copies of the queries / supports, fetched only when a row needs the replay
struct RnHost {
    std::vector<float> q, s;
    bool loaded = false;
};

int rn_fetch(const RnPlan &P, hipStream_t st, RnHost &H) {
    if (H.loaded) return PCR_OK;
    H.q.resize(3 * (size_t)P.a.nq);
    H.s.resize(3 * (size_t)P.a.ns);
    if (P.a.nq) PCR_HIP_CHECK(hipMemcpyAsync(H.q.data(), P.a.q, 12 * (size_t)P.a.nq, hipMemcpyDeviceToHost, st));
    if (P.a.ns) PCR_HIP_CHECK(hipMemcpyAsync(H.s.data(), P.a.s, 12 * (size_t)P.a.ns, hipMemcpyDeviceToHost, st));
    PCR_HIP_CHECK(hipStreamSynchronize(st));
    H.loaded = true;
    return PCR_OK;
}

// the reference's neighbour lists of `rows` (ascending), recomputed on the host
int rn_replay(const RnPlan &P, hipStream_t st, RnHost &H, const std::vector<int> &rows,
              std::vector<std::vector<int>> &res) {
    const int rc = rn_fetch(P, st, H);
    if (rc != PCR_OK) return rc;
    std::vector<int> qb(rows.size());
    for (size_t k = 0; k < rows.size(); ++k)
        qb[k] = (int)(std::upper_bound(P.qoff.begin(), P.qoff.end(), rows[k]) - P.qoff.begin()) - 1;
    kd_replay_rows(H.q.data(), H.s.data(), P.soff.data(), rows, qb, P.a.r2, res);
    return PCR_OK;
}

// pass-1 epilogue: exact counts of the near-radius rows and the reference's
// max_count (hdr = the synchronized header)
int rn_boundary(const RnPlan &P, hipStream_t st, const u64 *hdr, RnHost &H, std::vector<int> &rows,
                std::vector<std::vector<int>> &res, int &max_count) {
    max_count = (int)(hdr[1] >> 32);
    rows.assign((size_t)(hdr[2] & 0xffffffffu), 0);
    res.clear();
    if (rows.empty()) return PCR_OK;
    std::vector<int> cnt((size_t)P.a.nq);
    PCR_HIP_CHECK(hipMemcpyAsync(rows.data(), P.a.blist, sizeof(int) * rows.size(), hipMemcpyDeviceToHost, st));
    PCR_HIP_CHECK(hipMemcpyAsync(cnt.data(), P.a.counts, sizeof(int) * cnt.size(), hipMemcpyDeviceToHost, st));
    PCR_HIP_CHECK(hipStreamSynchronize(st));
    std::sort(rows.begin(), rows.end());
    const int rc = rn_replay(P, st, H, rows, res);
    if (rc != PCR_OK) return rc;
    for (size_t k = 0; k < rows.size(); ++k) cnt[rows[k]] = (int)res[k].size();
    max_count = 0;
    for (int c : cnt) max_count = c > max_count ? c : max_count;
    return PCR_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// host replay of the reference's unordered_map<size_t, SampledData> order
// ---------------------------------------------------------------------------
void voxel_map_order(const uint64_t *keys, int n, int32_t *order) {
    std::unordered_map<size_t, int> m;  // grid_subsampling.cpp :46-58: one map per cloud
    for (int r = 0; r < n; ++r) m.emplace((size_t)keys[r], r);
    int k = 0;
    for (const auto &kv : m) order[k++] = kv.second;  // :84 for (auto& v : data)
}

}  // namespace pcr

extern "C" int pcr_voxel_map_order(const uint64_t *keys, int32_t n, int32_t *order) {
    pcr::clear_error();
    PCR_REQUIRE(n >= 0 && (n == 0 || (keys && order)), PCR_ERR_ARG, "voxel_map_order: bad arguments");
    pcr::voxel_map_order(keys, n, order);
    return PCR_OK;
}

extern "C" int pcr_grid_subsample(const float *points, int32_t n, const int32_t *batch_len,
                                  int32_t nb, const float *features, int32_t fdim, float dl,
                                  int32_t max_p, float *out_points, float *out_features,
                                  int32_t *out_batch_len, int32_t *out_total, pcr_stream_t stream) {
    using namespace pcr;
    clear_error();
    PCR_REQUIRE(n >= 0 && nb >= 1 && fdim >= 0 && batch_len && out_batch_len && out_total, PCR_ERR_ARG,
                "grid_subsample: bad arguments");
    PCR_REQUIRE(!(fdim > 0) || features, PCR_ERR_ARG, "grid_subsample: fdim > 0 without features");
    PCR_REQUIRE(n == 0 || (points && out_points), PCR_ERR_ARG, "grid_subsample: null points");
    PCR_REQUIRE(__builtin_isfinite(dl) && dl > 0.0f, PCR_ERR_ARG, "grid_subsample: sampleDl must be a positive float");
    std::vector<int> off(nb + 1, 0);
    for (int b = 0; b < nb; ++b) {
        PCR_REQUIRE(batch_len[b] >= 0, PCR_ERR_ARG, "grid_subsample: negative batch length");
        off[b + 1] = off[b] + batch_len[b];
    }
    // batch_grid_subsampling.cpp :140-145 reads past the cloud when the lengths
    // overrun it; trailing points beyond the batches are ignored, as there
    PCR_REQUIRE(off[nb] <= n, PCR_ERR_ARG, "grid_subsample: batches sum to %d > %d points", off[nb], n);
    const int N = off[nb];
    *out_total = 0;
    for (int b = 0; b < nb; ++b) out_batch_len[b] = 0;
    if (N == 0) return PCR_OK;
    hipStream_t st = as_stream(stream);
    Carver c;
    const size_t o_off = c.take<int>(nb + 1), o_org = c.take<float>(3 * nb), o_nxy = c.take<u64>(2 * nb),
                 o_mk = c.take<u64>(2), o_key = c.take<u64>(N), o_bat = c.take<int>(N),
                 o_ck = c.take<u64>(N), o_ck2 = c.take<u64>(N), o_iota = c.take<int>(N),
                 o_v = c.take<int>(N), o_v2 = c.take<int>(N), o_head = c.take<unsigned char>(N),
                 o_start = c.take<int>(N + 1), o_mark = c.take<int>(N), o_list = c.take<int>(N),
                 o_okey = c.take<u64>(N), o_obat = c.take<int>(N), o_outr = c.take<int>(N),
                 o_cnt = c.take<int>(2);
    char *ws = (char *)workspace(16, c.used);
    PCR_REQUIRE(ws, PCR_ERR_NOMEM, "grid_subsample: %s", pcr_last_error());
    GsArgs a;
    a.pts = points; a.feat = fdim > 0 ? features : nullptr; a.n = N; a.fdim = fdim; a.nb = nb;
    a.off = (int *)(ws + o_off); a.dl = dl;
    a.origin = (float *)(ws + o_org); a.nxy = (u64 *)(ws + o_nxy);
    a.maxkey = (u64 *)(ws + o_mk); a.bad = (int *)(a.maxkey + 1);
    a.key = (u64 *)(ws + o_key); a.bat = (int *)(ws + o_bat);
    u64 *ck = (u64 *)(ws + o_ck), *ck2 = (u64 *)(ws + o_ck2);
    int *iota = (int *)(ws + o_iota), *v = (int *)(ws + o_v), *v2 = (int *)(ws + o_v2);
    unsigned char *head = (unsigned char *)(ws + o_head);
    int *start = (int *)(ws + o_start), *mark = (int *)(ws + o_mark), *list = (int *)(ws + o_list);
    u64 *okey = (u64 *)(ws + o_okey);
    int *obat = (int *)(ws + o_obat), *outr = (int *)(ws + o_outr), *dcnt = (int *)(ws + o_cnt);

    PCR_HIP_CHECK(hipMemcpyAsync((void *)a.off, off.data(), sizeof(int) * (nb + 1), hipMemcpyHostToDevice, st));
    PCR_HIP_CHECK(hipMemsetAsync(a.maxkey, 0, 2 * sizeof(u64), st));
    hipLaunchKernelGGL(gs_bbox, dim3(nb), dim3(256), 0, st, a);
    PCR_LAUNCH_CHECK();
    const dim3 gN((N + 255) / 256), blk(256);
    hipLaunchKernelGGL(gs_key, gN, blk, 0, st, a);
    PCR_LAUNCH_CHECK();
    u64 hk[2];
    PCR_HIP_CHECK(hipMemcpyAsync(hk, a.maxkey, sizeof(hk), hipMemcpyDeviceToHost, st));
    PCR_HIP_CHECK(hipStreamSynchronize(st));
    PCR_REQUIRE(!(int)hk[1], PCR_ERR_ARG,
                "grid_subsample: non-finite point coordinates (the reference's voxel index is undefined there)");
    const unsigned kbits = nbits(hk[0]) ? nbits(hk[0]) : 1u, bbits = nbits((u64)(nb - 1));

    // stable radix sort by (batch, key): input order kept inside a voxel
    size_t tb = 0, t1 = 0;
    PCR_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, t1, ck, ck2, iota, v, N, 0, 64, st));
    tb = t1;
    PCR_HIP_CHECK(rocprim::select(nullptr, t1, rocprim::counting_iterator<int>(0), head, start, dcnt, (size_t)N, st));
    tb = tb > t1 ? tb : t1;
    PCR_HIP_CHECK(rocprim::select(nullptr, t1, mark, list, dcnt + 1, (size_t)N, NonNeg(), st));
    tb = tb > t1 ? tb : t1;
    void *tmp = workspace(17, tb);
    PCR_REQUIRE(tmp, PCR_ERR_NOMEM, "grid_subsample: %s", pcr_last_error());
    if (kbits + bbits <= 64) {
        hipLaunchKernelGGL(gs_compose, gN, blk, 0, st, a.key, a.bat, N, (int)kbits, ck, iota);
        PCR_LAUNCH_CHECK();
        t1 = tb;
        PCR_HIP_CHECK(rocprim::radix_sort_pairs(tmp, t1, ck, ck2, iota, v, N, 0, kbits + bbits, st));
    } else {  // keys wider than the composite: LSD in two stable passes
        hipLaunchKernelGGL(gs_compose, gN, blk, 0, st, a.key, a.bat, N, 64, ck, iota);
        PCR_LAUNCH_CHECK();
        t1 = tb;
        PCR_HIP_CHECK(rocprim::radix_sort_pairs(tmp, t1, ck, ck2, iota, v2, N, 0, kbits, st));
        hipLaunchKernelGGL(gs_batch_key, gN, blk, 0, st, a.bat, v2, N, ck);
        PCR_LAUNCH_CHECK();
        t1 = tb;
        PCR_HIP_CHECK(rocprim::radix_sort_pairs(tmp, t1, ck, ck2, v2, v, N, 0, bbits ? bbits : 1u, st));
    }
    hipLaunchKernelGGL(gs_heads, gN, blk, 0, st, a.key, a.bat, v, N, head);
    PCR_LAUNCH_CHECK();
    t1 = tb;
    PCR_HIP_CHECK(rocprim::select(tmp, t1, rocprim::counting_iterator<int>(0), head, start, dcnt, (size_t)N, st));
    int V = 0;
    PCR_HIP_CHECK(hipMemcpyAsync(&V, dcnt, sizeof(int), hipMemcpyDeviceToHost, st));
    PCR_HIP_CHECK(hipStreamSynchronize(st));
    PCR_HIP_CHECK(hipMemcpyAsync(start + V, &N, sizeof(int), hipMemcpyHostToDevice, st));
    PCR_HIP_CHECK(hipMemsetAsync(mark, 0xFF, sizeof(int) * N, st));
    const dim3 gV((V + 255) / 256);
    hipLaunchKernelGGL(gs_mark, gV, blk, 0, st, start, v, V, mark);
    PCR_LAUNCH_CHECK();
    t1 = tb;
    PCR_HIP_CHECK(rocprim::select(tmp, t1, mark, list, dcnt + 1, (size_t)N, NonNeg(), st));
    hipLaunchKernelGGL(gs_okey, gV, blk, 0, st, list, start, v, a.key, a.bat, V, okey, obat);
    PCR_LAUNCH_CHECK();
    std::vector<u64> hkey(V);
    std::vector<int> hbat(V), hout;
    PCR_HIP_CHECK(hipMemcpyAsync(hkey.data(), okey, sizeof(u64) * V, hipMemcpyDeviceToHost, st));
    PCR_HIP_CHECK(hipMemcpyAsync(hbat.data(), obat, sizeof(int) * V, hipMemcpyDeviceToHost, st));
    PCR_HIP_CHECK(hipStreamSynchronize(st));
    // per cloud: the map's iteration order, truncated to max_p (:180-204)
    const int cap = max_p < 1 ? n : max_p;  // :134-135 (N = all points of the call)
    hout.reserve(V);
    std::vector<int32_t> ord(V);
    for (int r0 = 0; r0 < V;) {
        int r1 = r0;
        while (r1 < V && hbat[r1] == hbat[r0]) ++r1;
        voxel_map_order(reinterpret_cast<const uint64_t *>(hkey.data()) + r0, r1 - r0, ord.data() + r0);
        const int take = (r1 - r0) < cap ? (r1 - r0) : cap;
        for (int k = 0; k < take; ++k) hout.push_back(r0 + ord[r0 + k]);
        out_batch_len[hbat[r0]] = take;
        r0 = r1;
    }
    const int total = (int)hout.size();
    PCR_HIP_CHECK(hipMemcpyAsync(outr, hout.data(), sizeof(int) * total, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(gs_emit, dim3((total + 255) / 256), blk, 0, st, a, outr, total, list, start, v,
                       out_points, fdim > 0 ? out_features : nullptr);
    PCR_LAUNCH_CHECK();
    PCR_HIP_CHECK(hipStreamSynchronize(st));  // hout is a host temporary
    *out_total = total;
    return PCR_OK;
}

extern "C" int pcr_radius_count(const float *queries, int32_t nq, const float *supports, int32_t ns,
                                const int32_t *q_batches, const int32_t *s_batches, int32_t nb,
                                float radius, int32_t *counts, int32_t *max_count,
                                pcr_stream_t stream) {
    using namespace pcr;
    clear_error();
    PCR_REQUIRE(max_count, PCR_ERR_ARG, "radius_count: null max_count");
    hipStream_t st = as_stream(stream);
    RnPlan P;
    const int rc = rn_prepare(queries, nq, supports, ns, q_batches, s_batches, nb, radius, st, P);
    if (rc != PCR_OK) return rc;
    if (counts && nq > 0)
        PCR_HIP_CHECK(hipMemcpyAsync(counts, P.a.counts, sizeof(int) * nq, hipMemcpyDeviceToDevice, st));
    u64 hdr[3];
    PCR_HIP_CHECK(hipMemcpyAsync(hdr, P.a.total, sizeof(hdr), hipMemcpyDeviceToHost, st));
    PCR_HIP_CHECK(hipStreamSynchronize(st));
    RnHost H;
    std::vector<int> brows;
    std::vector<std::vector<int>> bres;
    int mc = 0;
    const int rb = rn_boundary(P, st, hdr, H, brows, bres, mc);
    if (rb != PCR_OK) return rb;
    *max_count = mc;
    if (counts && !brows.empty()) {
        std::vector<int> bc(brows.size());
        for (size_t k = 0; k < brows.size(); ++k) {
            bc[k] = (int)bres[k].size();
            PCR_HIP_CHECK(hipMemcpyAsync(counts + brows[k], &bc[k], sizeof(int), hipMemcpyHostToDevice, st));
        }
        PCR_HIP_CHECK(hipStreamSynchronize(st));
    }
    return PCR_OK;
}

extern "C" int pcr_radius_neighbors(const float *queries, int32_t nq, const float *supports, int32_t ns,
                                    const int32_t *q_batches, const int32_t *s_batches, int32_t nb,
                                    float radius, int32_t width, int32_t *out, int32_t *max_count,
                                    pcr_stream_t stream) {
    using namespace pcr;
    clear_error();
    PCR_REQUIRE(width >= 0 && (out || (size_t)nq * width == 0), PCR_ERR_ARG, "radius_neighbors: bad output");
    hipStream_t st = as_stream(stream);
    RnPlan P;
    int rc = rn_prepare(queries, nq, supports, ns, q_batches, s_batches, nb, radius, st, P);
    if (rc != PCR_OK) return rc;
    u64 hdr[3];
    PCR_HIP_CHECK(hipMemcpyAsync(hdr, P.a.total, sizeof(hdr), hipMemcpyDeviceToHost, st));
    PCR_HIP_CHECK(hipStreamSynchronize(st));
    const u64 total = hdr[0];
    RnHost H;
    std::vector<int> brows;
    std::vector<std::vector<int>> bres;
    int mc = 0;
    rc = rn_boundary(P, st, hdr, H, brows, bres, mc);
    if (rc != PCR_OK) return rc;
    if (max_count) *max_count = mc;
    const size_t cells = (size_t)nq * width;
    if (cells == 0) return PCR_OK;
    PCR_REQUIRE(total < 0xFFFFFFFFull, PCR_ERR_ARG, "radius_neighbors: %llu neighbour pairs exceed 2^32",
                (unsigned long long)total);
    // pass 2: offsets, (d, index) keys, per-query sort, padded rows
    size_t t1 = P.tmp_bytes;
    PCR_HIP_CHECK(rocprim::exclusive_scan(P.tmp, t1, (const int *)P.a.counts, (unsigned *)P.a.offs, 0u,
                                          (size_t)nq + 1, rocprim::plus<unsigned>(), st));
    u64 *keys2 = nullptr;
    if (total > 0) {
        const unsigned ebit = 31u + (unsigned)P.a.ibits;
        size_t tb = 0;
        PCR_HIP_CHECK(rocprim::segmented_radix_sort_keys(nullptr, tb, (const u64 *)nullptr, (u64 *)nullptr,
                                                         (unsigned)total, (unsigned)nq, P.a.offs, P.a.offs + 1,
                                                         0u, ebit, st));
        Carver c;
        const size_t o_k = c.take<u64>(total), o_k2 = c.take<u64>(total), o_t = c.take<char>(tb);
        char *ws = (char *)workspace(20, c.used);
        PCR_REQUIRE(ws, PCR_ERR_NOMEM, "radius_neighbors: %s", pcr_last_error());
        P.a.keys = (u64 *)(ws + o_k);
        keys2 = (u64 *)(ws + o_k2);
        hipLaunchKernelGGL(rn_query<true>, dim3((nq + 255) / 256), dim3(256), 0, st, P.a);
        PCR_LAUNCH_CHECK();
        PCR_HIP_CHECK(rocprim::segmented_radix_sort_keys(ws + o_t, tb, (const u64 *)P.a.keys, keys2,
                                                         (unsigned)total, (unsigned)nq, P.a.offs, P.a.offs + 1,
                                                         0u, ebit, st));
        hipLaunchKernelGGL(rn_ties, dim3((nq + 255) / 256), dim3(256), 0, st, (const u64 *)keys2, P.a.offs,
                           (const int *)P.a.counts, nq, P.a.ibits, P.a.tcnt, P.a.tlist);
        PCR_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(rn_emit, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, st, keys2, P.a.offs,
                       P.a.counts, nq, width, ns, (unsigned)((1ull << P.a.ibits) - 1), out);
    PCR_LAUNCH_CHECK();
    if (total == 0) return PCR_OK;
    // rows the distance sort cannot decide: the reference's own order, from the host
    int ntie = 0;
    PCR_HIP_CHECK(hipMemcpyAsync(&ntie, P.a.tcnt, sizeof(int), hipMemcpyDeviceToHost, st));
    PCR_HIP_CHECK(hipStreamSynchronize(st));
    std::vector<int> rows(brows);
    std::vector<std::vector<int>> res(bres);
    if (ntie > 0) {
        std::vector<int> trows((size_t)ntie);
        PCR_HIP_CHECK(hipMemcpyAsync(trows.data(), P.a.tlist, sizeof(int) * trows.size(), hipMemcpyDeviceToHost, st));
        PCR_HIP_CHECK(hipStreamSynchronize(st));
        std::sort(trows.begin(), trows.end());
        std::vector<int> extra;
        std::set_difference(trows.begin(), trows.end(), brows.begin(), brows.end(), std::back_inserter(extra));
        std::vector<std::vector<int>> eres;
        rc = rn_replay(P, st, H, extra, eres);
        if (rc != PCR_OK) return rc;
        rows.insert(rows.end(), extra.begin(), extra.end());
        res.insert(res.end(), eres.begin(), eres.end());
    }
    if (rows.empty()) return PCR_OK;
    std::vector<int32_t> rowbuf(rows.size() * (size_t)width);
    for (size_t k = 0; k < rows.size(); ++k) {
        int32_t *r = rowbuf.data() + k * width;
        for (int j = 0; j < width; ++j) r[j] = j < (int)res[k].size() ? res[k][j] : ns;
        PCR_HIP_CHECK(hipMemcpyAsync(out + (size_t)rows[k] * width, r, sizeof(int32_t) * width,
                                     hipMemcpyHostToDevice, st));
    }
    PCR_HIP_CHECK(hipStreamSynchronize(st));
    return PCR_OK;
}
