// Hashed uniform grid over a target cloud for radius-limited 1-NN queries
// (Open3D KDTreeFlann::SearchHybrid(r, 1) semantics: nearest target with
// d2 < thr strictly, lowest index on exact ties).
//
// HBM layout per pair: pts [mstride] float4 (x, y, z, index bits) sorted by
// slot, start [S+1] u32 slot offsets.  Cells are 2.01*r wide, so a query ball
// touches at most 2x2x2 cells.  Hash collisions only add candidates; the exact
// distance test decides, so results are independent of slot order and equal to
// brute force.  Consumers that own a pair (RANSAC, ICP) copy the grid into LDS
// as one float4 per point (x, y, z, index bits) and u16 slot starts (GridP4,
// 16 B per point + 2 B per slot: 144 KiB at 8192 points).
#pragma once
#include <hip/hip_runtime.h>
#include "geom.h"


namespace pcr {

__device__ __forceinline__ int cell_coord(double v, double cell) {
    return (int)__builtin_floor(v / cell);
}

// Slot of cell (x, y, z): the three coordinates' low 10 bits packed into one
// word, then murmur3's 32-bit finaliser.  (The classic x*73856093 ^ y*19349663 ^
// z*83492791 collides on small coordinate ranges: a C4 target at d = 0.04 has
// 1,365 cells but only 1,105 distinct 32-bit values, so a RANSAC query walked
// ~56 candidates where its own cells held ~34; with this mix ~40.)  Cells 1024
// apart share a slot -- collisions only add candidates.
__device__ __forceinline__ unsigned cell_key(int x, int y, int z) {
    return ((unsigned)x & 1023u) | (((unsigned)y & 1023u) << 10) | (((unsigned)z & 1023u) << 20);
}
__device__ __forceinline__ unsigned key_slot(unsigned k, int S) {
    k ^= k >> 16;
    k *= 0x85ebca6bu;
    k ^= k >> 13;
    k *= 0xc2b2ae35u;
    k ^= k >> 16;
    return (unsigned)(((unsigned long long)k * (unsigned)S) >> 32);  // any S, not only powers of two
}
__device__ __forceinline__ unsigned cell_hash(int x, int y, int z, int S) {
    return key_slot(cell_key(x, y, z), S);
}

// view of one pair's grid in HBM: one float4 per point (x, y, z, index bits)
struct GridView {
    const float4 *pts;
    const uint32_t *start;
    int S;
    double cell;
    double inv_cell;  // queries use v * inv_cell: the 1.001 r margin covers the rounding
    // candidate access shared with GridP4: coordinates of slot s, then (only for
    // candidates inside the radius) its point index
    __device__ __forceinline__ void load(int s, float &ax, float &ay, float &az, float &aw) const {
        const float4 v = pts[s];
        ax = v.x; ay = v.y; az = v.z; aw = v.w;
    }
    __device__ __forceinline__ int index_of(int, float aw) const { return __float_as_int(aw); }
};

// LDS copy for the consumers that own a pair (RANSAC, ICP): one float4 per
// point (x, y, z, index bits) -- one ds_read_b128 and one address per
// candidate instead of four reads at four addresses -- and u16 slot starts
// (16 B per point + 2 B per slot: 144 KiB at 8192 points)
struct GridP4 {
    const float4 *pts;
    const uint16_t *start;
    int S;
    double cell;
    double inv_cell;
    __device__ __forceinline__ void load(int s, float &ax, float &ay, float &az, float &aw) const {
        const float4 v = pts[s];
        ax = v.x; ay = v.y; az = v.z; aw = v.w;
    }
    __device__ __forceinline__ int index_of(int, float aw) const { return __float_as_int(aw); }
};

// squared distance from p to cell c's box [c*cell, (c+1)*cell] along one axis,
// the box grown by a relative 1e-12 (the build assigns cells by floor(v / cell):
// a point may sit an ulp outside the multiplied bounds)
__device__ __forceinline__ double cell_gap(double p, int c, double cell) {
    const double lo = (double)c * cell, hi = (double)(c + 1) * cell;
    const double eps = 1e-12 * (__builtin_fabs(lo) + __builtin_fabs(hi) + cell);
    const double g = __builtin_fmax(__builtin_fmax((lo - eps) - p, p - (hi + eps)), 0.0);
    return g * g;
}

// The query box: cells [x0, x1] x [y0, y1] x [z0, z1] of floor(v * inv_cell) over
// [p - 1.001 r, p + 1.001 r].  The build assigns cells by floor(v / cell); the
// 0.1 % margin (w = 1.001 r inv_cell, ~0.5 cells) exceeds the rounding
// difference, so every point within r of p lies in a cell of the box.
struct QueryBox {
    int x0, x1, y0, y1, z0, z1;
};
__device__ __forceinline__ QueryBox query_box(double px, double py, double pz, double w, double ic) {
    const double ux = px * ic, uy = py * ic, uz = pz * ic;
    return QueryBox{(int)__builtin_floor(ux - w), (int)__builtin_floor(ux + w),
                    (int)__builtin_floor(uy - w), (int)__builtin_floor(uy + w),
                    (int)__builtin_floor(uz - w), (int)__builtin_floor(uz + w)};
}

// Per-axis squared gaps from p to the two cells c0, c0 + 1 of a 2-cell axis of
// the box (f32; 0 for a 1-cell axis).  Cell c0's box starts left of p and cell
// c1 = c0 + 1's ends right of it (the margin w), so the only gap along the axis
// is to the boundary B = c1 * cell: p - B for c0, B - p for c1, shrunk by a
// relative 1e-12 (the build's floor(v / cell) may put a point an ulp across B).
// The caller drops a cell when (gx + gy) + gz > thr (1 + 1e-6) in f32: the f32
// roundings (< 2^-22 relative over the sum) can only keep a cell whose box lies
// beyond r, never drop one a point within r sits in -- the candidates still
// cover every point the exact test can accept, which is all the result depends on.
__device__ __forceinline__ void axis_gaps(double p, int c0, int c1, double cell, float g[2]) {
    g[0] = 0.f;
    g[1] = 0.f;
    if (c1 != c0) {
        const double B = (double)c1 * cell;
        const double d = p - B;
        const double a = __builtin_fmax(__builtin_fabs(d) - 1e-12 * (__builtin_fabs(B) + cell), 0.0);
        const float a2 = (float)(a * a);
        if (d > 0.0) g[0] = a2;
        else g[1] = a2;
    }
}

// returns target index or -1; d2out = its squared distance.  Cells whose box
// is farther than r from p are skipped (they cannot hold a point with
// d2 < thr <= r^2 (1 + 2^-23)); candidates are taken two at a time so their
// LDS loads overlap.  The update order (slot order, strict < then lower index
// on ties) makes the result independent of both.
// kSlot: also report the winner's slot (its coordinates are g.x/y/z[slot])
// kClear (icp.hip's correspondence reuse): also report the smallest and the
// second smallest d2 computed over EVERY examined candidate (inside the radius
// or not; +inf when there are fewer) in s12out[0..1], and in s12out[2] a lower
// bound rho^2 on the squared distance from p to any target the walk did NOT
// examine: the distance to the faces of the walked block of cells and the
// gaps of its skipped cells (each shrunk by the build's rounding slack; the
// general walk reports (min(r, sqrt(thr)) (1 - 1e-6))^2).  So every target
// lies at least min(sqrt(s1), rho) from p, and every target other than the
// winner at least min(sqrt(s2), rho).
template <typename View, bool kSlot = false, int kW = 2, bool kClear = false>
__device__ __forceinline__ int grid_query_exact(const View &g, double r, double thr, double px,
                                                double py, double pz, double &d2out, int *slot = nullptr,
                                                double *s12out = nullptr) {
    const QueryBox bx = query_box(px, py, pz, 1.001 * r * g.inv_cell, g.inv_cell);
    const int x0 = bx.x0, x1 = bx.x1, y0 = bx.y0, y1 = bx.y1, z0 = bx.z0, z1 = bx.z1;
    const double lim = thr * (1.0 + 1e-9);
    double best = __builtin_inf();
    double e1 = __builtin_inf(), e2 = __builtin_inf();  // kClear: the two smallest examined d2
    auto seen = [&](double d) {
        if constexpr (kClear) {
            e2 = __builtin_fmin(e2, __builtin_fmax(e1, d));
            e1 = __builtin_fmin(e1, d);
        }
    };
    double rho2 = 0.0;
    if constexpr (kClear) {
        const double rl = __builtin_fmin(r, __builtin_sqrt(thr)) * (1.0 - 1e-6);
        rho2 = rl * rl;
    }
    int bj = -1, bs = -1;
    auto take = [&](int s) {
        float ax, ay, az, aw;
        g.load(s, ax, ay, az, aw);
        const double d2 = dist2(px, py, pz, (double)ax, (double)ay, (double)az);
        seen(d2);
        if (d2 < thr) {
            const int j = g.index_of(s, aw);
            if (d2 < best || (d2 == best && j < bj)) { best = d2; bj = j; if constexpr (kSlot) bs = s; }
        }
    };
    if (x1 - x0 <= 1 && y1 - y0 <= 1 && z1 - z0 <= 1 && g.S <= 32768) {
        // The usual case (cells 2.01 r wide, <= 32768 points): at most 2 x 2 x 2
        // cells, slot numbers below 2^16.  Their
        // slot ranges form one flat candidate sequence walked two at a time, so
        // a wave runs as long as its longest lane's TOTAL, not the sum over cells
        // of each cell's longest lane (the nested cell / slot loops did that).
        // q[k] = (lo | hi << 16) of the k-th non-empty range, queued from q[0].
        // per-axis box gaps and hash terms of the (up to) two cells per axis, computed
        // once (the cell test below adds them in the same order, (gx + gy) + gz)
        float gx[2], gy[2], gz[2];
        axis_gaps(px, x0, x1, g.cell, gx);
        axis_gaps(py, y0, y1, g.cell, gy);
        axis_gaps(pz, z0, z1, g.cell, gz);
        const float lim32 = (float)(thr * (1.0 + 1e-6));
        float skip_min = __builtin_inff();  // kClear: smallest gap^2 of a skipped cell of the block
        const unsigned hx[2] = {(unsigned)x0 & 1023u, (unsigned)(x0 + 1) & 1023u};
        const unsigned hy[2] = {((unsigned)y0 & 1023u) << 10, ((unsigned)(y0 + 1) & 1023u) << 10};
        const unsigned hz[2] = {((unsigned)z0 & 1023u) << 20, ((unsigned)(z0 + 1) & 1023u) << 20};
        unsigned q[8];
        int nq = 0, total = 0;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int ix = c >> 2, iy = (c >> 1) & 1, iz = c & 1;
            const bool inb = x0 + ix <= x1 && y0 + iy <= y1 && z0 + iz <= z1;
            const float gsum = (gx[ix] + gy[iy]) + gz[iz];
            const bool in = inb && gsum <= lim32;
            if constexpr (kClear)
                if (inb && !in) skip_min = __builtin_fminf(skip_min, gsum);
            q[c] = 0u;
            if (in) {
                const unsigned h = key_slot(hx[ix] | hy[iy] | hz[iz], g.S);
                const int lo = (int)g.start[h], hi = (int)g.start[h + 1];
                if (hi > lo) {
                    // compact: the k-th non-empty range goes to q[k]
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (k == nq) q[k] = (unsigned)lo | ((unsigned)hi << 16);
                    ++nq;
                    total += hi - lo;
                }
            }
        }
        if constexpr (kClear) {
            // faces of the walked block [x0, x1+1] x ... (cells by floor(v / cell):
            // the relative 1e-12 slack of axis_gaps), then the skipped cells (f32
            // sums of f32-rounded squares: -2^-20 relative covers them)
            auto face = [&](double p, int c0, int c1) {
                const double lo = (double)c0 * g.cell, hi = (double)(c1 + 1) * g.cell;
                const double eps = 1e-12 * (__builtin_fabs(lo) + __builtin_fabs(hi) + g.cell);
                return __builtin_fmax(__builtin_fmin(p - lo, hi - p) - eps, 0.0);
            };
            const double b = __builtin_fmin(__builtin_fmin(face(px, x0, x1), face(py, y0, y1)), face(pz, z0, z1));
            rho2 = __builtin_fmin(b * b * (1.0 - 1e-12), (double)skip_min * (1.0 - 0x1p-20));
        }
        int s = (int)(q[0] & 0xffffu), e = (int)(q[0] >> 16);
        // up to two candidates per step, both from the current range (one site
        // shifts the queue: a wave pays the shift once per step, not twice)
        while (total > 0) {
            // up to kW candidates per step, all from the current range
            int sl[kW];
            bool ok[kW];
#pragma unroll
            for (int u = 0; u < kW; ++u) {
                ok[u] = u == 0 || s + u < e;
                sl[u] = ok[u] ? s + u : s;
            }
            int took = 1;
#pragma unroll
            for (int u = 1; u < kW; ++u) took += ok[u] ? 1 : 0;
            s += took;
            total -= took;
            if (s >= e) {  // next range: shift the queue down by one
#pragma unroll
                for (int k = 0; k < 7; ++k) q[k] = q[k + 1];
                q[7] = 0u;
                s = (int)(q[0] & 0xffffu);
                e = (int)(q[0] >> 16);
            }
            float cx[kW], cy[kW], cz[kW], cw[kW];
#pragma unroll
            for (int u = 0; u < kW; ++u) g.load(sl[u], cx[u], cy[u], cz[u], cw[u]);
            double dd[kW];
#pragma unroll
            for (int u = 0; u < kW; ++u) dd[u] = dist2(px, py, pz, (double)cx[u], (double)cy[u], (double)cz[u]);
#pragma unroll
            for (int u = 0; u < kW; ++u)
                if (ok[u]) seen(dd[u]);
#pragma unroll
            for (int u = 0; u < kW; ++u) {
                if (ok[u] && dd[u] < thr) {
                    const int j = g.index_of(sl[u], cw[u]);
                    if (dd[u] < best || (dd[u] == best && j < bj)) { best = dd[u]; bj = j; if constexpr (kSlot) bs = sl[u]; }
                }
            }
        }
    } else {
        for (int x = x0; x <= x1; ++x) {
            const double gx = cell_gap(px, x, g.cell);
            if (gx > lim) continue;
            for (int y = y0; y <= y1; ++y) {
                const double gxy = gx + cell_gap(py, y, g.cell);
                if (gxy > lim) continue;
                for (int z = z0; z <= z1; ++z) {
                    if (gxy + cell_gap(pz, z, g.cell) > lim) continue;
                    const unsigned h = cell_hash(x, y, z, g.S);
                    int s = (int)g.start[h];
                    const int s1 = (int)g.start[h + 1];
                    for (; s + 1 < s1; s += 2) {
                        // both loads first, then the two updates in slot order
                        float ax, ay, az, aw, bx, by, bz, bw;
                        g.load(s, ax, ay, az, aw);
                        g.load(s + 1, bx, by, bz, bw);
                        const double da = dist2(px, py, pz, (double)ax, (double)ay, (double)az);
                        const double db = dist2(px, py, pz, (double)bx, (double)by, (double)bz);
                        seen(da);
                        seen(db);
                        if (da < thr) {
                            const int j = g.index_of(s, aw);
                            if (da < best || (da == best && j < bj)) { best = da; bj = j; if constexpr (kSlot) bs = s; }
                        }
                        if (db < thr) {
                            const int j = g.index_of(s + 1, bw);
                            if (db < best || (db == best && j < bj)) { best = db; bj = j; if constexpr (kSlot) bs = s + 1; }
                        }
                    }
                    if (s < s1) take(s);
                }
            }
        }
    }
    d2out = best;
    if constexpr (kSlot) *slot = bs;
    if constexpr (kClear) {
        s12out[0] = e1;
        s12out[1] = e2;
        s12out[2] = rho2;
    }
    return bj;
}

template <typename View, bool kSlot = false, int kW = 2>
__device__ __forceinline__ int grid_query(const View &g, double r, double thr, double px,
                                          double py, double pz, double &d2out, int *slot = nullptr) {
    // (an f32-screened walk with a rigorous bound -- f64 only for the winner --
    // measured no faster in round 4: the LDS candidate gathers bind as much)
    return grid_query_exact<View, kSlot, kW>(g, r, thr, px, py, pz, d2out, slot);
}

// Grids for P target clouds (device, workspace-backed; see grid.hip).
struct GridBatch {
    float4 *pts;        // P * mstride: x, y, z, index bits
    uint32_t *start;    // P * (S+1)
    int S;
    int mstride;
    double cell;
    __device__ GridView view(int p) const {
        return GridView{pts + (size_t)p * mstride, start + (size_t)p * (S + 1), S, cell, 1.0 / cell};
    }
};

// bytes of the float4 LDS copy of one pair's grid (0 if it does not fit)
inline size_t grid_lds4_bytes(int mstride, int S, size_t budget) {
    if (mstride > 65535 || S + 1 > 65536) return 0;
    const size_t b = (size_t)mstride * 16 + (size_t)(S + 1) * 2;
    const size_t a = (b + 15) & ~size_t(15);
    return a <= budget ? a : 0;
}

// cooperative float4 copy of pair p's grid into LDS (all threads of the block
// call; ends with a barrier); layout: pts[m] (x, y, z, index bits), start16[S+1]
__device__ inline GridP4 grid_to_lds4(const GridBatch &gb, int p, int m, char *lds) {
    const size_t o = (size_t)p * gb.mstride;
    float4 *lp = (float4 *)lds;
    uint16_t *ls = (uint16_t *)(lp + gb.mstride);
    for (int i = threadIdx.x; i < m; i += blockDim.x) lp[i] = gb.pts[o + i];
    const uint32_t *st = gb.start + (size_t)p * (gb.S + 1);
    for (int i = threadIdx.x; i <= gb.S; i += blockDim.x) ls[i] = (uint16_t)st[i];
    __syncthreads();
    return GridP4{lp, ls, gb.S, gb.cell, 1.0 / gb.cell};
}

// view of a float4 copy that grid_to_lds4 placed at `lds` (no data movement)
__device__ inline GridP4 grid_lds4_view(const GridBatch &gb, char *lds) {
    const float4 *lp = (const float4 *)lds;
    return GridP4{lp, (const uint16_t *)(lp + gb.mstride), gb.S, gb.cell, 1.0 / gb.cell};
}

// host: spatial (Morton-of-cell) order of each cloud's points, (P, Nmax) i32 in a
// workspace slot; with perm, also the points themselves in that order, (P, Nmax, 3)
// f32 in slot perm_slot (a sweep in spatial order then reads its 64-point chunk
// as one contiguous run instead of 64 scattered points)
int spatial_order(const float *pts, const int32_t *n, int P, int Nmax, double cell, hipStream_t s,
                  int ws_slot, const int32_t **order, const float **perm = nullptr, int perm_slot = -1);

// host: allocate (workspace slot) + build; returns PCR_OK or error
// slots: the power of two >= Mmax (>= 256), times slot_num / 2 (3: 1.5x the
// slots -- fewer collisions -- where the consumer's LDS has room for them)
int build_grids(const float *tgt, const int32_t *n_tgt, int P, int Mmax, double r,
                hipStream_t s, int ws_slot, GridBatch &out, double cell_factor = 2.01, int slot_num = 2);

}  // namespace pcr
