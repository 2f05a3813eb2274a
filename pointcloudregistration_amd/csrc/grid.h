// Hashed uniform grid over a target cloud for radius-limited 1-NN queries
// (Open3D KDTreeFlann::SearchHybrid(r, 1) semantics: nearest target with
// d2 < thr strictly, lowest index on exact ties).
//
// HBM layout per pair (SoA): x/y/z [mstride] f32 and idx [mstride] u32 sorted by
// slot, start [S+1] u32 slot offsets.  Cells are 2.01*r wide, so a query ball
// touches at most 2x2x2 cells.  Hash collisions only add candidates; the exact
// distance test decides, so results are independent of slot order and equal to
// brute force.  Consumers that own a pair (RANSAC, ICP) copy the grid into LDS
// with u16 idx/start (14 B per point + 2 B per slot; 128 KiB at 8192 points).
#pragma once
#include <hip/hip_runtime.h>
#include "geom.h"

namespace pcr {

__device__ __forceinline__ int cell_coord(double v, double cell) {
    return (int)__builtin_floor(v / cell);
}

__device__ __forceinline__ unsigned cell_hash(int x, int y, int z, int S) {
    return (((unsigned)x * 73856093u) ^ ((unsigned)y * 19349663u) ^ ((unsigned)z * 83492791u)) &
           (unsigned)(S - 1);
}

// generic view: IdxT = uint32_t (HBM) or uint16_t (LDS copy)
template <typename IdxT>
struct GridT {
    const float *x, *y, *z;
    const IdxT *idx;
    const IdxT *start;
    int S;
    double cell;
};
using GridView = GridT<uint32_t>;

// returns target index or -1; d2out = its squared distance
template <typename IdxT>
__device__ __forceinline__ int grid_query(const GridT<IdxT> &g, double r, double thr, double px,
                                          double py, double pz, double &d2out) {
    const double rr = 1.001 * r;
    const int x0 = cell_coord(px - rr, g.cell), x1 = cell_coord(px + rr, g.cell);
    const int y0 = cell_coord(py - rr, g.cell), y1 = cell_coord(py + rr, g.cell);
    const int z0 = cell_coord(pz - rr, g.cell), z1 = cell_coord(pz + rr, g.cell);
    double best = __builtin_inf();
    int bj = -1;
    for (int x = x0; x <= x1; ++x)
        for (int y = y0; y <= y1; ++y)
            for (int z = z0; z <= z1; ++z) {
                const unsigned h = cell_hash(x, y, z, g.S);
                const int s1 = (int)g.start[h + 1];
                for (int s = (int)g.start[h]; s < s1; ++s) {
                    const double d2 = dist2(px, py, pz, (double)g.x[s], (double)g.y[s], (double)g.z[s]);
                    if (d2 < thr) {
                        const int j = (int)g.idx[s];
                        if (d2 < best || (d2 == best && j < bj)) { best = d2; bj = j; }
                    }
                }
            }
    d2out = best;
    return bj;
}

// Grids for P target clouds (device, workspace-backed; see grid.hip).
struct GridBatch {
    float *x, *y, *z;   // P * mstride
    uint32_t *idx;      // P * mstride
    uint32_t *start;    // P * (S+1)
    int S;
    int mstride;
    double cell;
    __device__ GridView view(int p) const {
        const size_t o = (size_t)p * mstride;
        return GridView{x + o, y + o, z + o, idx + o, start + (size_t)p * (S + 1), S, cell};
    }
};

// bytes of the LDS copy of one pair's grid (0 if it does not fit the budget)
inline size_t grid_lds_bytes(int mstride, int S, size_t budget) {
    if (mstride > 65535 || S + 1 > 65536) return 0;
    const size_t b = (size_t)mstride * 14 + (size_t)(S + 1) * 2;
    const size_t a = (b + 15) & ~size_t(15);
    return a <= budget ? a : 0;
}

// cooperative copy of pair p's grid into LDS (all threads of the block call);
// layout: x[m] y[m] z[m] idx16[m] start16[S+1]
__device__ inline GridT<uint16_t> grid_to_lds(const GridBatch &gb, int p, int m, char *lds) {
    const size_t o = (size_t)p * gb.mstride;
    float *lx = (float *)lds;
    float *ly = lx + gb.mstride;
    float *lz = ly + gb.mstride;
    uint16_t *li = (uint16_t *)(lz + gb.mstride);
    uint16_t *ls = li + gb.mstride;
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        lx[i] = gb.x[o + i];
        ly[i] = gb.y[o + i];
        lz[i] = gb.z[o + i];
        li[i] = (uint16_t)gb.idx[o + i];
    }
    const uint32_t *st = gb.start + (size_t)p * (gb.S + 1);
    for (int i = threadIdx.x; i <= gb.S; i += blockDim.x) ls[i] = (uint16_t)st[i];
    __syncthreads();
    return GridT<uint16_t>{lx, ly, lz, li, ls, gb.S, gb.cell};
}

// host: allocate (workspace slot) + build; returns PCR_OK or error
int build_grids(const float *tgt, const int32_t *n_tgt, int P, int Mmax, double r,
                hipStream_t s, int ws_slot, GridBatch &out);

}  // namespace pcr
