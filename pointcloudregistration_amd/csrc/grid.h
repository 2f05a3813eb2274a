// Hashed uniform grid over a target cloud for radius-limited 1-NN queries
// (Open3D KDTreeFlann::SearchHybrid(r, 1) semantics: nearest target with
// d2 < thr strictly, lowest index on exact ties).
//
// Layout per pair in HBM: `start` [S+1] int32 slot offsets, `pts` [m] float4
// (x, y, z, original index as int bits) sorted by slot.  Cells are 2.01*r wide,
// so a query ball touches at most 2x2x2 cells.  Hash collisions only add
// candidates; the exact distance test decides, so results are independent of
// the slot order (and identical to brute force).
#pragma once
#include <hip/hip_runtime.h>
#include "geom.h"

namespace pcr {

struct GridView {
    const float4 *pts;
    const int *start;
    int S;  // power of two
    double cell;
};

__device__ __forceinline__ int cell_coord(double v, double cell) {
    return (int)__builtin_floor(v / cell);
}

__device__ __forceinline__ unsigned cell_hash(int x, int y, int z, int S) {
    return (((unsigned)x * 73856093u) ^ ((unsigned)y * 19349663u) ^ ((unsigned)z * 83492791u)) &
           (unsigned)(S - 1);
}

// returns target index or -1; d2out = its squared distance
__device__ inline int grid_query(const GridView &g, double r, double thr, double px, double py,
                                 double pz, double &d2out) {
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
                const int s1 = g.start[h + 1];
                for (int s = g.start[h]; s < s1; ++s) {
                    const float4 q = g.pts[s];
                    const int j = __float_as_int(q.w);
                    const double d2 = dist2(px, py, pz, (double)q.x, (double)q.y, (double)q.z);
                    if (d2 < thr && (d2 < best || (d2 == best && j < bj))) { best = d2; bj = j; }
                }
            }
    d2out = best;
    return bj;
}

// Build grids for P target clouds (device).  Workspace-backed; see grid.hip.
struct GridBatch {
    float4 *pts;   // P * mstride
    int *start;    // P * (S+1)
    int S;
    int mstride;
    double cell;
    __device__ GridView view(int p) const {
        return GridView{pts + (size_t)p * mstride, start + (size_t)p * (S + 1), S, cell};
    }
};

// host: allocate (workspace slot) + build; returns PCR_OK or error
int build_grids(const float *tgt, const int32_t *n_tgt, int P, int Mmax, double r,
                hipStream_t s, int ws_slot, GridBatch &out);

}  // namespace pcr
