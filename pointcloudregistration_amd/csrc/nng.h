// Device helpers of the certified grid 1-NN (a1), shared by the nnd drop-in
// (nnd_grid.hip) and the NDP level Chamfer (ndp_chamfer.hip).
//
// Contract (my_lib.cpp:3-25): the candidate minimising d = (dx*dx + dy*dy) +
// dz*dz in f32 (dx = c - q, no FMA), lowest index on ties: for finite inputs
// the lexicographic minimum of (d, j), which any search over a superset of the
// winners returns unchanged.
#pragma once
#include <hip/hip_runtime.h>

namespace pcr {
namespace nng {

// slot of cell (x, y, z): the low 10 bits of each coordinate packed, then
// murmur3's finaliser (grid.h cell_hash; the XOR-multiply hash collided on small
// coordinate ranges: C4 Chamfer query 0.51 -> 0.47 ms per step with this one)
__device__ __forceinline__ unsigned nhash(int x, int y, int z, int S) {
    unsigned k = ((unsigned)x & 1023u) | (((unsigned)y & 1023u) << 10) | (((unsigned)z & 1023u) << 20);
    k ^= k >> 16;
    k *= 0x85ebca6bu;
    k ^= k >> 13;
    k *= 0xc2b2ae35u;
    k ^= k >> 16;
    return k & (unsigned)(S - 1);
}

__device__ __forceinline__ int ccoord(float v, double ic) { return (int)__builtin_floor((double)v * ic); }

__device__ __forceinline__ float d2f(float cx, float cy, float cz, float qx, float qy, float qz) {
    const float dx = cx - qx, dy = cy - qy, dz = cz - qz;
    return (dx * dx + dy * dy) + dz * dz;
}

// (d, j) lexicographic update
__device__ __forceinline__ void take(float d, int j, float &best, int &bj) {
    if (d < best || (d == best && j < bj)) { best = d; bj = j; }
}

// the same update as selects (no branch: for many independent minima per lane)
__device__ __forceinline__ void take_sel(float d, int j, float &best, int &bj) {
    const bool lt = (d < best) | ((d == best) & (j < bj));
    best = lt ? d : best;
    bj = lt ? j : bj;
}

// a grid view: cell edge, S hash slots, slot starts (S + 1), float4 (x, y, z,
// index bits) points sorted by slot
struct View {
    float cell;
    int S;
    const int *start;
    const float4 *pts;
};

// Chebyshev rings k = 0..kmax around q's cell; the LPQ lanes of a query split
// each ring's (dx, dy) columns and merge their minima before every
// certification test.  After ring k every unvisited point is at least g (the
// distance from q to the faces of the (2k+1)^3 block, minus a 1e-6 relative
// margin) away, and its computed f32 distance at least g^2 (1 - 8 * 2^-24)
// (five relative f32 roundings); strictly above the best: final.  Returns
// whether the answer was certified.
//
// Inside a ring a cell (a column of cells) is skipped when its box is provably
// farther than the lane's best: a lower bound G on the squared distance from q
// to the box, from q's margin-shrunk distances to its own cell's faces plus
// whole cells, in f32 (relative error below 16 * 2^-24); a skipped cell's
// points have computed distances >= G (1 - 8 * 2^-24) >= 0.99999 G > best, so
// they could neither win nor tie.  A lane's best only falls, and the merged
// best is at most the lane's: the skips are exact for every LPQ.  kSkip = false
// walks every cell of a ring (the NDP level Chamfer: ring cap 1, four lanes per
// query -- the bounds cost more there than the cells they save).
template <int LPQ, bool kSkip = true, typename V>
__device__ __forceinline__ bool ring_walk(const V &v, float qx, float qy, float qz, int sub, int kmax,
                                          float &best, int &bj) {
    auto merge = [&]() {
#pragma unroll
        for (int o = 1; o < LPQ; o <<= 1) {
            const float ob = __shfl_xor(best, o, 64);
            const int oj = __shfl_xor(bj, o, 64);
            take(ob, oj, best, bj);
        }
    };
    const double cell = (double)v.cell, ic = 1.0 / cell;
    const int cx = ccoord(qx, ic), cy = ccoord(qy, ic), cz = ccoord(qz, ic);
    const double margin = 1e-6 * (fabs((double)qx) + fabs((double)qy) + fabs((double)qz) + cell);
    // q's distances to the low / high faces of its own cell, less the margin
    const float lx = (float)fmax((double)qx - (double)cx * cell - margin, 0.0);
    const float hx = (float)fmax((double)(cx + 1) * cell - (double)qx - margin, 0.0);
    const float ly = (float)fmax((double)qy - (double)cy * cell - margin, 0.0);
    const float hy = (float)fmax((double)(cy + 1) * cell - (double)qy - margin, 0.0);
    const float lz = (float)fmax((double)qz - (double)cz * cell - margin, 0.0);
    const float hz = (float)fmax((double)(cz + 1) * cell - (double)qz - margin, 0.0);
    const float cf = v.cell;
    // squared gap along one axis to the cell at offset d (lower bound)
    auto gap2 = [&](int d, float lo, float hi) -> float {
        const float g = d == 0 ? 0.f : (d > 0 ? hi : lo) + (float)((d > 0 ? d : -d) - 1) * cf;
        return g * g;
    };
    constexpr float kLb = 0.99999f;
    // up to three cells (x, y, z0 + t dz), t < n, each unless its box is beyond
    // the best: every slot bound is loaded first, then each cell's points four
    // at a time, so a lane waits on one round trip per batch instead of one per
    // cell and one per point (the walk is bound by the latency of these
    // dependent loads; take() is order-free)
    auto scan_cells = [&](int x, int y, int z0, int dz, int n, float gxy) {
        int s0[3], s1[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            s0[t] = 0;
            s1[t] = 0;
            const int z = z0 + t * dz;
            if (t < n && (!kSkip || (gxy + gap2(z - cz, lz, hz)) * kLb <= best)) {
                const unsigned h = nhash(x, y, z, v.S);
                s0[t] = v.start[h];
                s1[t] = v.start[h + 1];
            }
        }
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            for (int s = s0[t]; s < s1[t]; s += 4) {
                float4 p[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (s + u < s1[t]) p[u] = v.pts[s + u];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (s + u < s1[t]) take(d2f(p[u].x, p[u].y, p[u].z, qx, qy, qz), __float_as_int(p[u].w), best, bj);
            }
        }
    };
    for (int k = 0; k <= kmax; ++k) {
        // column c = (dx, dy) of ring k; lane sub takes columns sub, sub + LPQ, ...
        const int side = 2 * k + 1;
        for (int c = sub; c < side * side; c += LPQ) {
            const int cq = c / side, dx = cq - k, dy = c - cq * side - k;
            const float gxy = gap2(dx, lx, hx) + gap2(dy, ly, hy);
            if (kSkip && gxy * kLb > best) continue;  // the whole column lies beyond the best
            if (dx == -k || dx == k || dy == -k || dy == k) {
                for (int z = cz - k; z <= cz + k; z += 3) scan_cells(cx + dx, cy + dy, z, 1, min(3, cz + k - z + 1), gxy);
            } else {
                scan_cells(cx + dx, cy + dy, cz - k, 2 * k, 2, gxy);
            }
        }
        merge();
        const double gx = fmin((double)qx - (double)(cx - k) * cell, (double)(cx + k + 1) * cell - (double)qx);
        const double gy = fmin((double)qy - (double)(cy - k) * cell, (double)(cy + k + 1) * cell - (double)qy);
        const double gz = fmin((double)qz - (double)(cz - k) * cell, (double)(cz + k + 1) * cell - (double)qz);
        const double gmin = fmin(gx, fmin(gy, gz)) - margin;
        if (gmin > 0.0 && gmin * gmin * (1.0 - 8.0 * 5.9604644775390625e-08) > (double)best) return true;
    }
    return false;
}

}  // namespace nng
}  // namespace pcr
