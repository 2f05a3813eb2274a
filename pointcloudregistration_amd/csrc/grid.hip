// Batched hashed-grid construction over target clouds (one launch per stage
// for all P pairs).  See grid.h for the layout and query semantics.
#include "pcr_internal.h"
#include "grid.h"
#include "scan.h"

namespace pcr {
namespace {

struct BuildArgs {
    const float *tgt;
    const int32_t *n_tgt;
    int Mmax, S;
    double cell;
    int *cnt;      // P*S
    int *start;    // P*(S+1)
    float4 *pts;   // P*Mmax: x, y, z, index bits (one 16-B store per point)
};

__device__ __forceinline__ int count_of(const int32_t *n, int p, int Mmax) {
    return n ? min(max(n[p], 0), Mmax) : Mmax;
}

__global__ void grid_count(BuildArgs a) {
    const int p = blockIdx.y;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= count_of(a.n_tgt, p, a.Mmax)) return;
    const float *q = a.tgt + ((size_t)p * a.Mmax + j) * 3;
    const unsigned h = cell_hash(cell_coord((double)q[0], a.cell), cell_coord((double)q[1], a.cell),
                                 cell_coord((double)q[2], a.cell), a.S);
    atomicAdd(a.cnt + (size_t)p * a.S + h, 1);
}

__global__ __launch_bounds__(1024) void grid_scan(BuildArgs a) {
    const int p = blockIdx.x;
    block_exclusive_scan_1024(a.cnt + (size_t)p * a.S, a.start + (size_t)p * (a.S + 1), a.S, true);
}

__global__ void grid_scatter(BuildArgs a) {
    const int p = blockIdx.y;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= count_of(a.n_tgt, p, a.Mmax)) return;
    const float *q = a.tgt + ((size_t)p * a.Mmax + j) * 3;
    const unsigned h = cell_hash(cell_coord((double)q[0], a.cell), cell_coord((double)q[1], a.cell),
                                 cell_coord((double)q[2], a.cell), a.S);
    const int pos = a.start[(size_t)p * (a.S + 1) + h] + atomicAdd(a.cnt + (size_t)p * a.S + h, 1);
    a.pts[(size_t)p * a.Mmax + pos] = make_float4(q[0], q[1], q[2], __int_as_float(j));
}

// count, scan and scatter of one pair's grid in one workgroup, the slot
// counters in LDS (S <= kLdsSlots): the per-point atomics stay on the CU
// (the global count / scatter passes took ~0.19 ms per grid per C4 step).
// Points land in a cell in atomic order, as before: every query takes the
// lexicographic (d2, j) minimum, so the order within a cell changes no result.
constexpr int kLdsSlots = 32768;

__global__ __launch_bounds__(1024) void grid_build_lds(BuildArgs a) {
    extern __shared__ int cnt[];  // S + 1: counts -> exclusive starts -> cursors
    const int p = blockIdx.x, S = a.S;
    const int m = count_of(a.n_tgt, p, a.Mmax);
    const float *q = a.tgt + (size_t)p * a.Mmax * 3;
    for (int i = threadIdx.x; i < S; i += 1024) cnt[i] = 0;
    __syncthreads();
    for (int j = threadIdx.x; j < m; j += 1024)
        atomicAdd(&cnt[cell_hash(cell_coord((double)q[3 * j], a.cell), cell_coord((double)q[3 * j + 1], a.cell),
                                 cell_coord((double)q[3 * j + 2], a.cell), S)],
                  1);
    __syncthreads();
    block_exclusive_scan_1024(cnt, cnt, S, false);
    int *st = a.start + (size_t)p * (S + 1);
    for (int i = threadIdx.x; i <= S; i += 1024) st[i] = cnt[i];
    __syncthreads();
    for (int j = threadIdx.x; j < m; j += 1024) {
        const float x = q[3 * j], y = q[3 * j + 1], z = q[3 * j + 2];
        const unsigned h = cell_hash(cell_coord((double)x, a.cell), cell_coord((double)y, a.cell),
                                     cell_coord((double)z, a.cell), S);
        a.pts[(size_t)p * a.Mmax + atomicAdd(&cnt[h], 1)] = make_float4(x, y, z, __int_as_float(j));
    }
}

// Spatial order of a cloud: points bucketed by the Morton code of their grid
// cell, 5 bits per axis relative to the cloud's minimum cell (cells merged in
// powers of two until the cloud's extent fits 32), by a counting sort in LDS --
// one 1024-thread workgroup per cloud: count, scan, scatter (the bitonic sort
// of full 30-bit codes it replaces took 128 us per C4 call).  Sweeps that walk
// a cloud in this order give each wave neighbouring queries: the same hash
// cells, similar candidate counts, coherent LDS reads.  Order within a bucket is
// atomic order; it changes timing only (every sweep's result is independent of
// the order: fixed-point or integer sums, per-point outputs, and an early stop
// that only fires on hypotheses that cannot win).
__device__ __forceinline__ unsigned spread10(unsigned v) {
    v &= 1023u;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

constexpr int kOrdBits = 5, kOrdBuckets = 1 << (3 * kOrdBits);

__global__ __launch_bounds__(1024) void spatial_order_kernel(const float *pts, const int32_t *n, int Nmax,
                                                             double inv_cell, int32_t *order, float *perm) {
    extern __shared__ int bk[];  // kOrdBuckets + 1: counts -> starts -> cursors
    __shared__ int smin[3][16], smax[3][16];
    constexpr int kReg = 8;      // points per thread whose cell coordinates stay in registers
    const int p = blockIdx.x, t = threadIdx.x;
    const int m = count_of(n, p, Nmax);
    const float *P = pts + (size_t)p * Nmax * 3;
    int32_t *o = order + (size_t)p * Nmax;
    float *pm = perm ? perm + (size_t)p * Nmax * 3 : nullptr;
    auto put = [&](int pos, int i) {
        o[pos] = i;
        if (pm) { pm[3 * pos] = P[3 * i]; pm[3 * pos + 1] = P[3 * i + 1]; pm[3 * pos + 2] = P[3 * i + 2]; }
    };
    auto cellq = [&](int i, int c) { return (int)__builtin_floor((double)P[3 * i + c] * inv_cell); };
    int qr[kReg][3];
    int mn[3] = {0x7fffffff, 0x7fffffff, 0x7fffffff}, mx[3] = {-0x7fffffff, -0x7fffffff, -0x7fffffff};
#pragma unroll
    for (int u = 0; u < kReg; ++u) {
        const int i = t + 1024 * u;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            qr[u][c] = i < m ? cellq(i, c) : 0;
            if (i < m) { mn[c] = min(mn[c], qr[u][c]); mx[c] = max(mx[c], qr[u][c]); }
        }
    }
    for (int i = t + 1024 * kReg; i < m; i += 1024)
        for (int c = 0; c < 3; ++c) {
            const int q = cellq(i, c);
            mn[c] = min(mn[c], q);
            mx[c] = max(mx[c], q);
        }
    for (int c = 0; c < 3; ++c) {
        for (int off = 32; off; off >>= 1) {
            mn[c] = min(mn[c], __shfl_xor(mn[c], off, 64));
            mx[c] = max(mx[c], __shfl_xor(mx[c], off, 64));
        }
        if ((t & 63) == 0) { smin[c][t >> 6] = mn[c]; smax[c][t >> 6] = mx[c]; }
    }
    for (int i = t; i < kOrdBuckets; i += 1024) bk[i] = 0;
    __syncthreads();
    int base[3], ext = 0;
    for (int c = 0; c < 3; ++c) {
        int lo = smin[c][0], hi = smax[c][0];
        for (int w = 1; w < 16; ++w) { lo = min(lo, smin[c][w]); hi = max(hi, smax[c][w]); }
        base[c] = lo;
        ext = max(ext, (int)min((long long)hi - lo, (long long)0x3fffffff));
    }
    int shift = 0;
    while ((ext >> shift) >= (1 << kOrdBits)) ++shift;
    auto key_of = [&](const int (&q)[3]) -> unsigned {
        unsigned k = 0;
        for (int c = 0; c < 3; ++c) {
            const int v = (q[c] - base[c]) >> shift;
            k |= spread10((unsigned)min(max(v, 0), (1 << kOrdBits) - 1)) << c;
        }
        return k;
    };
    auto key = [&](int i) -> unsigned {
        const int q[3] = {cellq(i, 0), cellq(i, 1), cellq(i, 2)};
        return key_of(q);
    };
    unsigned kr[kReg];
#pragma unroll
    for (int u = 0; u < kReg; ++u) {
        kr[u] = key_of(qr[u]);
        if (t + 1024 * u < m) atomicAdd(&bk[kr[u]], 1);
    }
    for (int i = t + 1024 * kReg; i < m; i += 1024) atomicAdd(&bk[key(i)], 1);
    __syncthreads();
    block_exclusive_scan_1024(bk, bk, kOrdBuckets, false);
#pragma unroll
    for (int u = 0; u < kReg; ++u) {
        const int i = t + 1024 * u;
        if (i < m) put(atomicAdd(&bk[kr[u]], 1), i);
    }
    for (int i = t + 1024 * kReg; i < m; i += 1024) put(atomicAdd(&bk[key(i)], 1), i);
    for (int i = m + t; i < Nmax; i += 1024) o[i] = i;
}

}  // namespace

int spatial_order(const float *pts, const int32_t *n, int P, int Nmax, double cell, hipStream_t s,
                  int ws_slot, const int32_t **order, const float **perm, int perm_slot) {
    int32_t *o = (int32_t *)workspace(ws_slot, sizeof(int32_t) * (size_t)P * Nmax + 64);
    PCR_REQUIRE(o, PCR_ERR_NOMEM, "spatial_order: %s", pcr_last_error());
    float *pm = nullptr;
    if (perm) {
        pm = (float *)workspace(perm_slot, sizeof(float) * 3 * (size_t)P * Nmax + 64);
        PCR_REQUIRE(pm, PCR_ERR_NOMEM, "spatial_order: %s", pcr_last_error());
    }
    const size_t sm = sizeof(int) * (size_t)(kOrdBuckets + 1);
    PCR_HIP_CHECK(hipFuncSetAttribute((const void *)spatial_order_kernel,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm));
    hipLaunchKernelGGL(spatial_order_kernel, dim3(P), dim3(1024), sm, s, pts, n, Nmax, 1.0 / cell, o, pm);
    PCR_LAUNCH_CHECK();
    *order = o;
    if (perm) *perm = pm;
    return PCR_OK;
}

int build_grids(const float *tgt, const int32_t *n_tgt, int P, int Mmax, double r, hipStream_t s,
                int ws_slot, GridBatch &out, double cell_factor, int slot_num) {
    int S = 256;
    while (S < Mmax) S <<= 1;
    S = S / 2 * slot_num;
    const size_t cnt_b = sizeof(int) * (size_t)P * S;
    const size_t start_b = sizeof(int) * (size_t)P * (S + 1);
    const size_t pts_b = 16 * (size_t)P * (Mmax > 0 ? Mmax : 1);
    char *ws = (char *)workspace(ws_slot, cnt_b + start_b + pts_b + 64);
    PCR_REQUIRE(ws, PCR_ERR_NOMEM, "grid workspace: %s", pcr_last_error());
    BuildArgs a;
    a.tgt = tgt;
    a.n_tgt = n_tgt;
    a.Mmax = Mmax;
    a.S = S;
    a.cell = cell_factor * r;
    a.cnt = (int *)ws;
    a.start = (int *)(ws + cnt_b);
    size_t off = (cnt_b + start_b + 15) & ~size_t(15);
    a.pts = (float4 *)(ws + off);
    if (S <= kLdsSlots) {
        PCR_HIP_CHECK(hipFuncSetAttribute((const void *)grid_build_lds, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)(sizeof(int) * (kLdsSlots + 1))));
        hipLaunchKernelGGL(grid_build_lds, dim3(P), dim3(1024), sizeof(int) * (size_t)(S + 1), s, a);
        PCR_LAUNCH_CHECK();
    } else {
        PCR_HIP_CHECK(hipMemsetAsync(a.cnt, 0, cnt_b, s));
        const dim3 g((Mmax + 255) / 256 > 0 ? (Mmax + 255) / 256 : 1, P);
        hipLaunchKernelGGL(grid_count, g, dim3(256), 0, s, a);
        PCR_LAUNCH_CHECK();
        hipLaunchKernelGGL(grid_scan, dim3(P), dim3(1024), 0, s, a);
        PCR_LAUNCH_CHECK();
        hipLaunchKernelGGL(grid_scatter, g, dim3(256), 0, s, a);
        PCR_LAUNCH_CHECK();
    }
    out.pts = a.pts;
    out.start = (uint32_t *)a.start;
    out.S = S;
    out.mstride = Mmax;
    out.cell = a.cell;
    return PCR_OK;
}

namespace {
__global__ void radius_nn_kernel(GridBatch g, const double *q, const int32_t *n_q, int Qmax,
                                 double r, double thr, int32_t *idx, double *d2o) {
    const int p = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= Qmax) return;
    const int nq = n_q ? min(max(n_q[p], 0), Qmax) : Qmax;
    int j = -1;
    double d2 = __builtin_inf();
    if (i < nq) {
        const double *x = q + ((size_t)p * Qmax + i) * 3;
        j = grid_query(g.view(p), r, thr, x[0], x[1], x[2], d2);
    }
    idx[(size_t)p * Qmax + i] = j;
    if (d2o) d2o[(size_t)p * Qmax + i] = d2;
}
}  // namespace

}  // namespace pcr

extern "C" int pcr_radius_nn(const float *tgt_xyz, int32_t P, int32_t Mmax, const int32_t *n_tgt,
                             const double *queries, int32_t Qmax, const int32_t *n_q, double r,
                             int32_t *idx, double *d2, pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(P >= 0 && Mmax >= 0 && Qmax >= 0, PCR_ERR_ARG, "radius_nn: negative size");
    if (P == 0 || Qmax == 0) return PCR_OK;
    PCR_REQUIRE(tgt_xyz && queries && idx, PCR_ERR_ARG, "radius_nn: null pointer");
    PCR_REQUIRE(r > 0.0, PCR_ERR_ARG, "radius_nn: r must be > 0");
    PCR_REQUIRE(P <= 65535, PCR_ERR_ARG, "radius_nn: P=%d > 65535", P);
    hipStream_t s = pcr::as_stream(stream);
    pcr::GridBatch g;
    int rc = pcr::build_grids(tgt_xyz, n_tgt, P, Mmax, r, s, 10, g);
    if (rc != PCR_OK) return rc;
    hipLaunchKernelGGL(pcr::radius_nn_kernel, dim3((Qmax + 255) / 256, P), dim3(256), 0, s, g,
                       queries, n_q, Qmax, r, pcr::radius_thr(r), idx, d2);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}
