// a1/a2: brute-force bidirectional 1-NN (nndistance) forward + deterministic backward.
//
// Reference: dip/torch-nndistance/src/nnd_cuda.cu:8-130 (NmDistanceKernel),
// :132-162 (launcher), :164-222 (grad); CPU semantics my_lib.cpp:3-25, 64-133.
//
// MI355X design (not a translation of the CUDA kernel):
//  * one launch covers BOTH directions and ALL batch elements
//    (grid.z = 2*b, grid.x = query tiles, grid.y = candidate slices), so even
//    b=1 fills the 256 CUs (the reference kernel keeps min(b,32)*16 blocks busy);
//  * each lane owns Q queries in registers; candidates are staged through LDS
//    as SoA float4 lines and read with broadcast ds_read_b128 (3 LDS reads feed
//    4 candidates x Q queries);
//  * padded candidates are NaN, which the strict '<' update skips, so the inner
//    loop has no tail branch;
//  * when the candidate axis is split (small b), every slice writes its (d, j)
//    partial to scratch and nnd_finalize_kernel takes the minimum over the
//    slices in slice order (strict <: the earlier slice -- the lower index --
//    keeps a tie), i.e. exactly "first index of the minimum";
//  * small problems (C2: one pair of 4096) use 2 queries per lane and
//    128-candidate tiles, so even b = 1 launches ~512 workgroups.
// Numerics: d = (dx*dx + dy*dy) + dz*dz, each op rounded (built with
// -ffp-contract=off), dx = cand.x - query.x as in my_lib.cpp:12-15.
#include "pcr_internal.h"
#include "scan.h"
#include <cstdlib>
#include <math.h>

namespace {

constexpr int kThreads = 256;
constexpr int kTileBig = 512;    // candidates per LDS stage (6 KiB)
constexpr int kTileSmall = 128;  // small problems: more, shorter slices

__device__ __forceinline__ float sqdist(float qx, float qy, float qz, float cx, float cy,
                                        float cz) {
    const float x2 = cx - qx;
    const float y2 = cy - qy;
    const float z2 = cz - qz;
    return x2 * x2 + y2 * y2 + z2 * z2;
}

struct NndArgs {
    const float *xyz1;
    const float *xyz2;
    float *dist1;
    float *dist2;
    int32_t *idx1;
    int32_t *idx2;
    float *pd;                  // split-candidate mode: [slice][2][b][nmax] partial minima
    int32_t *pj;                //   and their indices
    int b, n, m;
    int slice_len;  // candidates per blockIdx.y slice (multiple of the tile)
    int nmax;       // max(n, m): the partial arrays' row stride
    int split;      // 1 if gridDim.y > 1
    const double *gate = nullptr;  // f4 early stop (pcr_internal.h)
};

typedef float f2 __attribute__((ext_vector_type(2)));

// Each lane owns 2*QP queries held as QP float2 pairs; every candidate is
// broadcast into both halves so one v_pk_add / v_pk_mul serves two queries:
// 4 packed arithmetic instructions + compare/select per pair-evaluation.
template <int QP, int kTileK>
__global__ __launch_bounds__(kThreads) void nnd_fwd_kernel(NndArgs a) {
    if (pcr::gated_off(a.gate)) return;
    constexpr int Q = 2 * QP;
    __shared__ float4 sx[kTileK / 4], sy[kTileK / 4], sz[kTileK / 4];

    const int dir = blockIdx.z & 1;
    const int bat = blockIdx.z >> 1;
    const int nq = dir ? a.m : a.n;
    const int nc = dir ? a.n : a.m;
    const float *qbase = (dir ? a.xyz2 : a.xyz1) + (size_t)bat * nq * 3;
    const float *cbase = (dir ? a.xyz1 : a.xyz2) + (size_t)bat * nc * 3;

    const int qtile0 = blockIdx.x * (kThreads * Q);
    if (qtile0 >= nq) return;  // block-uniform
    const int c0 = blockIdx.y * a.slice_len;
    if (c0 >= nc) return;
    const int c1 = min(nc, c0 + a.slice_len);

    const int tid = threadIdx.x;
    f2 qx[QP], qy[QP], qz[QP], best[QP];
    int bi[Q];
#pragma unroll
    for (int i = 0; i < QP; ++i) {
        const int q0 = min(qtile0 + (2 * i) * kThreads + tid, nq - 1);
        const int q1 = min(qtile0 + (2 * i + 1) * kThreads + tid, nq - 1);
        qx[i] = f2{qbase[q0 * 3 + 0], qbase[q1 * 3 + 0]};
        qy[i] = f2{qbase[q0 * 3 + 1], qbase[q1 * 3 + 1]};
        qz[i] = f2{qbase[q0 * 3 + 2], qbase[q1 * 3 + 2]};
        best[i] = f2{INFINITY, INFINITY};
        bi[2 * i] = c0;
        bi[2 * i + 1] = c0;
    }

    float *fx = reinterpret_cast<float *>(sx);
    float *fy = reinterpret_cast<float *>(sy);
    float *fz = reinterpret_cast<float *>(sz);
    for (int t0 = c0; t0 < c1; t0 += kTileK) {
        __syncthreads();
        // stage kTileK candidates AoS -> SoA (pad with NaN: never selected)
        for (int e = tid; e < kTileK * 3; e += kThreads) {
            const int ci = t0 * 3 + e;
            const float v = (ci < c1 * 3) ? cbase[ci] : __builtin_nanf("");
            const int k = e / 3, c = e - 3 * (e / 3);
            (c == 0 ? fx : (c == 1 ? fy : fz))[k] = v;
        }
        __syncthreads();
        const int kend = min(kTileK, c1 - t0);
        const int kend4 = (kend + 3) >> 2;
        for (int k4 = 0; k4 < kend4; ++k4) {
            const float4 X = sx[k4], Y = sy[k4], Z = sz[k4];
            const float cx[4] = {X.x, X.y, X.z, X.w};
            const float cy[4] = {Y.x, Y.y, Y.z, Y.w};
            const float cz[4] = {Z.x, Z.y, Z.z, Z.w};
            const int kb = t0 + k4 * 4;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const f2 CX = f2{cx[c], cx[c]}, CY = f2{cy[c], cy[c]}, CZ = f2{cz[c], cz[c]};
#pragma unroll
                for (int i = 0; i < QP; ++i) {
                    const f2 dx = CX - qx[i], dy = CY - qy[i], dz = CZ - qz[i];
                    const f2 d = (dx * dx + dy * dy) + dz * dz;
                    const bool l0 = d.x < best[i].x, l1 = d.y < best[i].y;
                    best[i].x = l0 ? d.x : best[i].x;
                    bi[2 * i] = l0 ? kb + c : bi[2 * i];
                    best[i].y = l1 ? d.y : best[i].y;
                    bi[2 * i + 1] = l1 ? kb + c : bi[2 * i + 1];
                }
            }
        }
    }

    float *dist = (dir ? a.dist2 : a.dist1) + (size_t)bat * nq;
    int32_t *idx = (dir ? a.idx2 : a.idx1) + (size_t)bat * nq;
    const size_t poff = (((size_t)blockIdx.y * 2 + dir) * a.b + bat) * a.nmax;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int qi = qtile0 + q * kThreads + tid;
        if (qi >= nq) continue;
        const float bq = (q & 1) ? best[q >> 1].y : best[q >> 1].x;
        const float px = (q & 1) ? qx[q >> 1].y : qx[q >> 1].x;
        const float py = (q & 1) ? qy[q >> 1].y : qy[q >> 1].x;
        const float pz = (q & 1) ? qz[q >> 1].y : qz[q >> 1].x;
        if (!a.split) {
            // seed rule of my_lib.cpp:16 (k == 0): a NaN distance to candidate 0
            // wins and freezes the result at (NaN, 0)
            float bb = bq;
            int ii = bi[q];
            const float d0 = sqdist(px, py, pz, cbase[0], cbase[1], cbase[2]);
            if (d0 != d0) { bb = d0; ii = 0; }
            dist[qi] = bb;
            idx[qi] = ii;
        } else {
            a.pd[poff + qi] = bq;
            a.pj[poff + qi] = bi[q];
        }
    }
}

__global__ __launch_bounds__(kThreads) void nnd_finalize_kernel(NndArgs a) {
    if (pcr::gated_off(a.gate)) return;
    const int dir = blockIdx.z & 1;
    const int bat = blockIdx.z >> 1;
    const int nq = dir ? a.m : a.n;
    const int nc = dir ? a.n : a.m;
    const int qi = blockIdx.x * kThreads + threadIdx.x;
    if (qi >= nq) return;
    const float *qp = (dir ? a.xyz2 : a.xyz1) + ((size_t)bat * nq + qi) * 3;
    const float *c0 = (dir ? a.xyz1 : a.xyz2) + (size_t)bat * nc * 3;
    // slices in order: strict < keeps the earlier slice (lower index) on ties;
    // the partials are loaded 8 at a time (independent loads in flight: C2's 32
    // slices one round trip each had made this launch the longer of the two)
    const int used = (nc + a.slice_len - 1) / a.slice_len;
    const size_t ostep = (size_t)2 * a.b * a.nmax;
    const size_t obase = ((size_t)dir * a.b + bat) * a.nmax + qi;
    float d = __builtin_inff();
    int i = 0;
    for (int s0 = 0; s0 < used; s0 += 8) {
        float v[8];
        int j[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (s0 + u < used) {
                v[u] = a.pd[obase + (size_t)(s0 + u) * ostep];
                j[u] = a.pj[obase + (size_t)(s0 + u) * ostep];
            }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (s0 + u < used && (s0 + u == 0 || v[u] < d)) { d = v[u]; i = j[u]; }
    }
    const float d0 = sqdist(qp[0], qp[1], qp[2], c0[0], c0[1], c0[2]);
    if (d0 != d0) { d = d0; i = 0; }
    (dir ? a.dist2 : a.dist1)[(size_t)bat * nq + qi] = d;
    (dir ? a.idx2 : a.idx1)[(size_t)bat * nq + qi] = i;
}

// ---------------------------------------------------------------------------
// backward: deterministic scatter via per-target buckets sorted by source index
// ---------------------------------------------------------------------------
// direction 0 sources: xyz1 points j (target idx1[j] in xyz2); their scatter
//   terms T1[j] = g1_j*(a_j - b_idx1[j]) are subtracted from grad2[idx1[j]].
// direction 1 sources: xyz2 points k (target idx2[k] in xyz1); T2[k] subtracted
//   from grad1[idx2[k]].  Buckets of direction d live in target space.
struct BwdArgs {
    const float *xyz1, *xyz2, *gd1, *gd2;
    const int32_t *idx1, *idx2;
    float *g1, *g2;
    int *cnt1, *cnt2;      // per target counts (b*m for dir0, b*n for dir1), then cursors
    int *start1, *start2;  // exclusive scan
    int *uns1, *uns2;      // bucketed sources (unordered)
    int *srt1, *srt2;      // bucketed sources (increasing)
    int b, n, m;
    const double *gate;    // f4 early stop (pcr_internal.h)
};

__device__ __forceinline__ bool bw_dir(const BwdArgs &a, int dir, int &nsrc, int &ntgt,
                                       const int32_t *&tidx, int *&cnt, int *&start, int *&uns,
                                       int *&srt) {
    nsrc = dir ? a.m : a.n;
    ntgt = dir ? a.n : a.m;
    tidx = dir ? a.idx2 : a.idx1;
    cnt = dir ? a.cnt2 : a.cnt1;
    start = dir ? a.start2 : a.start1;
    uns = dir ? a.uns2 : a.uns1;
    srt = dir ? a.srt2 : a.srt1;
    return true;
}

__global__ void bw_count(BwdArgs a) {
    if (pcr::gated_off(a.gate)) return;
    int nsrc, ntgt; const int32_t *tidx; int *cnt, *start, *uns, *srt;
    const int dir = blockIdx.z & 1, bat = blockIdx.z >> 1;
    bw_dir(a, dir, nsrc, ntgt, tidx, cnt, start, uns, srt);
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nsrc) return;
    const int t = tidx[(size_t)bat * nsrc + e];
    if (t < 0 || t >= ntgt) return;  // invalid index: contributes nothing
    atomicAdd(cnt + (size_t)bat * ntgt + t, 1);
}

// one block per (dir, batch): exclusive scan of counts; counts reset to 0 to be
// reused as fill cursors
__global__ __launch_bounds__(1024) void bw_scan(BwdArgs a) {
    if (pcr::gated_off(a.gate)) return;
    int nsrc, ntgt; const int32_t *tidx; int *cnt, *start, *uns, *srt;
    const int dir = blockIdx.z & 1, bat = blockIdx.z >> 1;
    bw_dir(a, dir, nsrc, ntgt, tidx, cnt, start, uns, srt);
    pcr::block_exclusive_scan_1024(cnt + (size_t)bat * ntgt, start + (size_t)bat * (ntgt + 1), ntgt, true);
}

__global__ void bw_fill(BwdArgs a) {
    if (pcr::gated_off(a.gate)) return;
    int nsrc, ntgt; const int32_t *tidx; int *cnt, *start, *uns, *srt;
    const int dir = blockIdx.z & 1, bat = blockIdx.z >> 1;
    bw_dir(a, dir, nsrc, ntgt, tidx, cnt, start, uns, srt);
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nsrc) return;
    const int t = tidx[(size_t)bat * nsrc + e];
    if (t < 0 || t >= ntgt) return;
    const int pos = start[(size_t)bat * (ntgt + 1) + t] + atomicAdd(cnt + (size_t)bat * ntgt + t, 1);
    uns[(size_t)bat * nsrc + pos] = e;
}

// rank each bucketed source among its bucket (sources are distinct) -> sorted slot
__global__ void bw_rank(BwdArgs a) {
    if (pcr::gated_off(a.gate)) return;
    int nsrc, ntgt; const int32_t *tidx; int *cnt, *start, *uns, *srt;
    const int dir = blockIdx.z & 1, bat = blockIdx.z >> 1;
    bw_dir(a, dir, nsrc, ntgt, tidx, cnt, start, uns, srt);
    const int *s = start + (size_t)bat * (ntgt + 1);
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= s[ntgt]) return;
    const int *u = uns + (size_t)bat * nsrc;
    const int e = u[p];
    const int t = tidx[(size_t)bat * nsrc + e];
    const int b0 = s[t], b1 = s[t + 1];
    int r = 0;
    for (int q = b0; q < b1; ++q) r += (u[q] < e);
    srt[(size_t)bat * nsrc + b0 + r] = e;
}

// per xyz1 point j (dir=0 targets are xyz2 points ... see header comment)
__global__ void bw_chain(BwdArgs a) {
    if (pcr::gated_off(a.gate)) return;
    const int which = blockIdx.z & 1;  // 0: grad1 over xyz1 points, 1: grad2 over xyz2 points
    const int bat = blockIdx.z >> 1;
    const int n = a.n, m = a.m;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const float *A = a.xyz1 + (size_t)bat * n * 3;
    const float *B = a.xyz2 + (size_t)bat * m * 3;
    const float *G1 = a.gd1 + (size_t)bat * n;
    const float *G2 = a.gd2 + (size_t)bat * m;
    const int32_t *I1 = a.idx1 + (size_t)bat * n;
    const int32_t *I2 = a.idx2 + (size_t)bat * m;
    if (which == 0) {
        if (p >= n) return;
        // grad1[j] = ((0 + T1[j]) - T2[k1]) - T2[k2] ...   k in bucket of j (dir 1), increasing
        const int j = p;
        float acc[3] = {0.f, 0.f, 0.f};
        const int t = I1[j];
        if (t >= 0 && t < m) {
            const float g = G1[j] * 2;
#pragma unroll
            for (int c = 0; c < 3; ++c) acc[c] += g * (A[j * 3 + c] - B[t * 3 + c]);
        }
        const int *s = a.start2 + (size_t)bat * (n + 1);
        const int *srt = a.srt2 + (size_t)bat * m;
        for (int q = s[j]; q < s[j + 1]; ++q) {
            const int k = srt[q];
            const float g = G2[k] * 2;
#pragma unroll
            for (int c = 0; c < 3; ++c) acc[c] -= (g * (B[k * 3 + c] - A[j * 3 + c]));
        }
        float *o = a.g1 + ((size_t)bat * n + j) * 3;
        o[0] = acc[0]; o[1] = acc[1]; o[2] = acc[2];
    } else {
        if (p >= m) return;
        // grad2[k] = (((0 - T1[j1]) - T1[j2]) ...) + T2[k]   j in bucket of k (dir 0), increasing
        const int k = p;
        float acc[3] = {0.f, 0.f, 0.f};
        const int *s = a.start1 + (size_t)bat * (m + 1);
        const int *srt = a.srt1 + (size_t)bat * n;
        for (int q = s[k]; q < s[k + 1]; ++q) {
            const int j = srt[q];
            const float g = G1[j] * 2;
#pragma unroll
            for (int c = 0; c < 3; ++c) acc[c] -= (g * (A[j * 3 + c] - B[k * 3 + c]));
        }
        const int t = I2[k];
        if (t >= 0 && t < n) {
            const float g = G2[k] * 2;
#pragma unroll
            for (int c = 0; c < 3; ++c) acc[c] += g * (B[k * 3 + c] - A[t * 3 + c]);
        }
        float *o = a.g2 + ((size_t)bat * m + k) * 3;
        o[0] = acc[0]; o[1] = acc[1]; o[2] = acc[2];
    }
}

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace

namespace pcr {
// large clouds: exact certified grid search (nnd_grid.hip), identical results;
// PCR_NND_ALGO=brute|grid overrides the size rule.  The grid's builds cost tens
// of microseconds of launches; below ~2^27 pair evaluations the brute force
// finishes first (C2: 2 x 4096^2)
bool nnd_uses_grid(int b, int n, int m) {
    const char *e = getenv("PCR_NND_ALGO");
    const bool force_brute = e && e[0] == 'b', force_grid = e && e[0] == 'g';
    const bool big = (long long)b * n * m > (1LL << 27);
    return force_grid || (!force_brute && n >= 1024 && m >= 1024 && big);
}
}  // namespace pcr

extern "C" int pcr_nnd_forward(const float *xyz1, const float *xyz2, int32_t b, int32_t n,
                               int32_t m, float *dist1, float *dist2, int32_t *idx1,
                               int32_t *idx2, pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(b >= 0 && n >= 0 && m >= 0, PCR_ERR_ARG, "nnd_forward: negative size");
    if (b == 0 || (n == 0 && m == 0)) return PCR_OK;
    PCR_REQUIRE(xyz1 && xyz2 && dist1 && dist2 && idx1 && idx2, PCR_ERR_ARG,
                "nnd_forward: null pointer");
    hipStream_t s = pcr::as_stream(stream);
    // empty candidate set: the reference loop never runs -> (0, 0) (my_lib.cpp:10-11)
    if (m == 0 || n == 0) {
        if (m == 0 && n > 0) {
            PCR_HIP_CHECK(hipMemsetAsync(dist1, 0, sizeof(float) * (size_t)b * n, s));
            PCR_HIP_CHECK(hipMemsetAsync(idx1, 0, sizeof(int32_t) * (size_t)b * n, s));
        }
        if (n == 0 && m > 0) {
            PCR_HIP_CHECK(hipMemsetAsync(dist2, 0, sizeof(float) * (size_t)b * m, s));
            PCR_HIP_CHECK(hipMemsetAsync(idx2, 0, sizeof(int32_t) * (size_t)b * m, s));
        }
        return PCR_OK;
    }
    if (pcr::nnd_uses_grid(b, n, m)) return pcr::nnd_forward_grid(xyz1, xyz2, b, n, m, dist1, dist2, idx1, idx2, s);
    const int nmax = n > m ? n : m;
    // 8 queries per lane (4 packed pairs) and 512-candidate tiles, or -- when that
    // cannot give the launch ~4 workgroups per CU (C2: one pair) -- 2 queries
    // per lane and 128-candidate tiles
    const bool small = (long long)cdiv(nmax, kThreads * 8) * 2 * b * cdiv(nmax, kTileBig) < 4LL * pcr::kCUs;
    const int Q = small ? 2 : 8, tile = small ? kTileSmall : kTileBig;
    const int qtiles = cdiv(nmax, kThreads * Q);
    const long long base_blocks = (long long)qtiles * 2 * b;
    // split the candidate axis until the launch has >= ~4 blocks per CU
    int slices = 1;
    while (base_blocks * slices < 4LL * pcr::kCUs && (long long)tile * slices * (small ? 1 : 2) < nmax)
        slices *= 2;
    NndArgs a{xyz1, xyz2, dist1, dist2, idx1, idx2, nullptr, nullptr, b, n, m, 0, slices > 1};
    a.slice_len = cdiv(cdiv(nmax, slices), tile) * tile;
    a.nmax = nmax;
    a.gate = pcr::current_gate();
    const int ys = cdiv(nmax, a.slice_len);
    a.split = ys > 1;
    PCR_REQUIRE(2LL * b <= 65535, PCR_ERR_ARG, "nnd_forward: b=%d too large (max 32767)", b);
    if (a.split) {
        const size_t cells = (size_t)ys * 2 * b * nmax;
        char *ws = (char *)pcr::workspace(0, cells * (sizeof(float) + sizeof(int32_t)));
        PCR_REQUIRE(ws, PCR_ERR_NOMEM, "nnd_forward: %s", pcr_last_error());
        a.pd = (float *)ws;
        a.pj = (int32_t *)(ws + cells * sizeof(float));
    }
    pcr::prof_begin(s, pcr::kProfNndFwd);
    if (small)
        hipLaunchKernelGGL((nnd_fwd_kernel<1, kTileSmall>), dim3(qtiles, ys, 2 * b), dim3(kThreads), 0, s, a);
    else
        hipLaunchKernelGGL((nnd_fwd_kernel<4, kTileBig>), dim3(qtiles, ys, 2 * b), dim3(kThreads), 0, s, a);
    PCR_LAUNCH_CHECK();
    pcr::prof_end(s, pcr::kProfNndFwd);
    if (a.split) {
        hipLaunchKernelGGL(nnd_finalize_kernel, dim3(cdiv(nmax, kThreads), 1, 2 * b),
                           dim3(kThreads), 0, s, a);
        PCR_LAUNCH_CHECK();
    }
    return PCR_OK;
}

extern "C" int pcr_nnd_backward(const float *xyz1, const float *xyz2, const float *gd1,
                                const float *gd2, const int32_t *idx1, const int32_t *idx2,
                                int32_t b, int32_t n, int32_t m, float *g1, float *g2,
                                pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(b >= 0 && n >= 0 && m >= 0, PCR_ERR_ARG, "nnd_backward: negative size");
    if (b == 0 || (n == 0 && m == 0)) return PCR_OK;
    PCR_REQUIRE(xyz1 && xyz2 && gd1 && gd2 && idx1 && idx2 && g1 && g2, PCR_ERR_ARG,
                "nnd_backward: null pointer");
    PCR_REQUIRE(2LL * b <= 65535, PCR_ERR_ARG, "nnd_backward: b=%d too large", b);
    hipStream_t s = pcr::as_stream(stream);
    const size_t bn = (size_t)b * n, bm = (size_t)b * m;
    // workspace: cnt1[bm] cnt2[bn] start1[b*(m+1)] start2[b*(n+1)] uns1[bn] uns2[bm] srt1[bn] srt2[bm]
    const size_t words = bm + bn + (size_t)b * (m + 1) + (size_t)b * (n + 1) + 2 * (bn + bm);
    int *ws = (int *)pcr::workspace(1, words * sizeof(int));
    PCR_REQUIRE(ws, PCR_ERR_NOMEM, "nnd_backward: %s", pcr_last_error());
    BwdArgs a;
    a.xyz1 = xyz1; a.xyz2 = xyz2; a.gd1 = gd1; a.gd2 = gd2; a.idx1 = idx1; a.idx2 = idx2;
    a.g1 = g1; a.g2 = g2; a.b = b; a.n = n; a.m = m;
    a.gate = pcr::current_gate();
    int *p = ws;
    a.cnt1 = p; p += bm;
    a.cnt2 = p; p += bn;
    a.start1 = p; p += (size_t)b * (m + 1);
    a.start2 = p; p += (size_t)b * (n + 1);
    a.uns1 = p; p += bn;
    a.uns2 = p; p += bm;
    a.srt1 = p; p += bn;
    a.srt2 = p; p += bm;
    PCR_HIP_CHECK(hipMemsetAsync(ws, 0, sizeof(int) * (bm + bn), s));
    const int nmax = n > m ? n : m;
    const dim3 g(cdiv(nmax > 0 ? nmax : 1, 256), 1, 2 * b);
    hipLaunchKernelGGL(bw_count, g, dim3(256), 0, s, a);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(bw_scan, dim3(1, 1, 2 * b), dim3(1024), 0, s, a);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(bw_fill, g, dim3(256), 0, s, a);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(bw_rank, g, dim3(256), 0, s, a);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(bw_chain, g, dim3(256), 0, s, a);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}
