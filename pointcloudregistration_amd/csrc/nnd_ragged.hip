// a1/a3: bidirectional 1-NN over RAGGED batches and in f64 -- the search behind
// the full compute_truncated_chamfer_distance interface
// (c2p-net/deformationpyramid/model/loss.py:60-160: x_lengths / y_lengths,
// pytorch3d.knn_points(lengths1, lengths2, K=1) in the dtype of its inputs;
// validationScript.py:273-283 hands it f64 tensors).
//
// Semantics per (batch b, direction): the queries i < nq[b] of one cloud against
// the candidates j < nc[b] of the other; d = (dx*dx + dy*dy) + dz*dz in Scalar
// with dx = cand - query, each op rounded (-ffp-contract=off), the FIRST j
// attaining the minimum, candidate 0's NaN seeding rule of my_lib.cpp:16 (the
// same contract as pcr_nnd_forward, now per cloud length and for f64).  Rows
// past a cloud's length, and queries of a batch whose other cloud is empty,
// get (0, 0) (my_lib.cpp's seed values; pytorch3d's zero-initialised outputs).
//
// Layout / kernel: grid (query tiles, candidate slices, 2 b); a slice of
// candidates is staged through LDS as SoA, every lane holds two queries; a
// slice's (d, j) partial goes to scratch and nnd_ragged_merge takes the
// lexicographic minimum over the slices in slice order (strict <: the earlier
// slice, i.e. the lower index, keeps a tie).  Not on the C4 hot path
// (pcr_nnd_forward serves homogeneous f32 batches); sized for the validation
// and loss calls of the reference's scripts.
#include "pcr_internal.h"

namespace {

constexpr int kRThreads = 256;
constexpr int kRQ = 2;          // queries per lane
constexpr int kRTile = 256;     // candidates per LDS stage

template <typename Scalar>
struct RaggedArgs {
    const Scalar *xyz1, *xyz2;
    const int32_t *n1, *n2;     // may be null: full length
    Scalar *dist1, *dist2;
    int32_t *idx1, *idx2;
    Scalar *pd;                 // [slices][2][b][nmax] partial distances
    int32_t *pj;                // [slices][2][b][nmax] partial indices
    int b, n, m, nmax;
    int slice_len, slices;
};

template <typename Scalar>
__device__ __forceinline__ Scalar sq3(Scalar qx, Scalar qy, Scalar qz, Scalar cx, Scalar cy,
                                      Scalar cz) {
    const Scalar x2 = cx - qx, y2 = cy - qy, z2 = cz - qz;
    return (x2 * x2 + y2 * y2) + z2 * z2;
}

template <typename Scalar>
__device__ __forceinline__ void dir_view(const RaggedArgs<Scalar> &a, int dir, int bat, int &nq,
                                         int &nc, int &cap_q, int &cap_c, const Scalar *&q,
                                         const Scalar *&c) {
    cap_q = dir ? a.m : a.n;
    cap_c = dir ? a.n : a.m;
    const int32_t *lq = dir ? a.n2 : a.n1;
    const int32_t *lc = dir ? a.n1 : a.n2;
    nq = lq ? min(max(lq[bat], 0), cap_q) : cap_q;
    nc = lc ? min(max(lc[bat], 0), cap_c) : cap_c;
    q = (dir ? a.xyz2 : a.xyz1) + (size_t)bat * cap_q * 3;
    c = (dir ? a.xyz1 : a.xyz2) + (size_t)bat * cap_c * 3;
}

template <typename Scalar>
__global__ __launch_bounds__(kRThreads) void nnd_ragged_kernel(RaggedArgs<Scalar> a) {
    __shared__ Scalar sx[kRTile], sy[kRTile], sz[kRTile];
    const int dir = blockIdx.z & 1, bat = blockIdx.z >> 1;
    int nq, nc, cap_q, cap_c;
    const Scalar *qb, *cb;
    dir_view(a, dir, bat, nq, nc, cap_q, cap_c, qb, cb);
    const int q0 = blockIdx.x * (kRThreads * kRQ);
    if (q0 >= nq) return;  // block-uniform
    const int c0 = blockIdx.y * a.slice_len;
    const int c1 = min(nc, c0 + a.slice_len);
    const int tid = threadIdx.x;
    Scalar qx[kRQ], qy[kRQ], qz[kRQ], best[kRQ];
    int bi[kRQ];
#pragma unroll
    for (int r = 0; r < kRQ; ++r) {
        const int qi = min(q0 + r * kRThreads + tid, nq - 1);
        qx[r] = qb[3 * qi];
        qy[r] = qb[3 * qi + 1];
        qz[r] = qb[3 * qi + 2];
        best[r] = (Scalar)INFINITY;
        bi[r] = c0;
    }
    for (int t0 = c0; t0 < c1; t0 += kRTile) {
        const int len = min(kRTile, c1 - t0);
        __syncthreads();
        for (int e = tid; e < len; e += kRThreads) {
            sx[e] = cb[3 * (t0 + e)];
            sy[e] = cb[3 * (t0 + e) + 1];
            sz[e] = cb[3 * (t0 + e) + 2];
        }
        __syncthreads();
        for (int k = 0; k < len; ++k) {
            const Scalar cx = sx[k], cy = sy[k], cz = sz[k];
#pragma unroll
            for (int r = 0; r < kRQ; ++r) {
                const Scalar d = sq3(qx[r], qy[r], qz[r], cx, cy, cz);
                const bool lt = d < best[r];
                best[r] = lt ? d : best[r];
                bi[r] = lt ? t0 + k : bi[r];
            }
        }
    }
    const size_t plane = (size_t)a.b * a.nmax;
    const size_t base = ((size_t)blockIdx.y * 2 + dir) * plane + (size_t)bat * a.nmax;
#pragma unroll
    for (int r = 0; r < kRQ; ++r) {
        const int qi = q0 + r * kRThreads + tid;
        if (qi >= nq) continue;
        a.pd[base + qi] = best[r];
        a.pj[base + qi] = bi[r];
    }
}

// one thread per (dir, batch, row) of the padded outputs
template <typename Scalar>
__global__ __launch_bounds__(256) void nnd_ragged_merge(RaggedArgs<Scalar> a) {
    const int dir = blockIdx.z & 1, bat = blockIdx.z >> 1;
    int nq, nc, cap_q, cap_c;
    const Scalar *qb, *cb;
    dir_view(a, dir, bat, nq, nc, cap_q, cap_c, qb, cb);
    const int qi = blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= cap_q) return;
    Scalar d = (Scalar)0;
    int j = 0;
    if (qi < nq && nc > 0) {
        const size_t plane = (size_t)a.b * a.nmax;
        const int used = (nc + a.slice_len - 1) / a.slice_len;
        d = (Scalar)INFINITY;
        for (int s = 0; s < used; ++s) {
            const size_t o = ((size_t)s * 2 + dir) * plane + (size_t)bat * a.nmax + qi;
            const Scalar v = a.pd[o];
            if (s == 0 || v < d) { d = v; j = a.pj[o]; }
        }
        // my_lib.cpp:16 seed: a NaN distance to candidate 0 freezes (NaN, 0)
        const Scalar d0 = sq3(qb[3 * qi], qb[3 * qi + 1], qb[3 * qi + 2], cb[0], cb[1], cb[2]);
        if (d0 != d0) { d = d0; j = 0; }
    }
    (dir ? a.dist2 : a.dist1)[(size_t)bat * cap_q + qi] = d;
    (dir ? a.idx2 : a.idx1)[(size_t)bat * cap_q + qi] = j;
}

inline int rcdiv(long long x, long long y) { return (int)((x + y - 1) / y); }

template <typename Scalar>
int nnd_ragged(const Scalar *xyz1, const Scalar *xyz2, int32_t b, int32_t n, int32_t m,
               const int32_t *n1, const int32_t *n2, Scalar *dist1, Scalar *dist2, int32_t *idx1,
               int32_t *idx2, pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(b >= 0 && n >= 0 && m >= 0, PCR_ERR_ARG, "nnd_forward_ragged: negative size");
    if (b == 0 || (n == 0 && m == 0)) return PCR_OK;
    PCR_REQUIRE(dist1 && dist2 && idx1 && idx2, PCR_ERR_ARG, "nnd_forward_ragged: null output");
    PCR_REQUIRE((n == 0 || xyz1) && (m == 0 || xyz2), PCR_ERR_ARG, "nnd_forward_ragged: null input");
    PCR_REQUIRE(2LL * b <= 65535, PCR_ERR_ARG, "nnd_forward_ragged: b=%d too large (max 32767)", b);
    hipStream_t s = pcr::as_stream(stream);
    const int nmax = n > m ? n : m;
    const int qtiles = rcdiv(nmax, kRThreads * kRQ);
    // split the candidate axis until the launch has >= ~4 blocks per CU
    int slices = 1;
    while ((long long)qtiles * 2 * b * slices < 4LL * pcr::kCUs && (long long)kRTile * slices * 2 <= nmax)
        slices *= 2;
    RaggedArgs<Scalar> a;
    a.xyz1 = xyz1; a.xyz2 = xyz2; a.n1 = n1; a.n2 = n2;
    a.dist1 = dist1; a.dist2 = dist2; a.idx1 = idx1; a.idx2 = idx2;
    a.b = b; a.n = n; a.m = m; a.nmax = nmax;
    a.slice_len = rcdiv(rcdiv(nmax, slices), kRTile) * kRTile;
    a.slices = rcdiv(nmax, a.slice_len);
    const size_t cells = (size_t)a.slices * 2 * b * nmax;
    char *ws = (char *)pcr::workspace(2, cells * (sizeof(Scalar) + sizeof(int32_t)));
    PCR_REQUIRE(ws, PCR_ERR_NOMEM, "nnd_forward_ragged: %s", pcr_last_error());
    a.pd = (Scalar *)ws;
    a.pj = (int32_t *)(ws + cells * sizeof(Scalar));
    hipLaunchKernelGGL(nnd_ragged_kernel<Scalar>, dim3(qtiles, a.slices, 2 * b), dim3(kRThreads), 0,
                       s, a);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(nnd_ragged_merge<Scalar>, dim3(rcdiv(nmax, 256), 1, 2 * b), dim3(256), 0, s, a);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

}  // namespace

extern "C" int pcr_nnd_forward_ragged(const float *xyz1, const float *xyz2, int32_t b, int32_t n,
                                      int32_t m, const int32_t *n1, const int32_t *n2, float *dist1,
                                      float *dist2, int32_t *idx1, int32_t *idx2,
                                      pcr_stream_t stream) {
    return nnd_ragged<float>(xyz1, xyz2, b, n, m, n1, n2, dist1, dist2, idx1, idx2, stream);
}

extern "C" int pcr_nnd_forward_f64(const double *xyz1, const double *xyz2, int32_t b, int32_t n,
                                   int32_t m, const int32_t *n1, const int32_t *n2, double *dist1,
                                   double *dist2, int32_t *idx1, int32_t *idx2,
                                   pcr_stream_t stream) {
    return nnd_ragged<double>(xyz1, xyz2, b, n, m, n1, n2, dist1, dist2, idx1, idx2, stream);
}
