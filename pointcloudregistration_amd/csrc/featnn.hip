// a5: exact feature-space 1-NN for batches of cloud pairs + mutual filter.
//
// Reference semantics: Open3D KDTreeFlann SearchKNN(k=1) over Feature.data
// inside registration_ransac_based_on_feature_matching (call sites
// DataPreparation/RANSAC.py:43-52, dip/demo.py:43-52, ngenet/utils/o3d.py:174-180)
// and torch.cdist + min in c2p-net/ngenet/models/vote.py:6-9.  Contract
// (oracle_featnn): argmin_j D_ij, D_ij = sum_k ((double)f_ik - (double)g_jk)^2
// summed sequentially in f64, lowest index on ties.
//
// MI355X design: screen every (row, column) pair of a
// cloud pair with an MFMA distance tile, keep a top-2 per row and per column,
// certify a winner when its top-2 gap exceeds a rigorous bound on the screen's
// error, and recompute every uncertified row / column exactly in f64.
//  * D <= 64 (the product's shapes): f16 x3 split operands on
//    v_mfma_f32_32x32x16_f16 (feat_maxabs, feat_pack5r / feat_pack5,
//    featnn_dual7, featnn_colmerge5, featnn_rescan3);
//  * 64 < D <= 128: the augmented f32 operands on v_mfma_f32_32x32x2_f32
//    (featnn_f32.hip).
// Both directions come out of one screen launch.
#include "featnn_common.h"
#include "scan.h"
#include <stdlib.h>
#include <algorithm>
#include <cstdio>
#include <vector>

namespace pcr {
namespace {

// mutual filter + ordered compaction (one block per pair)
__global__ __launch_bounds__(1024) void corres_build(const int32_t *nn12, const int32_t *nn21,
                                                     const int32_t *n_src, const int32_t *n_tgt,
                                                     int Nmax, int Mmax, int mutual, int ransac_n,
                                                     int *scratch, int32_t *corres,
                                                     int32_t *n_corres) {
    const int p = blockIdx.x;
    const int n = count_of(n_src, p, Nmax);
    const int m = count_of(n_tgt, p, Mmax);
    const int32_t *a12 = nn12 + (size_t)p * Nmax;
    const int32_t *a21 = nn21 + (size_t)p * Mmax;
    int *f = scratch + (size_t)p * (Nmax + 1);
    int32_t *co = corres + (size_t)p * Nmax * 2;
    for (int i = threadIdx.x; i < n; i += 1024) {
        const int j = a12[i];
        f[i] = (mutual && j >= 0 && j < m && a21[j] == i) ? 1 : 0;
    }
    __syncthreads();
    block_exclusive_scan_1024(f, f, n, false);
    const int total = f[n];
    const bool use_mutual = mutual && total >= 3 * ransac_n;
    if (use_mutual) {
        for (int i = threadIdx.x; i < n; i += 1024) {
            const int pos = f[i];
            if (f[i + 1] != pos) { co[2 * pos] = i; co[2 * pos + 1] = a12[i]; }
        }
    } else {
        for (int i = threadIdx.x; i < n; i += 1024) { co[2 * i] = i; co[2 * i + 1] = a12[i]; }
    }
    if (threadIdx.x == 0) n_corres[p] = use_mutual ? total : n;
}

// ---------------------------------------------------------------------------
// v5: f16 x3 split screen on v_mfma_f32_32x32x16_f16 (32 cycles per 16-deep
// k-step vs 64 per 2-deep step of the f32 MFMA: 7 instead of 17 x 4 cycles
// per 32x32 tile at D = 32).
//   scale: per pair x = f * 2^e (exact), e chosen so max|x| in [2^(T-1), 2^T)
//          (T = 12 at D <= 64) -> every x fits f16 with room for the products.
//   split: x = hi + lo + e_x, hi = f16(x), lo = f16(x - hi): |e_x| <= 2^-22|x|
//          + 2^-14 (the 2^-14 covers f16 subnormals even if flushed).
//   operands (k order, each D-segment padded to S = ceil(D/16) chunks of 16):
//          A_i = [-2hi | -2hi | -2lo | nx_hi nx_mid nx_lo | c c c | 0 | 2^15]
//          B_j = [  hi |   lo |   hi | c c c | ny_hi ny_mid ny_lo | 2^15 | 0]
//          (norm chunk k = 6 / k = 7: the bias slots.  The G image (role 1)
//          stores 2^15 at k = 6, the F image (role 0) at k = 7; featnn_row8
//          patches the row operand's opposite slot in registers -- 1.0 at k = 6
//          for pass 1 (F rows), k = 7 for pass 2 (G rows), 64 for the 1-term
//          screens -- see kRowBias / kRowBias1)
//          nx = |x|^2 / c split into three f16 parts, c = 2^cs fits f16.
//          Executed: NX = 3S + 1 k-chunks (one MFMA each).  Stored: NM = 2S + 1
//          -- A as [-2hi | -2lo | norms], B as [hi | lo | norms]; the MFMA of
//          chunk c reads A chunk amap(c) and B chunk bmap(c) (the repeated
//          segment is the same registers), so the packed operands, the
//          L2 -> LDS stream and the B-fragment LDS reads are 5/7 of the
//          executed k at D = 32.
//   C = 0 -> d'_ij = |x_i|^2 + |y_j|^2 - 2 x_i.y_j (scaled by 2^2e) with
//   |d' - d'_exact| <= err(q, G) (bound5 below).  Products are exact in f32;
//   the accumulation is charged 2 (Kt + 2) u (|x| + |y|)^2 whatever the
//   MFMA's internal summation order.  Rows/columns whose top-2 gap is not
//   above 2 err are rescanned exactly in f64 (featnn_rescan2).
// Packed layout: [pair][tile][stored chunk][lane] of 8 halves (lane l: row/col l&31,
// k = 16 chunk + 8 (l>>5) + j); padded tiles are valid encodings of +inf
// rows, so no loop has a tail.  Grid: 1-D, XCD-aware: all row blocks of a
// pair run on one XCD, whose L2 then holds that pair's B image (1.8 MB).
// ---------------------------------------------------------------------------
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// executed k-chunk c -> stored A / B chunk (see the operand layout above)
__host__ __device__ constexpr int amap(int c, int S) { return c < S ? c : (c < 3 * S ? c - S : 2 * S); }
__host__ __device__ constexpr int bmap(int c, int S) { return c < 2 * S ? c : (c < 3 * S ? c - 2 * S : 2 * S); }

struct Split5 {
    int T;   // target exponent of max|x|
    int cs;  // norm slot scale c = 2^cs
};
inline Split5 split5_params(int D) {
    int L = 0;
    while ((1 << L) < D) ++L;
    Split5 s;
    s.T = (30 - L) / 2 < 12 ? (30 - L) / 2 : 12;
    s.cs = 2 * s.T + L - 15;
    return s;
}

// Round 5: the pair's scale without a separate pass over the descriptors.
// The split needs every |x s| below 2^T (f16 range of hi / lo and of the norm
// parts); round 4 read both clouds once for their max (feat_maxabs, 537 MB per
// 256-pair step) before the packs read them again.  Now:
//   feat_sample  -- per pair, the max |x| of the first kSampleRows rows of each cloud;
//   the packs    -- scale s = 2^(T - kSpecMargin - 1 - e) for the sample max in
//                   [2^e, 2^(e+1)), i.e. kSpecMargin binades of headroom; a row
//                   with an element at or above 2^T after scaling (or not
//                   finite) flags its pair;
//   repair       -- feat_maxabs and the packs again, for the flagged pairs only
//                   (the round-4 path: s from the full max), launched every
//                   call on a small grid that walks the flags (empty in the
//                   common case).
// The screens' bounds are in the units of the scale actually used (the packs
// store it per pair), so a smaller-than-optimal scale only loosens the
// certification by its absolute (f16 subnormal, norm-split) terms: one binade
// of headroom (any element up to 2-4x the sample's max stays in range) cost
// ~2 % of the bound at the bench's magnitudes; three binades cost 25 % (27 %
// more rows rescanned, measured).
constexpr int kSpecMargin = 1;
constexpr int kSampleRows = 64;  // rows of each cloud in the sample
constexpr int kRepairR = 8;  // repair launches' grid.y (flagged pairs by rank mod R)

// the flagged pairs of rank y, y + R, ... (every wave walks the same flags, so
// control flow stays uniform across the block)
template <class Fn>
__device__ __forceinline__ void for_flagged(const int *bad, int P, int y, int R, Fn fn) {
    const int l = threadIdx.x & 63;
    int rank = 0;
    for (int b = 0; b < P; b += 64) {
        unsigned long long f = __ballot(b + l < P && bad[b + l] != 0);
        while (f) {
            const int q = b + __builtin_ctzll(f);
            f &= f - 1;
            if (rank % R == y) fn(q);
            ++rank;
        }
    }
}

// sample max bits per pair; clears the pair's counters that the stage's later
// launches accumulate into (norm maxima, rescan list counts) and its flag
__global__ __launch_bounds__(256) void feat_sample(const float *F, const int32_t *nf, int Nmax,
                                                   const float *G, const int32_t *ng, int Mmax, int D,
                                                   unsigned *smax, unsigned *clr, int *bad, int P) {
    const int p = blockIdx.x, t = threadIdx.x;
    float m = 0.0f;
    for (int which = 0; which < 2; ++which) {
        const float *x = (which ? G + (size_t)p * Mmax * D : F + (size_t)p * Nmax * D);
        const int rows = min(which ? count_of(ng, p, Mmax) : count_of(nf, p, Nmax), kSampleRows);
        for (int i = t; i < rows * D; i += 256) m = fmaxf(m, fabsf(x[i]));
    }
#pragma unroll
    for (int o = 32; o; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    __shared__ float wm[4];
    if ((t & 63) == 0) wm[t >> 6] = m;
    __syncthreads();
    if (t == 0) {
        smax[p] = __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3])));  // >= 0, never NaN
        clr[p] = 0u;          // gmax
        clr[P + p] = 0u;      // fmax
        clr[3 * P + p] = 0u;  // cnt12
        clr[4 * P + p] = 0u;  // cnt21
        clr[5 * P + p] = 0u;  // gemax
        clr[6 * P + p] = 0u;  // femax
        clr[7 * P + p] = 0u;  // fbc12
        clr[8 * P + p] = 0u;  // fbc21
        bad[p] = 0;
    }
}

// repair: max |element| of each FLAGGED pair's clouds, gridDim.z 1024-thread
// blocks per (pair, cloud), each a contiguous slice of float4 loads; partial
// maxima, one plain store per block (mxp[(p * 2 + which) * Z + z]); block
// (., 0, 0) also clears the pair's norm maxima for the repair packs
__global__ __launch_bounds__(1024) void feat_maxabs(const float *F, const int32_t *nf, int Nmax,
                                                    const float *G, const int32_t *ng, int Mmax,
                                                    int D, unsigned *mxp, unsigned *clr, const int *bad, int P) {
    const int which = blockIdx.y, t = threadIdx.x, z = blockIdx.z, Z = gridDim.z;
    for_flagged(bad, P, blockIdx.x, gridDim.x, [&](int p) {
        const float *X = which ? G : F;
        const int cnt = which ? count_of(ng, p, Mmax) : count_of(nf, p, Nmax);
        const size_t tot = (size_t)cnt * D;
        const float *x = X + (size_t)p * (which ? Mmax : Nmax) * D;
        float m = 0.0f;
        if (((uintptr_t)x & 15) == 0) {
            const float4 *x4 = reinterpret_cast<const float4 *>(x);
            const size_t t4 = tot >> 2;
            const size_t per = (t4 + Z - 1) / Z, lo = min(t4, per * z), hi = min(t4, lo + per);
            for (size_t i = lo + t; i < hi; i += 1024) {
                const float4 v = x4[i];
                m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
            }
            if (z == Z - 1)
                for (size_t i = (t4 << 2) + t; i < tot; i += 1024) m = fmaxf(m, fabsf(x[i]));
        } else {
            for (size_t i = (size_t)z * 1024 + t; i < tot; i += (size_t)Z * 1024) m = fmaxf(m, fabsf(x[i]));
        }
#pragma unroll
        for (int o = 32; o; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        __shared__ float wm[16];
        if ((t & 63) == 0) wm[t >> 6] = m;
        __syncthreads();
        if (t == 0) {
            float r = wm[0];
            for (int w = 1; w < 16; ++w) r = fmaxf(r, wm[w]);
            mxp[((size_t)p * 2 + which) * Z + z] = __float_as_uint(r);  // r >= 0, never NaN
            if (which == 0 && z == 0) {  // gmax, fmax, gemax, femax: the repair packs max into them again
                clr[p] = 0u;
                clr[P + p] = 0u;
                clr[5 * P + p] = 0u;
                clr[6 * P + p] = 0u;
            }
        }
        __syncthreads();
    });
}

// the pair's max |element| from feat_maxabs' 2 Z partials (bits of non-negative
// floats: unsigned order = float order), reduced by every wave on its own
__device__ __forceinline__ unsigned pair_max_bits(const unsigned *mxp, int Z, int p) {
    const int l = threadIdx.x & 63;
    unsigned m = 0u;
    for (int k = l; k < 2 * Z; k += 64) m = max(m, mxp[(size_t)p * 2 * Z + k]);
#pragma unroll
    for (int o = 32; o; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o, 64));
    return m;
}

__device__ __forceinline__ float pair_scale5(unsigned mbits, int T) {
    const int E = (int)((mbits >> 23) & 0xff);
    if (E == 0 || E == 255) return 1.0f;
    const int e = min(max(T + 126 - E, -126), 127);
    return __int_as_float((e + 127) << 23);
}

// Where a pack launch takes its pairs and their scale (see feat_sample):
// normal: grid.y = P, the pair's sample max with kSpecMargin binades of
// headroom, rows outside the split's range flag the pair; repair: grid.y =
// kRepairR, the flagged pairs by rank, the full max from feat_maxabs.
struct PackCtl {
    const unsigned *smax;  // [P] sample max bits (normal)
    const unsigned *mxp;   // [P][2][Z] full partial maxima (repair)
    int Z, P, repair;
    int *bad;              // [P] flags
    unsigned *sc;          // [P] the scale used (f32 bits), for the rescans
};

// both clouds in one launch: blockIdx.z = role (0: F as rows, 1: G as columns)
struct PackIO {
    const float *X[2];
    const int32_t *n[2];
    int Nmax[2], ntiles[2];
    f16x8 *Xp[2];
    float *nrm[2];
    unsigned *nmax[2];
    unsigned *emax[2];  // per pair: max over the cloud's rows of |x s - f16(x s)| (the 1-term screen's bound)
    float *rex[2];      // per row: its |x s - f16(x s)| (rounded up; featnn_regroup9's bound)
    float *ct[2];       // per row: f32(|x s|^2), -1 on padding rows (feat_colterms adds the bias)
};

// |x - f16(x)| of one row (x already scaled), rounded up: e^2 summed exactly
// enough in f64 (each term exact), the sqrt's rounding covered by the factor
__device__ __forceinline__ float split_err_norm(double e2) {
    return (float)(__builtin_sqrt(e2) * (1.0 + 1e-6));
}

// one atomic per workgroup: max of the four waves' values (bit patterns of
// non-negative floats; unsigned order = float order)
__device__ __forceinline__ void block_max_atomic(unsigned v, unsigned *wm, unsigned *dst) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v = max(v, (unsigned)__shfl_xor((int)v, o, 64));
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned m = max(max(wm[0], wm[1]), max(wm[2], wm[3]));
        if (m != 0u) atomicMax(dst, m);
    }
}

template <class Body>
__device__ __forceinline__ void pack_pairs(const PackCtl &c, int T, Body body) {
    if (!c.repair) {
        const int p = blockIdx.y;
        const float s = pair_scale5(c.smax[p], T - kSpecMargin);
        if (blockIdx.x == 0 && threadIdx.x == 0) c.sc[p] = __float_as_uint(s);
        body(p, s, true);
    } else {
        for_flagged(c.bad, c.P, blockIdx.y, gridDim.y, [&](int p) {
            const float s = pair_scale5(pair_max_bits(c.mxp, c.Z, p), T);
            if (blockIdx.x == 0 && threadIdx.x == 0) c.sc[p] = __float_as_uint(s);
            body(p, s, false);
            __syncthreads();  // the block's LDS is reused by the next pair
        });
    }
}

// role 0: rows (A), role 1: columns (B).  256-thread blocks, one wave per
// 32-row tile; each tile is staged through LDS with coalesced loads (scaled,
// exact) and every lane emits its 2S + 1 stored 16-byte operand fragments.
__global__ __launch_bounds__(256) void feat_pack5(PackIO io, int D, int S, Split5 sp, PackCtl pc) {
    const int role = blockIdx.z;
    const float *X = io.X[role];
    const int32_t *n = io.n[role];
    const int Nmax = io.Nmax[role], ntiles = io.ntiles[role];
    f16x8 *Xp = io.Xp[role];
    float *nrm = io.nrm[role];
    unsigned *nmax = io.nmax[role];
    if ((int)blockIdx.x * 4 >= ntiles) return;  // whole block: the other cloud has more tiles
    __shared__ float xs[4][32][65];  // D <= 64 (+1 pad: conflict-free row reads)
    __shared__ unsigned wmax[4];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + w;  // ntiles is a multiple of 8 (host pads)
    const float lim = __builtin_ldexpf(1.0f, sp.T);
    pack_pairs(pc, sp.T, [&](int p, float s, bool check) {
        const int cnt = count_of(n, p, Nmax);
        const int nrows = min(max(cnt - t * 32, 0), 32);
        const float *base = X + ((size_t)p * Nmax + (size_t)t * 32) * D;
        float (*x)[65] = xs[w];
        // e / D by a 64-bit reciprocal (exact for e < 2^16; 2^32/D + 1 needs 33 bits at D = 1)
        const unsigned long long invD = 0xFFFFFFFFull / (unsigned long long)D + 1ull;
        bool ok = true;
        for (int e = l; e < 32 * D; e += 64) {
            const int r = (int)(((unsigned long long)e * invD) >> 32), k = e - r * D;
            const float v = r < nrows ? base[e] * s : 0.0f;
            ok = ok && __builtin_fabsf(v) < lim;  // NaN / inf: not ok
            x[r][k] = v;
        }
        if (check && !ok) pc.bad[p] = 1;
        __syncthreads();
        const int rr = l & 31, h = l >> 5;
        const bool valid = rr < nrows;
        double acc = 0.0, ea = 0.0;
        for (int k = 0; k < D; ++k) {
            const double v = (double)x[rr][k];
            acc = acc + v * v;
            const double e = (double)(x[rr][k] - (float)(_Float16)x[rr][k]);  // exact in f32
            ea = ea + e * e;
        }
        // norm parts of acc / c (exact power-of-two division)
        _Float16 np[3];
        if (valid) {
            double wv = acc * __builtin_ldexp(1.0, -sp.cs);
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                np[q] = (_Float16)(float)wv;  // |wv| < 2^15: double->float->half may round twice;
                wv = wv - (double)np[q];      // the bound charges 2^-11 per part regardless
            }
        } else {
            // finite sentinel 3 * 65504 * c > any real distance (<= 4 D 2^2T):
            // index bits are OR-ed into screen values, which must not be inf
            np[0] = (_Float16)65504.0f;
            np[1] = (_Float16)65504.0f;
            np[2] = (_Float16)65504.0f;
        }
        const _Float16 cval = (_Float16)__builtin_ldexpf(1.0f, sp.cs);
        const int NM = 2 * S + 1;
        f16x8 *dst = Xp + ((size_t)p * ntiles + t) * NM * 64 + l;
        for (int c = 0; c < NM; ++c) {
            f16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int seg = c < S ? 0 : (c < 2 * S ? 1 : 2);   // hi | lo | norms
                const int k = 16 * (c - seg * S) + 8 * h + j;      // index inside the segment
                _Float16 v = (_Float16)0.0f;
                if (seg < 2) {
                    if (k < D) {
                        const float xv = x[rr][k];
                        const _Float16 hi = (_Float16)xv;
                        const _Float16 lo = (_Float16)(xv - (float)hi);
                        const _Float16 part = seg == 0 ? hi : lo;
                        v = role == 0 ? (_Float16)(-2.0f * (float)part) : part;
                    }
                } else {
                    if (k < 3) v = role == 0 ? np[k] : cval;
                    else if (k < 6) v = role == 0 ? cval : np[k - 3];
                    else if (k == 6 && role == 1) v = (_Float16)32768.0f;  // featnn_row8's biases
                    else if (k == 7 && role == 0) v = (_Float16)32768.0f;
                }
                o[j] = v;
            }
            dst[(size_t)c * 64] = o;
        }
        // the pair's max norm: one atomic per WORKGROUP.  The P words share a few
        // cache lines, and one atomic per wave (256 per cloud) serialised at the
        // L2: ~80 us per launch whatever the batch.  Max of the bit patterns: the
        // same word per-lane atomics would leave, NaN included.
        const float r = (h == 0 && valid) ? (float)__builtin_sqrt(acc) : 0.0f;
        if (h == 0) {
            nrm[(size_t)p * ntiles * 32 + t * 32 + rr] = r;
            io.rex[role][(size_t)p * ntiles * 32 + t * 32 + rr] = valid ? split_err_norm(ea) : 0.0f;
            io.ct[role][(size_t)p * ntiles * 32 + t * 32 + rr] = valid ? (float)acc : -1.0f;
        }
        block_max_atomic(__float_as_uint(r), wmax, nmax + p);
        __syncthreads();
        block_max_atomic(valid ? __float_as_uint(split_err_norm(ea)) : 0u, wmax, io.emax[role] + p);
    });
}

// Register-resident pack for a compile-time D (the hot D = 32): one lane per
// (row, half), the row loaded with 16-byte loads (both halves of the wave share
// the cache lines), the split computed once per element, and each 16-byte
// operand fragment selected between the two compile-time candidates of the
// lane's half -- no LDS, no per-half segment arithmetic.  Same values as
// feat_pack5 (same operations, same order).
template <int D>
__global__ __launch_bounds__(256) void feat_pack5r(PackIO io, Split5 sp, PackCtl pc) {
    const int role = blockIdx.z;
    const float *X = io.X[role];
    const int32_t *n = io.n[role];
    const int Nmax = io.Nmax[role], ntiles = io.ntiles[role];
    f16x8 *Xp = io.Xp[role];
    float *nrm = io.nrm[role];
    unsigned *nmax = io.nmax[role];
    if ((int)blockIdx.x * 4 >= ntiles) return;  // whole block: the other cloud has more tiles
    constexpr int S = (D + 15) / 16;  // chunks per segment
    constexpr int NM = 2 * S + 1;     // stored chunks
    constexpr int G = 2 * S;          // 8-half fragments per segment
    __shared__ unsigned wmax[4];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + w;  // ntiles is a multiple of 8 (host pads)
    const float lim = __builtin_ldexpf(1.0f, sp.T);
    pack_pairs(pc, sp.T, [&](int p, float s, bool check) {
        const int cnt = count_of(n, p, Nmax);
        const int nrows = min(max(cnt - t * 32, 0), 32);
        const int rr = l & 31, h = l >> 5;
        const bool valid = rr < nrows;
        float x[D];
        if (valid) {
            const float4 *row = reinterpret_cast<const float4 *>(X + ((size_t)p * Nmax + (size_t)t * 32 + rr) * D);
#pragma unroll
            for (int q = 0; q < D / 4; ++q) {
                const float4 v = row[q];
                x[4 * q] = v.x * s; x[4 * q + 1] = v.y * s; x[4 * q + 2] = v.z * s; x[4 * q + 3] = v.w * s;
            }
        } else {
#pragma unroll
            for (int k = 0; k < D; ++k) x[k] = 0.0f;
        }
        if (check) {
            bool ok = true;
#pragma unroll
            for (int k = 0; k < D; ++k) ok = ok && __builtin_fabsf(x[k]) < lim;  // NaN / inf: not ok
            if (!ok) pc.bad[p] = 1;
        }
        double acc = 0.0, ea = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const double v = (double)x[k];
            acc = acc + v * v;
            const double e = (double)(x[k] - (float)(_Float16)x[k]);  // exact in f32
            ea = ea + e * e;
        }
        _Float16 np[3];
        if (valid) {
            double wv = acc * __builtin_ldexp(1.0, -sp.cs);
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                np[q] = (_Float16)(float)wv;
                wv = wv - (double)np[q];
            }
        } else {
            np[0] = (_Float16)65504.0f;
            np[1] = (_Float16)65504.0f;
            np[2] = (_Float16)65504.0f;
        }
        const _Float16 cval = (_Float16)__builtin_ldexpf(1.0f, sp.cs);
        _Float16 s0[D], s1[D];  // the two stored segments of this role: hi | lo
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const _Float16 hi = (_Float16)x[k];
            const _Float16 lo = (_Float16)(x[k] - (float)hi);
            if (role == 0) {
                s0[k] = (_Float16)(-2.0f * (float)hi);
                s1[k] = (_Float16)(-2.0f * (float)lo);
            } else {
                s0[k] = hi;
                s1[k] = lo;
            }
        }
        auto frag = [&](int g) {  // compile-time g after unrolling
            f16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                _Float16 v = (_Float16)0.0f;
                const int k0 = 8 * (g % G) + j;
                if (g < G) v = k0 < D ? s0[k0 < D ? k0 : 0] : (_Float16)0.0f;
                else if (g < 2 * G) v = k0 < D ? s1[k0 < D ? k0 : 0] : (_Float16)0.0f;
                else if (g == 2 * G) {
                    if (j < 3) v = role == 0 ? np[j] : cval;
                    else if (j < 6) v = role == 0 ? cval : np[j - 3];
                    else if (j == 6 && role == 1) v = (_Float16)32768.0f;  // featnn_row8's biases
                    else if (j == 7 && role == 0) v = (_Float16)32768.0f;
                }
                o[j] = v;
            }
            return o;
        };
        f16x8 *dst = Xp + ((size_t)p * ntiles + t) * NM * 64 + l;
#pragma unroll
        for (int c = 0; c < NM; ++c) {
            const f16x8 a = frag(2 * c), b = frag(2 * c + 1);
            dst[(size_t)c * 64] = h ? b : a;
        }
        // the pair's max norm: one atomic per WORKGROUP (see feat_pack5)
        const float r = (h == 0 && valid) ? (float)__builtin_sqrt(acc) : 0.0f;
        if (h == 0) {
            nrm[(size_t)p * ntiles * 32 + t * 32 + rr] = r;
            io.rex[role][(size_t)p * ntiles * 32 + t * 32 + rr] = valid ? split_err_norm(ea) : 0.0f;
            io.ct[role][(size_t)p * ntiles * 32 + t * 32 + rr] = valid ? (float)acc : -1.0f;
        }
        block_max_atomic(__float_as_uint(r), wmax, nmax + p);
        __syncthreads();
        block_max_atomic(valid ? __float_as_uint(split_err_norm(ea)) : 0u, wmax, io.emax[role] + p);
    });
}

// certification threshold for a top-2 gap in scaled units (see header)
__device__ __forceinline__ double bound5(double q, double G, int Kt, int D) {
    const double u = 5.9604644775390625e-08;  // 2^-24
    const double qg = q + G;
    const double err = 2.0 * (Kt + 2) * u * qg * qg + 6.0 * 2.384185791015625e-07 * q * G +
                       1.220703125e-04 * __builtin_sqrt((double)D) * qg +
                       1.1641532182693481e-10 * (q * q + G * G) + 4.0;
    return 2.0 * err;
}

struct DualArgs5 {
    const f16x8 *Ap, *Bp;
    const float *fnr, *gnr;  // scaled norms
    const unsigned *fmax, *gmax;
    const int32_t *n_src, *n_tgt;
    int P, Nmax, Mmax, ntn, ntm, nrb, D, ctbits;
    int32_t *nn12;
    int *list12, *count12;
    float *cp1, *cp2;
    int *cpi;
};

// raw v_min / v_med3 on bit-packed values: as builtins the compiler inserts a
// NaN canonicalisation (v_max x,x) per packed operand.  Inputs are never
// signalling NaNs; a quiet NaN (NaN feature) is ignored by IEEE min, as the
// oracle's strict < ignores it, or forces a rescan.
// NEVER feed an MFMA accumulator straight into these: the compiler does not
// place the MFMA read-after-write wait states in front of inline asm, and the
// first registers read come back without the chain's last MFMA (measured:
// featnn_row7 with asm reads of acc).  Here every operand comes from a
// compiler-visible instruction (the index pack).
__device__ __forceinline__ float vmin(float a, float b) {
    float d;
    asm("v_min_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
// a NaN operand yields the other value: the pair's second value then equals its
// first (a tie), which only fails certification (exact rescan)
__device__ __forceinline__ float vmax(float a, float b) {
    float d;
    asm("v_max_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
__device__ __forceinline__ float vmed3(float a, float b, float c) {
    float d;
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// ---------------------------------------------------------------------------
// v7 = v5 with an in-wave software pipeline.  Ablations of v5 showed its
// phases add: MFMA chain (after its B-fragment LDS reads have landed) and
// the VALU epilogue never overlap.  Here iteration g of a group issues, in one
// scheduling region, the 7 MFMAs of tile g, the ds_read_b128 B fragments of
// tile g+1 (register double buffer) and the epilogue of tile g-1, interleaved
// 1 MFMA : 1 LDS read : V VALU by sched_group_barrier.  G = 8 tiles per LDS
// group halves the barriers (B double buffer 2 x 57 KB + partials 32 KB).
// ---------------------------------------------------------------------------
template <int S, int G>
__global__ __launch_bounds__(512) void featnn_dual7(DualArgs5 a) {
    constexpr int W = 8;  // waves per workgroup, one 32-row tile each
    constexpr int NX = 3 * S + 1, NM = 2 * S + 1;  // executed / stored k-chunks
    constexpr int kB = G * NM * 64;  // f16x8 per B buffer
    constexpr int kP = G * W * 32;
    __shared__ __attribute__((aligned(16))) char smem[2 * kB * 16 + 2 * 2 * kP * 4];
    // column partials first: their per-tile stores then fit the ds_write
    // immediate offset (below 64 KiB), the B buffers follow
    float *Pc1 = reinterpret_cast<float *>(smem);  // [2][G][W waves][32 cols]
    float *Pc2 = Pc1 + 2 * kP;
    f16x8 *Bs = reinterpret_cast<f16x8 *>(smem + 2 * 2 * kP * 4);
    const int b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const int p = (slot / a.nrb) * 8 + xcd, rb = slot - (slot / a.nrb) * a.nrb;
    if (p >= a.P) return;  // whole block
    const int wid = threadIdx.x >> 6, l = threadIdx.x & 63, h = l >> 5;
    const int n = count_of(a.n_src, p, a.Nmax), m = count_of(a.n_tgt, p, a.Mmax);
    const int qt = rb * W + wid;
    const int ntc = (m + 31) >> 5;
    const int ngroups = (ntc + G - 1) / G;
    const unsigned ctmask = (1u << a.ctbits) - 1u;
    unsigned keep_r = ~ctmask;
    asm("" : "+v"(keep_r));
    unsigned ccode[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        ccode[r] = (unsigned)((wid << 5) | (h << 4) | r);
        asm("" : "+v"(ccode[r]));
    }
    f16x8 A[NM];
    const f16x8 *qp = a.Ap + ((size_t)p * a.ntn + qt) * NM * 64 + l;
#pragma unroll
    for (int c = 0; c < NM; ++c) A[c] = qp[(size_t)c * 64];
    float b1[16], b2[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) { b1[r] = __builtin_inff(); b2[r] = __builtin_inff(); }

    const f16x8 *bsrc = a.Bp + (size_t)p * a.ntm * NM * 64 + l;
    auto issue = [&](int grp, int bufi) {
        for (int c = wid; c < G * NM; c += W) {
            const f16x8 *src = bsrc + ((size_t)grp * G * NM + c) * 64;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)src,
                (__attribute__((address_space(3))) void *)(Bs + bufi * kB + c * 64), 16, 0, 0);
        }
    };
    auto epilogue = [&](const f32x16 &acc, unsigned ct, int pbase, int pe) {
        asm("" : "+s"(ct));
        float c1[2], c2[2];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const unsigned ub = __float_as_uint(acc[r]);
            const float vr = __uint_as_float((ub & keep_r) | ct);
            const float vc = __uint_as_float((ub & 0xFFFFFF00u) | ccode[r]);
            b2[r] = vmed3(b1[r], b2[r], vr);
            b1[r] = vmin(b1[r], vr);
            // column top-2 of the lane's 16 values in two interleaved chains
            // (one merge; no +inf staged: the first two values give min / max)
            const int q = r & 1;
            if (r < 2) {
                c1[q] = vc;
            } else if (r < 4) {
                c2[q] = vmax(c1[q], vc);
                c1[q] = vmin(c1[q], vc);
            } else {
                c2[q] = vmed3(c1[q], c2[q], vc);
                c1[q] = vmin(c1[q], vc);
            }
        }
        {
            const float m2 = vmin(c2[0], c2[1]);
            c2[0] = vmed3(c1[0], c1[1], m2);
            c1[0] = vmin(c1[0], c1[1]);
        }
        // merge with the other half-wave without LDS (a ds_bpermute here would share
        // lgkmcnt with the B-fragment reads in flight).  One swap of (c1, c2)
        // leaves lanes 0-31 with (own c1, other c1) and lanes 32-63 with
        // (own c2, other c2): their min is the new c1 below and min(c2, c2')
        // above, which a second swap brings down for the med3 -- 5 VALU, where
        // swapping c1 and c2 separately needed 4 copies more.
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(c1[0]),
                                                         __float_as_uint(c2[0]), false, false);
        const float lo = __uint_as_float(sw[0]), up = __uint_as_float(sw[1]);
        const float mm = vmin(lo, up);
        const auto sw2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(mm), __float_as_uint(mm),
                                                          false, false);
        c2[0] = vmed3(lo, up, __uint_as_float(sw2[1]));
        c1[0] = __uint_as_float(sw2[0]);  // lanes 0-31 of the swapped mm: mm itself
        if (h == 0) {
            const int e = pbase + pe * (W * 32);  // pe: compile-time tile of the group
            Pc1[e] = c1[0];
            Pc2[e] = c2[0];
        }
    };
    const size_t cpoff = ((size_t)p * a.nrb + rb) * (size_t)a.ntm * 32;
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int grp = 0; grp < ngroups; ++grp) {
        const int buf = grp & 1;
        if (grp + 1 < ngroups) issue(grp + 1, buf ^ 1);
        const f16x8 *Bb = Bs + buf * kB + l;
        const int pbase = buf * (G * W * 32) + wid * 32 + l;  // this group's column partials
        f16x8 Bf[2][NM];
        f32x16 acc[2];
#pragma unroll
        for (int c = 0; c < NM; ++c) Bf[0][c] = Bb[c * 64];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int cur = g & 1;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[cur][r] = 0.0f;
#pragma unroll
            for (int c = 0; c < NX; ++c)
                acc[cur] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[amap(c, S)], Bf[cur][bmap(c, S)], acc[cur],
                                                                  0, 0, 0);
            if (g + 1 < G) {
#pragma unroll
                for (int c = 0; c < NM; ++c) Bf[cur ^ 1][c] = Bb[((g + 1) * NM + c) * 64];
            }
            if (g > 0) epilogue(acc[cur ^ 1], (unsigned)(grp * G + g - 1), pbase, g - 1);
            // one region per iteration: MFMA : LDS read : VALU = 1 : 1 : 18
#pragma unroll
            for (int c = 0; c < NX; ++c) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if (g + 1 < G && c < NM) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                if (g > 0) __builtin_amdgcn_sched_group_barrier(0x002, 18, 0);
            }
        }
        epilogue(acc[(G - 1) & 1], (unsigned)(grp * G + G - 1), pbase, G - 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const int t = threadIdx.x;
        if (t < G * 32) {
            const int g = t >> 5, col = t & 31, ct = grp * G + g;
            if (ct < ntc) {
                const int e0 = (buf * G + g) * (W * 32) + col;
                float m1 = Pc1[e0], mm2 = Pc2[e0];
#pragma unroll
                for (int w = 1; w < W; ++w) {
                    const float o1 = Pc1[e0 + 32 * w], o2 = Pc2[e0 + 32 * w];
                    const float t2 = vmin(mm2, o2);
                    mm2 = vmed3(m1, o1, t2);
                    m1 = vmin(m1, o1);
                }
                // no row index stored: featnn_colmerge5 decodes it from m1's
                // code bits (a third fewer column-partial bytes written and read)
                const size_t o = cpoff + (size_t)ct * 32 + col;
                a.cp1[o] = m1;
                a.cp2[o] = mm2;
            }
        }
    }
    if (qt * 32 >= n) return;
    int i1[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) i1[r] = (int)(__float_as_uint(b1[r]) & ctmask) * 32 + (l & 31);
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float ob1 = __shfl_xor(b1[r], o, 64);
            const float ob2 = __shfl_xor(b2[r], o, 64);
            const int oi1 = __shfl_xor(i1[r], o, 64);
            top2_merge(b1[r], i1[r], b2[r], ob1, oi1, ob2);
        }
    }
    const int lr = l & 31;
    if (lr >= 16) return;
    float mb1 = 0.f, mb2 = 0.f;
    int mi1 = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r)
        if (lr == r) { mb1 = b1[r]; mb2 = b2[r]; mi1 = i1[r]; }
    const int row = qt * 32 + (lr & 3) + 8 * (lr >> 2) + 4 * h;
    if (row >= n) return;
    if (m == 0) { a.nn12[(size_t)p * a.Nmax + row] = 0; return; }
    a.nn12[(size_t)p * a.Nmax + row] = mi1;
    const double Gm = (double)__uint_as_float(a.gmax[p]);
    const double qn = (double)a.fnr[(size_t)p * a.ntn * 32 + row];
    const double pert = __builtin_ldexp(1.0, a.ctbits - 23) *
                        (__builtin_fabs((double)mb1) + __builtin_fabs((double)mb2));
    if (!((double)mb2 - (double)mb1 > bound5(qn, Gm, 16 * NX, a.D) + pert))
        a.list12[(size_t)p * a.Nmax + atomicAdd(a.count12 + p, 1)] = row;
}

__global__ void featnn_colmerge5(DualArgs5 a, int32_t *nn21, int *list21, int *count21, int Kt,
                                 int W) {
    const int p = blockIdx.y;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int m = count_of(a.n_tgt, p, a.Mmax);
    if (j >= m) return;
    const int n = count_of(a.n_src, p, a.Nmax);
    if (n == 0) { nn21[(size_t)p * a.Mmax + j] = 0; return; }
    const int nrb_used = (((n + 31) >> 5) + 7) >> 3;
    float b1 = __builtin_inff(), b2 = __builtin_inff();
    int i1 = 0;
    for (int rb = 0; rb < nrb_used; ++rb) {
        const size_t o = ((size_t)p * a.nrb + rb) * (size_t)a.ntm * 32 + j;
        // row index of the partial's winner from its code bits (wave, half,
        // register), as the screen kernels packed them
        const float v1 = a.cp1[o];
        const unsigned code = __float_as_uint(v1) & (unsigned)(W * 32 - 1);
        const int r = code & 15;
        const int vi = rb * (W * 32) + (int)(code >> 5) * 32 + (int)((code >> 4) & 1) * 4 + (r & 3) + 8 * (r >> 2);
        top2_merge(b1, i1, b2, v1, vi, a.cp2[o]);
    }
    nn21[(size_t)p * a.Mmax + j] = i1;
    const double F = (double)__uint_as_float(a.fmax[p]);
    const double gn = (double)a.gnr[(size_t)p * a.ntm * 32 + j];
    const double pert = 3.0517578125e-05 /* 2^-15: 8-bit row code */ *
                        (__builtin_fabs((double)b1) + __builtin_fabs((double)b2));
    if (!((double)b2 - (double)b1 > bound5(gn, F, Kt, a.D) + pert))
        list21[(size_t)p * a.Mmax + atomicAdd(count21 + p, 1)] = j;
}

// exact f64 rescan of v5's per-pair ambiguous lists: one 256-thread block per
// batch of R listed rows of one pair and direction; the rows sit in LDS as
// f64, every thread streams candidates j = tid + 256 i once (float4 rows) and
// keeps R running minima, so a pair's candidate cloud is read once per batch
// instead of once per row.  blockIdx.z = direction (0: F->G, 1: G->F).
// rows sent to the exact rescan since the last reset (diagnostic, pcr_featnn_rescan_rows)
__device__ unsigned long long g_featnn_rescan_rows[2];

struct RescanArgs5 {
    const float *F, *G;
    const int32_t *n_src, *n_tgt;
    int Nmax, Mmax, D;
    const int *list12, *list21, *cnt12, *cnt21;
    int32_t *nn12, *nn21;
    // candidate slices (gridDim.z = S): the first `cap` listed rows of a pair and
    // direction are scanned by S blocks over disjoint candidate ranges, each
    // writing its lexicographic (d, j) minimum to slot (p, dir, e, s), merged by
    // featnn_rescan_merge; rows past `cap` are scanned whole by slice 0
    int cap;
    double *sd;
    int *sj;
    // mutual path (feature_corres_v5): the exact distance of a rescanned F row,
    // in the screen's scaled units (x s^2, s = pair_scale5(mx[p], T): a power of
    // two, exact), and its error 0; null elsewhere
    double *v12;
    float *e12;
    const unsigned *mx;
    int T;
};

__device__ __forceinline__ void rescan_out(const RescanArgs5 &a, int dir, int p, int row, double best,
                                           int bj, int32_t *nn) {
    nn[row] = (bj == 0x7fffffff) ? 0 : bj;
    if (dir == 0 && a.v12) {
        const double sc = (double)__uint_as_float(a.mx[p]);  // the scale the packs used
        a.v12[(size_t)p * a.Nmax + row] = best * sc * sc;
        a.e12[(size_t)p * a.Nmax + row] = 0.0f;
    }
}

typedef float f2v __attribute__((ext_vector_type(2)));

template <int DV, bool V4>
__global__ __launch_bounds__(256) void featnn_rescan3(RescanArgs5 a) {
    // thread (row r = tid>>3, slice sl = tid&7): row r of the current batch of
    // 32 listed rows (held as f64 in registers) against candidates sl, sl+8,
    // ... of each 128-candidate chunk staged in LDS.  Row stride DV+4 floats:
    // the 8 slices' ds_read_b128 hit disjoint banks, the rows of a slice
    // broadcast.  Dims in [D, DV) are zero on both sides (exact zero terms).
    constexpr int kChunk = 128, kSt = DV + 4;
    __shared__ __attribute__((aligned(16))) float csb[2][kChunk * kSt];  // double buffer (V4 path)
    const int dir = blockIdx.y, p = blockIdx.x, S = gridDim.z, sid = blockIdx.z;
    const int tid = threadIdx.x, r = tid >> 3, sl = tid & 7;
    const float *Q = dir ? a.G : a.F;
    const float *C = dir ? a.F : a.G;
    const int Nq = dir ? a.Mmax : a.Nmax, Nc = dir ? a.Nmax : a.Mmax;
    const int ncand = count_of(dir ? a.n_src : a.n_tgt, p, Nc);
    const int *list = (dir ? a.list21 : a.list12) + (size_t)p * Nq;
    const int cnt = (dir ? a.cnt21 : a.cnt12)[p];
    if (tid == 0 && sid == 0 && cnt > 0) atomicAdd(&g_featnn_rescan_rows[dir], (unsigned long long)cnt);
    int32_t *nn = (dir ? a.nn21 : a.nn12) + (size_t)p * Nq;
    const int D = a.D;
    const float *cb = C + (size_t)p * Nc * D;
    // this slice's candidates: whole 128-candidate chunks [clo, chi)
    const int nchunk = (ncand + kChunk - 1) / kChunk;
    const int clo = S > 1 ? min(ncand, (int)((long long)nchunk * sid / S) * kChunk) : 0;
    const int chi = S > 1 ? min(ncand, (int)((long long)nchunk * (sid + 1) / S) * kChunk) : ncand;
    const int ecap = S > 1 ? min(cnt, a.cap) : 0;  // rows handled by the slices
    // slices take rows [0, ecap); slice 0 also the rows past the cap, whole
    for (int b0 = 0; b0 < (sid > 0 ? ecap : cnt); b0 += 32) {
        const bool sliced = b0 < ecap;
        const int c_lo = sliced ? clo : 0, c_hi = sliced ? chi : ncand;
        const int bend = sliced ? ecap : cnt;
        const bool act = b0 + r < bend;
        const int row = act ? list[b0 + r] : 0;
        const float *q = Q + ((size_t)p * Nq + row) * D;
        double qd[DV];
        float qf[DV];
#pragma unroll
        for (int k = 0; k < DV; ++k) {
            qf[k] = k < D ? q[k] : 0.0f;
            qd[k] = (double)qf[k];
        }
        double best = __builtin_inf();
        int bj = 0x7fffffff;
        float m32 = __builtin_inff();
        const float kRel = 1.0f + 3.0f * (float)(D + 5) * 5.9604644775390625e-08f;
        // candidate chunk -> registers -> LDS; with V4 the next chunk's global
        // loads are in flight while the current chunk is scanned
        constexpr int kPer = kChunk * (DV / 4) / 256;  // float4 per thread per chunk
        float4 stage[kPer];
        auto gload = [&](int c0, int cend) {
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                const int e = tid + 256 * u, i = e / (DV / 4), k = (e - i * (DV / 4)) * 4;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (c0 + i < cend && k < D)
                    v = *reinterpret_cast<const float4 *>(cb + (size_t)(c0 + i) * D + k);
                stage[u] = v;
            }
        };
        auto lstore = [&](float *cs) {
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                const int e = tid + 256 * u, i = e / (DV / 4), k = (e - i * (DV / 4)) * 4;
                *reinterpret_cast<float4 *>(cs + i * kSt + k) = stage[u];
            }
        };
        auto scan = [&](const float *cs, int c0, int ncand) {
            // f32 screen of the thread's kChunk / 8 candidates (packed: two
            // dims per v_pk_fma): all terms are >= 0, so |d32 - d| <= (D+3) u d
            // whatever the order; only candidates within kRel of the thread's
            // running f32 minimum after the chunk (>= the global one) can be
            // the exact winner.  Those are re-ranked in f64 AFTER the chunk's
            // screen, in candidate order (first index on ties): a wave runs
            // one or two f64 ranks per chunk instead of one wherever any lane
            // had a running-minimum candidate (~a quarter of the steps).
            constexpr int kPer8 = kChunk / 8;
            float a32v[kPer8];
#pragma unroll
            for (int t = 0; t < kPer8; ++t) {
                const int i = sl + 8 * t;
                float a32 = __builtin_inff();
                if (i < ncand) {
                    const float *cp = cs + i * kSt;
                    f2v acc = {0.0f, 0.0f};
#pragma unroll
                    for (int k = 0; k < DV; k += 4) {
                        const float4 v = *reinterpret_cast<const float4 *>(cp + k);
                        const f2v d0 = f2v{v.x, v.y} - f2v{qf[k], qf[k + 1]};
                        const f2v d1 = f2v{v.z, v.w} - f2v{qf[k + 2], qf[k + 3]};
                        acc = __builtin_elementwise_fma(d0, d0, acc);
                        acc = __builtin_elementwise_fma(d1, d1, acc);
                    }
                    a32 = acc.x + acc.y;
                }
                a32v[t] = a32;
                m32 = fminf(m32, a32);
            }
            const float lim = m32 * kRel + 1e-30f;
            unsigned pend = 0;
#pragma unroll
            for (int t = 0; t < kPer8; ++t) pend |= (sl + 8 * t < ncand && a32v[t] <= lim ? 1u : 0u) << t;
            while (pend) {
                const int t = __builtin_ctz(pend);
                pend &= pend - 1;
                const int i = sl + 8 * t;
                const float *cp = cs + i * kSt;
                double acc = 0.0;
#pragma unroll
                for (int k = 0; k < DV; k += 4) {
                    const float4 v = *reinterpret_cast<const float4 *>(cp + k);
                    double df = qd[k] - (double)v.x;
                    acc = acc + df * df;
                    df = qd[k + 1] - (double)v.y;
                    acc = acc + df * df;
                    df = qd[k + 2] - (double)v.z;
                    acc = acc + df * df;
                    df = qd[k + 3] - (double)v.w;
                    acc = acc + df * df;
                }
                if (acc < best) { best = acc; bj = c0 + i; }
            }
        };
        if (V4) {
            __syncthreads();  // previous batch done with both buffers
            if (c_lo < c_hi) {
                gload(c_lo, c_hi);
                lstore(csb[0]);
            }
            __syncthreads();
            int buf = 0;
            for (int c0 = c_lo; c0 < c_hi; c0 += kChunk, buf ^= 1) {
                const bool more = c0 + kChunk < c_hi;
                if (more) gload(c0 + kChunk, c_hi);
                scan(csb[buf], c0, min(kChunk, c_hi - c0));
                if (more) lstore(csb[buf ^ 1]);  // read last in the previous iteration
                __syncthreads();
            }
        } else {
            for (int c0 = c_lo; c0 < c_hi; c0 += kChunk) {
                const int nin = min(kChunk, c_hi - c0);
                __syncthreads();  // previous chunk fully consumed
                for (int e = tid; e < kChunk * DV; e += 256) {
                    const int i = e / DV, k = e - i * DV;
                    csb[0][i * kSt + k] = (i < nin && k < D) ? cb[(size_t)(c0 + i) * D + k] : 0.0f;
                }
                __syncthreads();
                scan(csb[0], c0, nin);
            }
        }
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) {
            const double ob = __shfl_xor(best, o, 64);
            const int oj = __shfl_xor(bj, o, 64);
            if (ob < best || (ob == best && oj < bj)) { best = ob; bj = oj; }
        }
        if (sl == 0 && act) {
            if (sliced) {
                const size_t slot = (((size_t)p * 2 + dir) * a.cap + b0 + r) * S + sid;
                a.sd[slot] = best;
                a.sj[slot] = bj;
            } else {
                rescan_out(a, dir, p, row, best, bj, nn);
            }
        }
    }
}

// lexicographic (d, j) minimum of the S slice results of each sliced row
__global__ __launch_bounds__(256) void featnn_rescan_merge(RescanArgs5 a, int S) {
    const int dir = blockIdx.y, p = blockIdx.x;
    const int Nq = dir ? a.Mmax : a.Nmax;
    const int cnt = min((dir ? a.cnt21 : a.cnt12)[p], a.cap);
    const int *list = (dir ? a.list21 : a.list12) + (size_t)p * Nq;
    int32_t *nn = (dir ? a.nn21 : a.nn12) + (size_t)p * Nq;
    for (int e = threadIdx.x; e < cnt; e += 256) {
        const size_t slot = (((size_t)p * 2 + dir) * a.cap + e) * S;
        double best = a.sd[slot];
        int bj = a.sj[slot];
        for (int s = 1; s < S; ++s) {
            const double d = a.sd[slot + s];
            const int j = a.sj[slot + s];
            if (d < best || (d == best && j < bj)) { best = d; bj = j; }
        }
        rescan_out(a, dir, p, list[e], best, bj, nn);
    }
}


// ---------------------------------------------------------------------------
// Mutual correspondences without the column screen (feature_corres_v5).
//
// corres_build reads nn21 only at j = nn12[i], and nn12 hits ~half of the
// targets, so the column direction is screened only for those: pass 1 screens
// the rows (F against every G column, a top-2 per row with the column-tile
// index packed into the value: 3 VALU per distance instead of dual7's ~6.6),
// the uncertified rows are rescanned exactly, then pass 2 screens the rows
// J = {nn12[i]} of G against every F column keeping top-2 VALUES only (2 VALU
// per distance, no index), and the candidate i of column j = nn12[i] is decided
// from values:
//   pass 2 certifies column j when its top-2 gap exceeds 2 (e2 + e1_i), e2 the
//   screen's bound for column j, e1_i that of row i's own value v_i (its pass-1
//   b1 with the code bits' perturbation, or 0 when the row was rescanned); then
//   the exact column argmin w has the screen minimum w1, D_w <= w1 + e2 and
//   every other row is >= w2 - e2, so i is mutual iff v_i <= w1 + e2 + e1_i.
//   A column that cannot be decided is rescanned exactly (featnn_rescan3,
//   direction 1) and its candidates compared with that argmin.
// The result is the same set corres_build forms from the exact nn12 / nn21.
// ---------------------------------------------------------------------------
struct RowArgs5 {
    const f16x8 *Ap;            // row operand (register-resident): [P][ntr][NM][64]
    const f16x8 *Bp;            // column operand (LDS-streamed): [P][ntc][NM][64]
    const float *rnr;           // scaled row norms, [P][ntr * 32] by original row index
    const unsigned *cmax;       // per pair max scaled column norm (f32 bits)
    const int32_t *n_rows, *n_cols;
    const int *rlist, *rcount;  // pass 2: rows rlist[p][0 .. rcount[p]) (original indices)
    int P, Rmax, Cmax, ntr, ntc, nrb, D, ctbits;
    int32_t *nn;                // pass 1: argmin (screened), value, its error, uncertified rows
    double *v;
    float *e;
    int *list, *count;
    float4 *wq;                 // pass 2: (top-2 values, the screen's error bound, -) by original row index
    // pass 2: the gathered rows built in registers from the f32 cloud (one
    // 128-byte row per lane instead of ten 16-byte pieces in ten lines of the
    // packed image), with the scale the packs used and the image's role
    const float *Xr;
    const unsigned *sc;
    int role, cs;
    const unsigned *cemax;      // featnn_row8<.., kOne>: per pair max |y - f16(y)| of the column image
    int32_t *nns;               // pass 1: a copy of the screened argmin for featmut_jbuild (nullable)
    int fbdiag;                 // 1 / 2: count the listed rows in g_featnn_fallback_rows[0 / 1]
    int rbmajor;                // featnn_row8: blocks ordered row block first (short lists, below)
    const float *rre;           // the rows' |x - f16(x)| from the pack, [P][ntr * 32]
    // featnn_row9's buckets (rows by winning step): [P][steps] counts and
    // [P][steps][bcap] entries (row, B1, B2, lane half of the winning group)
    int *bcnt, bcap;
    uint4 *blist;
    uint4 *rec;                 // featnn_regroup9 -> featnn_finish9, by row: (column, B1, B2, skip)
    int *llist, *lcount;        // featnn_finish9: where its failing rows go (nullable)
    // featnn_row8 list mode over column slices (csl > 1: short lists at small
    // batches): slice sl's partial (B1, B2, column) per listed row position k,
    // [P][csl][Rmax], merged by featnn_slicemerge
    int csl;
    uint4 *part;
    // featnn_row9: the column cloud's and the row cloud's per-row terms
    // f32(|.|^2 + B) ([P][ntc * 32], [P][ntr * 32]) and B
    const float *cct, *rct;
    const float *cbias;  // [P] B
};

// rows (pass 1) and J columns (pass 2) the 1-term screens left to the 3-term
// ones since the last reset (diagnostic, pcr_featnn_fallback_rows)
__device__ unsigned long long g_featnn_fallback_rows[2];

// featnn_row9's column terms (after the packs and their repairs): the packs
// stored f32(|x s|^2) per row, -1 on padding rows; here ct = f32(that + B) with
// B the pair's smallest power of two above both clouds' max |x s|^2 (from the
// packs' max norms, a rounding's margin added), so every screened value
// ct_j - 2 x.y_j >= B - |x|^2 > 0 (unsigned order = float order) and ct lies in
// [B, 2B] (2B - ct exact).  Padding rows: 16 B, above every real value (< 4 B).
// A pair with a non-finite norm takes B = 2^60 (its rows certify nothing).
__global__ __launch_bounds__(256) void feat_colterms(float *fct, float *gct, int ntn, int ntm,
                                                     const unsigned *fmax, const unsigned *gmax, float *cbias) {
    const int p = blockIdx.y, role = blockIdx.z;
    const float mf = __builtin_fmaxf(__uint_as_float(fmax[p]), __uint_as_float(gmax[p]));
    double B = 0x1p60;
    if (mf < 0x1p50f) {
        const double m2 = (double)mf * (double)mf * (1.0 + 0x1p-18) + 1.0;
        const int e = (int)((__double_as_longlong(m2) >> 52) & 0x7ff) - 1023;  // m2 in [2^e, 2^(e+1))
        B = __builtin_ldexp(1.0, e + 1);
    }
    if (blockIdx.x == 0 && role == 0 && threadIdx.x == 0) cbias[p] = (float)B;
    const int nt = role ? ntm : ntn;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nt * 32) return;
    float *ct = (role ? gct : fct) + (size_t)p * nt * 32 + i;
    const float x = *ct;
    *ct = x < 0.0f ? (float)(16.0 * B) : (float)((double)x + B);
}

// One row's operand fragments exactly as feat_pack5 / feat_pack5r store them
// (same scale, same operations in the same order), for lane half h: x the
// row's f32 values (DV >= D, zero beyond D).
template <int S>
__device__ __forceinline__ void row_frags(const float *x, int D, int h, int role, int cs,
                                          f16x8 (&out)[2 * S + 1]) {
    constexpr int DV = 16 * S;
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < DV; ++k)
        if (k < D) {
            const double v = (double)x[k];
            acc = acc + v * v;
        }
    _Float16 np[3];
    double wv = acc * __builtin_ldexp(1.0, -cs);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        np[q] = (_Float16)(float)wv;
        wv = wv - (double)np[q];
    }
    const _Float16 cval = (_Float16)__builtin_ldexpf(1.0f, cs);
    _Float16 s0[DV], s1[DV];
#pragma unroll
    for (int k = 0; k < DV; ++k) {
        const _Float16 hi = (_Float16)x[k];
        const _Float16 lo = (_Float16)(x[k] - (float)hi);
        s0[k] = role == 0 ? (_Float16)(-2.0f * (float)hi) : hi;
        s1[k] = role == 0 ? (_Float16)(-2.0f * (float)lo) : lo;
    }
#pragma unroll
    for (int c = 0; c < 2 * S + 1; ++c) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            _Float16 v0 = (_Float16)0.0f, v1 = (_Float16)0.0f;  // lane halves 0 / 1
            if (c < 2 * S) {
                const int k0 = 16 * (c % S) + j;
                const _Float16 *sg = c < S ? s0 : s1;
                v0 = k0 < D ? sg[k0] : (_Float16)0.0f;
                v1 = k0 + 8 < D ? sg[k0 + 8] : (_Float16)0.0f;
            } else {
                if (j < 3) v0 = role == 0 ? np[j] : cval;
                else if (j < 6) v0 = role == 0 ? cval : np[j - 3];
                else if (j == 6 && role == 1) v0 = (_Float16)32768.0f;  // featnn_row8's biases
                else if (j == 7 && role == 0) v0 = (_Float16)32768.0f;
            }
            out[c][j] = h ? v1 : v0;
        }
    }
}

// RT row tiles per wave share every B fragment read (two MFMAs per ds_read):
// a workgroup covers 8 * RT * 32 rows per pass over the pair's column stream,
// which halves the L2 -> LDS traffic at RT = 2 (at RT = 1 the stream of the
// packed columns ran near the chip's LDS-DMA rate: waves parked ~35 %).
//
// Pass 1's index: the column-tile number packed into the low ctbits mantissa
// bits of every value (one v_and_or) before the top-2 (featnn_row8 does the
// same on two column tiles at a time for S <= 2).
template <int S, int G, bool kIdx, int RT>
__global__ __launch_bounds__(512) void featnn_row7(RowArgs5 a) {
    constexpr int W = 8;              // waves per workgroup, RT 32-row tiles each
    constexpr int NX = 3 * S + 1, NM = 2 * S + 1;  // executed / stored k-chunks
    constexpr int kB = G * NM * 64;   // f16x8 per B buffer
    __shared__ __attribute__((aligned(16))) f16x8 Bs[2 * kB];
    const int b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const int p = (slot / a.nrb) * 8 + xcd, rb = slot - (slot / a.nrb) * a.nrb;
    if (p >= a.P) return;  // whole block
    const int nr = a.rlist ? a.rcount[p] : count_of(a.n_rows, p, a.Rmax);
    if (rb * W * RT * 32 >= nr) return;  // whole block: no rows here
    const int wid = threadIdx.x >> 6, l = threadIdx.x & 63, h = l >> 5;
    const int m = count_of(a.n_cols, p, a.Cmax);
    const int qt0 = (rb * W + wid) * RT;  // this wave's first row tile
    const int ntc = (m + 31) >> 5;
    const int ngroups = (ntc + G - 1) / G;
    const unsigned ctmask = (1u << a.ctbits) - 1u;
    unsigned keep_r = ~ctmask;
    asm("" : "+v"(keep_r));
    f16x8 A[RT][NM];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
        const int qt = qt0 + t;
        if (a.rlist) {  // gathered rows: lane l holds row slot qt*32 + (l & 31), half h
            const int k = qt * 32 + (l & 31);
            if (k < nr && a.Xr) {
                const int j = a.rlist[(size_t)p * a.Rmax + k];
                const float *xr = a.Xr + ((size_t)p * a.Rmax + j) * a.D;
                const float sc = __uint_as_float(a.sc[p]);
                float x[16 * S];
                if (a.D == 16 * S && ((uintptr_t)xr & 15) == 0) {
#pragma unroll
                    for (int q = 0; q < 4 * S; ++q) {
                        const float4 v = reinterpret_cast<const float4 *>(xr)[q];
                        x[4 * q] = v.x * sc; x[4 * q + 1] = v.y * sc; x[4 * q + 2] = v.z * sc; x[4 * q + 3] = v.w * sc;
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 16 * S; ++q) x[q] = q < a.D ? xr[q] * sc : 0.0f;
                }
                row_frags<S>(x, a.D, h, a.role, a.cs, A[t]);
            } else if (k < nr) {
                const int j = a.rlist[(size_t)p * a.Rmax + k];
                const f16x8 *qp = a.Ap + ((size_t)p * a.ntr + (j >> 5)) * NM * 64 + (j & 31) + 32 * h;
#pragma unroll
                for (int c = 0; c < NM; ++c) A[t][c] = qp[(size_t)c * 64];
            } else {
#pragma unroll
                for (int c = 0; c < NM; ++c)
#pragma unroll
                    for (int q = 0; q < 8; ++q) A[t][c][q] = (_Float16)0.0f;
            }
        } else {  // padded row tiles (qt < ntr) hold sentinel rows
            const f16x8 *qp = a.Ap + ((size_t)p * a.ntr + qt) * NM * 64 + l;
#pragma unroll
            for (int c = 0; c < NM; ++c) A[t][c] = qp[(size_t)c * 64];
        }
    }
    float b1[RT][16], b2[RT][16];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) { b1[t][r] = __builtin_inff(); b2[t][r] = __builtin_inff(); }
    const f16x8 *bsrc = a.Bp + (size_t)p * a.ntc * NM * 64 + l;
    auto issue = [&](int grp, int bufi) {
        for (int c = wid; c < G * NM; c += W) {
            const f16x8 *src = bsrc + ((size_t)grp * G * NM + c) * 64;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)src,
                (__attribute__((address_space(3))) void *)(Bs + bufi * kB + c * 64), 16, 0, 0);
        }
    };
    // row top-2 of the tile's 16 values per lane, values only (2 VALU per
    // value; pass 1's group code is applied at the group's end, above).
    // No inline asm here: the compiler must see every instruction that touches
    // the accumulators (its MFMA hazard wait states are not placed around
    // inline asm; with asm v_min / v_med3 the first registers of some tiles
    // read stale values).  min(a, b) is written med3(a, b, -FLT_MAX): the min
    // builtin would add a NaN canonicalisation per operand.  A NaN value makes
    // the row's top-2 NaN (uncertified: the exact rescan decides it).
    auto epilogue = [&](const f32x16 (&acc)[RT], unsigned ct) {
        asm("" : "+s"(ct));
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float vr = acc[t][r];
                if constexpr (kIdx) vr = __uint_as_float((__float_as_uint(vr) & keep_r) | ct);
                b2[t][r] = __builtin_amdgcn_fmed3f(b1[t][r], b2[t][r], vr);
                b1[t][r] = __builtin_amdgcn_fmed3f(b1[t][r], vr, -3.40282347e+38f);
            }
    };
    // VALU per MFMA slot below: the epilogue spread evenly (denser or sparser
    // spreads measured slower in round 4)
    constexpr int kV = (kIdx ? 48 : 32) * RT / NX + 1;
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int grp = 0; grp < ngroups; ++grp) {
        const int buf = grp & 1;
        if (grp + 1 < ngroups) issue(grp + 1, buf ^ 1);
        const f16x8 *Bb = Bs + buf * kB + l;
        f16x8 Bf[2][NM];
        f32x16 acc[2][RT];
#pragma unroll
        for (int c = 0; c < NM; ++c) Bf[0][c] = Bb[c * 64];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int cur = g & 1;
#pragma unroll
            for (int t = 0; t < RT; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[cur][t][r] = 0.0f;
#pragma unroll
            for (int c = 0; c < NX; ++c)
#pragma unroll
                for (int t = 0; t < RT; ++t)
                    acc[cur][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[t][amap(c, S)], Bf[cur][bmap(c, S)],
                                                                         acc[cur][t], 0, 0, 0);
            if (g + 1 < G) {
#pragma unroll
                for (int c = 0; c < NM; ++c) Bf[cur ^ 1][c] = Bb[((g + 1) * NM + c) * 64];
            }
            if (g > 0) epilogue(acc[cur ^ 1], (unsigned)(grp * G + g - 1));
#pragma unroll
            for (int c = 0; c < NX; ++c) {
                __builtin_amdgcn_sched_group_barrier(0x008, RT, 0);
                if (g + 1 < G && c < NM) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                if (g > 0) __builtin_amdgcn_sched_group_barrier(0x002, kV, 0);
            }
            // one scheduling region per tile: the next tile's fragments stay
            // prefetches (without it the scheduler sank them next to their
            // MFMAs: an LDS round trip in front of every MFMA)
            __builtin_amdgcn_sched_barrier(0);
        }
        epilogue(acc[(G - 1) & 1], (unsigned)(grp * G + G - 1));
        // the next group's DMA has landed for every wave, and every wave is done
        // reading this buffer before the group after next overwrites it
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    const int lr = l & 31;
#pragma unroll
    for (int t = 0; t < RT; ++t) {
        const int qt = qt0 + t;
        if (qt * 32 >= nr) break;
        if constexpr (kIdx) {
            int i1[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) i1[r] = (int)(__float_as_uint(b1[t][r]) & ctmask) * 32 + lr;
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float ob1 = __shfl_xor(b1[t][r], o, 64);
                    const float ob2 = __shfl_xor(b2[t][r], o, 64);
                    const int oi1 = __shfl_xor(i1[r], o, 64);
                    top2_merge(b1[t][r], i1[r], b2[t][r], ob1, oi1, ob2);
                }
            }
            float mb1 = 0.f, mb2 = 0.f;
            int mi1 = 0;
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (lr == r) { mb1 = b1[t][r]; mb2 = b2[t][r]; mi1 = i1[r]; }
            const int rin = (lr & 3) + 8 * (lr >> 2) + 4 * h;  // this lane's row of the tile
            const int row = qt * 32 + rin;
            const bool own = lr < 16 && row < nr;
            const size_t o = (size_t)p * a.Rmax + row;
            int want = -1;  // certified rows: the winner's column
            if (own && m == 0) {
                a.nn[o] = 0;
                a.v[o] = __builtin_inf();
                a.e[o] = 0.0f;
            } else if (own) {
                const double Gm = (double)__uint_as_float(a.cmax[p]);
                const double qn = (double)a.rnr[(size_t)p * a.ntr * 32 + row];
                const double bnd = bound5(qn, Gm, 16 * NX, a.D);
                const double pk = __builtin_ldexp(1.0, a.ctbits - 23);
                a.v[o] = (double)mb1;
                a.e[o] = (float)((0.5 * bnd + pk * __builtin_fabs((double)mb1)) * (1.0 + 1e-6));
                // uncertified rows too: the screened argmin, which the exact
                // rescan overwrites (featmut_jbuild may read either)
                want = mi1;
                if (!((double)mb2 - (double)mb1 > bnd + pk * (__builtin_fabs((double)mb1) + __builtin_fabs((double)mb2))))
                    a.list[(size_t)p * a.Rmax + atomicAdd(a.count + p, 1)] = row;
            }
            if (own && want >= 0) a.nn[o] = want;
        } else {
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float ob1 = __shfl_xor(b1[t][r], o, 64);
                    const float ob2 = __shfl_xor(b2[t][r], o, 64);
                    // second of {b1, b2} u {ob1, ob2} = med3(b1, ob1, min(b2, ob2))
                    // for sorted pairs; NaN stays NaN (uncertified)
                    const float m2 = __builtin_amdgcn_fmed3f(b2[t][r], ob2, -3.40282347e+38f);
                    b2[t][r] = __builtin_amdgcn_fmed3f(b1[t][r], ob1, m2);
                    b1[t][r] = __builtin_amdgcn_fmed3f(b1[t][r], ob1, -3.40282347e+38f);
                }
            }
            float mb1 = 0.f, mb2 = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (lr == r) { mb1 = b1[t][r]; mb2 = b2[t][r]; }
            const int k = qt * 32 + (lr & 3) + 8 * (lr >> 2) + 4 * h;
            if (lr >= 16 || k >= nr) continue;
            const int j = a.rlist[(size_t)p * a.Rmax + k];
            // the row's bound beside its values: featmut_resolve gathers one
            // 16-byte record per candidate (rounded up: a bound stays a bound)
            const double e2 = 0.5 * bound5((double)a.rnr[(size_t)p * a.ntr * 32 + j],
                                           (double)__uint_as_float(a.cmax[p]), 16 * NX, a.D);
            a.wq[(size_t)p * a.Rmax + j] = make_float4(m == 0 ? __builtin_inff() : mb1,
                                                       m == 0 ? __builtin_inff() : mb2,
                                                       (float)(e2 * (1.0 + 1e-6)), 0.0f);
        }
    }
}

// Pass 1, round 5 (S <= 2): the row top-2 of TWO column tiles at a time.
//
// featnn_row7 spends 3 VALU per distance (code, med3, min) against 7 MFMAs per
// 32x32 tile: 262 issue cycles per tile beside 224 of MFMA pipe, so the screen
// was bound by SIMD issue.  Here a wave holds RT = 2 row tiles and walks the
// LDS group in steps of two column tiles (c0, c1): each slot (row, column lane)
// takes its pair of values (x, y) at once --
//     t = med3(b1, x, y);  b2 = min(b2, t);  b1 = min3(b1, x, y)
// (the second smallest of {b1, b2, x, y} is min(b2, med3(b1, x, y)) for
// b1 <= b2) -- 2.5 VALU per distance with the tile code, 40 per tile: 226
// issue cycles, i.e. the kernel becomes MFMA-pipe bound.  The top-2 runs on
// the f32 BIT PATTERNS as unsigned integers (v_med3_u32 / v_min3_u32 /
// v_min_u32: no NaN canonicalisation, no inline asm next to the accumulators):
// that order is the float order for non-negative values, so every value is
// shifted up by a bias B = 2^15 -- the row operand's norm chunk carries 1.0 at
// k = 6 (patched in registers) against 2^15 in the column image's (the other
// screens multiply it by 0) -- larger than any screen error (bound5 at the
// split's range |x| < 2^T, D <= 32: < 29,000 in scaled units), so no screened
// value is negative; NaN patterns sort above +inf, so NaN distances never win (as
// in the oracle's strict <), and a pair with a non-finite value is uncertified
// by its bound anyway.  The certification charges the bias's rounding.
// Schedule per step, two phases of 14 MFMAs (accumulators acc[t][c]: 64 VGPRs):
//   A: row tile 0's MFMAs | row tile 1's epilogue of the previous step
//   B: row tile 1's MFMAs | row tile 0's epilogue of this step
// so each phase is 14 MFMAs beside 80 VALU (5.7 per 32-cycle MFMA slot) and no
// accumulator is double-buffered.  The step's B fragments (10 ds_read_b128)
// open phase A, their latency covered by the epilogue's first VALU.
// ---------------------------------------------------------------------------
constexpr int kRow8Head = 24;  // epilogue VALU in front of phase A's first MFMA (the B reads' latency)
constexpr int kRow8G = 8;      // column tiles per LDS group (16: the whole LDS, measured no faster)
#ifndef PCR_ROW9_G
#define PCR_ROW9_G 16  // 8: pass 1 1.12 vs 1.09 ms, pass 2 0.76 vs 0.74 (C4, featnn_bench)
#endif
#ifndef PCR_ROW9_G1
#define PCR_ROW9_G1 PCR_ROW9_G
#endif
constexpr int kRow9G = PCR_ROW9_G;     // featnn_row9's: pass 2 (and the padding)
constexpr int kRow9G1 = PCR_ROW9_G1;   // pass 1 (<= kRow9G)
// B: pass 1 1.0 (row k = 6) x 2^15 (G's column image, k = 6); pass 2 (featnn_row8
// <.., false>, the J rows of G against F's image) 1.0 (row k = 7) x 2^15 (F's
// image, k = 7).  dual7 pairs F's image with G's: 0 x 2^15 at both slots.
constexpr double kRowBias = 32768.0;

__device__ __forceinline__ unsigned umin2(unsigned a, unsigned b) { return a < b ? a : b; }
__device__ __forceinline__ unsigned umax2(unsigned a, unsigned b) { return a > b ? a : b; }

// The 1-term screen (round 6, kOne): the row operand is -2 f16(x) and the column
// operand f16(y) -- one k-segment instead of the split's three (hi.hi', hi.lo',
// lo.hi'), so S + 1 MFMAs per 32 x 32 tile instead of 3 S + 1, and the column
// stream carries only the [hi | norms] chunks of the stored image.  Its error
// is larger: with e_x = x - f16(x) (exact in f32),
//   |x.y - f16(x).f16(y)| = |e_x.y + f16(x).e_y| <= |e_x| |y| + (|x| + |e_x|) |e_y|
// by Cauchy-Schwarz; the row's |e_x| is computed here from the row itself, the
// columns' max |e_y| by the pack (emax), and both carry 2^-14 sqrt(D) for f16
// subnormals the MFMA may flush (bound1).  ~4 % of the rows (C4) do not
// certify under it: they are listed for the 3-term screen of the same rows
// (featnn_row8<.., false> over the list, the rows it cannot certify going on to
// the exact rescan as before).  The bias is 2^21 (the row patch 64 against the
// image's 2^15): the 1-term error reaches ~2^20 at the split's range.
constexpr double kRowBias1 = 2097152.0;  // 2^21
#ifdef PCR_NOSCHED
#define SGB(...) ((void)0)
#else
#define SGB(...) __builtin_amdgcn_sched_group_barrier(__VA_ARGS__)
#endif
#ifndef PCR_VA
#define PCR_VA ((80 - kRow8Head + 2 * NX - 1) / (2 * NX))
#endif
#ifndef PCR_VB
#define PCR_VB ((80 - 16 + 2 * NX - 3) / (2 * NX - 2))
#endif

// certification threshold of the 1-term screen (scaled units), 2 x the error
// bound; ex, E: the row's and the columns' max |x - f16(x)|, subnormal term added
__device__ __forceinline__ double bound1(double q, double ex, double G, double E, int Kt) {
    const double u = 5.9604644775390625e-08;  // 2^-24
    const double qg = q + G;
    const double err = 2.0 * (Kt + 2) * u * qg * qg + 2.0 * (ex * G + (q + ex) * E) +
                       1.1641532182693481e-10 * (q * q + G * G) + 4.0;
    return 2.0 * err;
}
__device__ __forceinline__ double sub_term(int D) { return 6.103515625e-05 * __builtin_sqrt((double)D); }  // 2^-14 sqrt(D)

// The certification and outputs of one screened row (featnn_row8's tail, and
// featnn_finish9's): B1 / B2 the row's smallest and second smallest biased
// value patterns, mi1 the column of B1, rexv the row's |x - f16(x)| (1-term),
// pk the relative truncation of the values' low bits (the column code of
// featnn_row8 pass 1; 0 when the values carry no code).  Returns whether the
// row goes to a.list (the caller appends it)
template <bool kIdx, bool kOne, int NX, bool kCT = false>
__device__ __forceinline__ bool row_tail(const RowArgs5 &a, int p, int row, int m, unsigned B1, unsigned B2,
                                         int mi1, float rexv, double pk, float ctr = 0.0f) {
    constexpr double kBias = kOne ? kRowBias1 : kRowBias;
    constexpr double u = 5.9604644775390625e-08;  // 2^-24
    const double sub = kOne ? sub_term(a.D) : 0.0;
    const float mb1 = __uint_as_float(B1), mb2 = __uint_as_float(B2);
    // this row's screen error bound (2x, as bound5): the split's or the 1-term's,
    // plus the bias's share of the accumulation error, 2 (Kt + 2) u B, doubled.
    // kCT (featnn_row9): the values are ct_j - 2 f16(x).f16(y_j) with the column
    // term ct_j = f32(|y_j|^2 + B) as the MFMA's accumulator input: the f32
    // accumulation over |C| + |products| <= B + G^2 + 2 (q + ex)(G + E), the f16
    // dot error as bound1, and ct_j's own roundings (f32 |y|^2, then + B),
    // u (2 B + G^2).  The row's |x|^2 is not in the values: its own ct (ctr,
    // rounding u (2 B + q^2)) turns a value into a distance, value - (2 B - ctr)
    // (exact: Sterbenz).  B: the pair's (feat_colterms).
    const double qn = (double)a.rnr[(size_t)p * a.ntr * 32 + row];
    const double Gm = (double)__uint_as_float(a.cmax[p]);
    double bnd, bias, ebias = 0.0;
    if constexpr (kCT) {
        const double ex = (double)rexv + sub, E = (double)__uint_as_float(a.cemax[p]) + sub;
        const double B = (double)a.cbias[p];
        const double err = 2.0 * (16 * NX + 2) * u * ((B + Gm * Gm) + 2.0 * (qn + ex) * (Gm + E)) +
                           2.0 * (ex * Gm + (qn + ex) * E) + u * (2.0 * B + Gm * Gm) * (1.0 + 0x1p-20) + 4.0;
        bnd = 2.0 * err;
        bias = 2.0 * B - (double)ctr;
        ebias = u * (2.0 * B + qn * qn) * (1.0 + 0x1p-20);
    } else {
        bnd = (kOne ? bound1(qn, (double)rexv + sub, Gm, (double)__uint_as_float(a.cemax[p]) + sub, 16 * NX)
                    : bound5(qn, Gm, 16 * NX, a.D)) +
              4.0 * (16 * NX + 2) * u * kBias;
        bias = kBias;
    }
    if constexpr (!kIdx) {  // pass 2: the row's biased top-2 values, its bound and the bias, by original row
        const double e2 = 0.5 * bnd + ebias;
        a.wq[(size_t)p * a.Rmax + row] = make_float4(m == 0 ? __builtin_inff() : mb1, m == 0 ? __builtin_inff() : mb2,
                                                     (float)(e2 * (1.0 + 1e-6)), (float)bias);
        // 1-term: a column whose gap the resolve could not use goes to the
        // 3-term screen (a.list; the 3-term pass lists nothing)
        return kOne && m != 0 && a.list &&
               !((double)mb2 - (double)mb1 > 2.0 * e2 * (1.0 + 1e-6) + 1e-6 * (double)mb1);
    }
    const size_t o = (size_t)p * a.Rmax + row;
    if (m == 0) {
        a.nn[o] = 0;
        if (a.nns) a.nns[o] = 0;
        a.v[o] = __builtin_inf();
        a.e[o] = 0.0f;
        return false;
    }
    a.v[o] = (double)mb1 - bias;  // exact (f32 values of a few binades: multiples of mb1's ulp)
    a.e[o] = (float)((0.5 * bnd + ebias + pk * __builtin_fabs((double)mb1)) * (1.0 + 1e-6));
    // the certificate: the top-2 gap against twice the per-value bound, or
    // (1-term) against a bound on the DIFFERENCE of two values' errors.  Only
    // columns j screened within 2 err of the winner j1 can overtake it, and
    // for those the dot-product errors differ by at most
    //   2 |e_x| |y_j - y_j1| + 2 |f16(x)| (|e_yj| + |e_yj1|),
    // |y_j - y_j1| <= sqrt(D_j) + sqrt(D_j1) <= sqrt(b1 + 3 err) + sqrt(b1 + err)
    // (b1 the winner's screened value): the row's nearest columns are much
    // closer together than 2 max|y|.  ~20 % fewer rows to the 3-term screen.
    double thr = bnd;
    if constexpr (kOne) {
        const double ex = (double)rexv + sub, E = (double)__uint_as_float(a.cemax[p]) + sub;
        const double dot = 2.0 * (ex * Gm + (qn + ex) * E);       // bound1's dot-product share
        const double rest = 0.5 * bnd - dot;                        // accumulation, norms, bias
        const double er = 0.5 * bnd + ebias + pk * __builtin_fabs((double)mb2);
        const double b1v = __builtin_fmax((double)mb1 - bias, 0.0);
        const double win = 2.0 * rest + 2.0 * ex * (__builtin_sqrt(b1v + 3.0 * er) + __builtin_sqrt(b1v + er)) +
                           4.0 * (qn + ex) * E;
        thr = __builtin_fmin(bnd, win * (1.0 + 1e-9));
    }
    // uncertified rows too: the screened argmin, which the 3-term pass or
    // the exact rescan overwrites; J is built from the copy in nns, which
    // nothing overwrites while featmut_jbuild reads it
    a.nn[o] = mi1;
    if (a.nns) a.nns[o] = mi1;
    return !((double)mb2 - (double)mb1 > thr + pk * (__builtin_fabs((double)mb1) + __builtin_fabs((double)mb2)));
}

// featnn_row9's early test: a row whose gap between its smallest value and
// the second smallest GROUP minimum -- an upper bound on its true second
// value -- already fails the certificate (row_tail's kCT one, pk = 0) fails it
// whatever the winning group's own second: it goes to the 3-term screen right
// after the sweep (beside the regroup) instead of through the regroup.
template <bool kIdx, int NX>
__device__ __forceinline__ bool one_term_fails(const RowArgs5 &a, int p, int row, unsigned B1, unsigned B2g,
                                               float rexv, float ctr) {
    constexpr double u = 5.9604644775390625e-08;  // 2^-24
    const double sub = sub_term(a.D);
    const double mb1 = (double)__uint_as_float(B1), mb2 = (double)__uint_as_float(B2g);
    const double qn = (double)a.rnr[(size_t)p * a.ntr * 32 + row];
    const double Gm = (double)__uint_as_float(a.cmax[p]);
    const double ex = (double)rexv + sub, E = (double)__uint_as_float(a.cemax[p]) + sub;
    const double B = (double)a.cbias[p];
    const double bnd = 2.0 * (2.0 * (16 * NX + 2) * u * ((B + Gm * Gm) + 2.0 * (qn + ex) * (Gm + E)) +
                              2.0 * (ex * Gm + (qn + ex) * E) + u * (2.0 * B + Gm * Gm) * (1.0 + 0x1p-20) + 4.0);
    const double ebias = u * (2.0 * B + qn * qn) * (1.0 + 0x1p-20);
    if constexpr (!kIdx) return !(mb2 - mb1 > (bnd + 2.0 * ebias) * (1.0 + 1e-6) + 1e-6 * mb1);
    const double dot = 2.0 * (ex * Gm + (qn + ex) * E);
    const double rest = 0.5 * bnd - dot;
    const double er = 0.5 * bnd + ebias;
    const double b1v = __builtin_fmax(mb1 - (2.0 * B - (double)ctr), 0.0);
    const double win = 2.0 * rest + 2.0 * ex * (__builtin_sqrt(b1v + 3.0 * er) + __builtin_sqrt(b1v + er)) +
                       4.0 * (qn + ex) * E;
    return !(mb2 - mb1 > __builtin_fmin(bnd, win * (1.0 + 1e-9)));
}

template <int S, int G, bool kIdx, bool kOne>
__global__ __launch_bounds__(512) void featnn_row8(RowArgs5 a) {
    constexpr int W = 8, RT = 2;                   // waves per workgroup, row tiles per wave
    constexpr int NM = 2 * S + 1;                  // stored k-chunks of the packed images
    constexpr int NX = kOne ? S + 1 : 3 * S + 1;   // executed k-chunks (MFMAs per tile)
    constexpr int NB = kOne ? S + 1 : NM;          // chunks per column tile in LDS / per row tile in registers
    constexpr int kB = G * NB * 64;                // f16x8 per B buffer
    constexpr double kBias = kOne ? kRowBias1 : kRowBias;
    static_assert(G % 2 == 0 && S <= 2, "column tiles in pairs; two row tiles fit up to S = 2");
    constexpr int kMerge = W * 64 * 17 * 8 / 16;  // the row merge's (b1, b2) slots, in f16x8
    __shared__ __attribute__((aligned(16))) f16x8 Bs[2 * kB > kMerge ? 2 * kB : kMerge];
    const int b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    // pair-major (a pair's row blocks back to back on its XCD, sharing its
    // column image in that L2) or, for the short lists the 3-term screens
    // take from the 1-term ones (one block per pair, the rest exit at once),
    // row-block-major: pair-major placed the working blocks 16 apart in an
    // XCD's dispatch order, and they piled onto a few of its CUs (3x slower)
    const int ppx = (a.P + 7) >> 3;
    // row-block-major blocks also split the columns into a.csl slices (list
    // mode at small batches: a pair's short list is one block per slice)
    const int rbs = a.rbmajor ? slot / ppx : 0, csl = a.rbmajor ? a.csl : 1, sl = rbs % csl;
    const int p = a.rbmajor ? (slot % ppx) * 8 + xcd : (slot / a.nrb) * 8 + xcd;
    const int rb = a.rbmajor ? rbs / csl : slot - (slot / a.nrb) * a.nrb;
    if (p >= a.P) return;  // whole block
    // the rows: in order (pass 1) or the listed ones rlist[p][0 .. rcount[p])
    // (pass 2: J; the 3-term passes behind a 1-term one: the rows it left)
    const int *rl = a.rlist ? a.rlist + (size_t)p * a.Rmax : nullptr;
    const int nr = rl ? a.rcount[p] : count_of(a.n_rows, p, a.Rmax);
    if (a.fbdiag && rb == 0 && sl == 0 && threadIdx.x == 0 && nr > 0)
        atomicAdd(&g_featnn_fallback_rows[a.fbdiag - 1], (unsigned long long)nr);
    if (rb * W * RT * 32 >= nr) return;  // whole block: no rows here
    const int wid = threadIdx.x >> 6, l = threadIdx.x & 63, h = l >> 5;
    const int m = count_of(a.n_cols, p, a.Cmax);
    const int qt0 = (rb * W + wid) * RT;  // this wave's first row tile
    const int ntc = (m + 31) >> 5;
    const int ngall = (ntc + G - 1) / G;
    // this slice's column groups [g0, ngroups)
    const int g0 = (int)((long long)ngall * sl / csl), ngroups = (int)((long long)ngall * (sl + 1) / csl);
    const unsigned ctmask = (1u << a.ctbits) - 1u;
    unsigned keep = ~ctmask;
    asm("" : "+v"(keep));  // a VGPR operand: one v_and_or_b32 per code with the SGPR tile number
    // the row operand built from the f32 rows (one 128-byte row per lane, the
    // operands exactly as the pack stores them: the packed row image is not read)
    f16x8 A[RT][NB];
    float rex[RT];  // kOne: the row's |x - f16(x)| (rounded up)
    {
        const float sc = __uint_as_float(a.sc[p]);
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            const int k = (qt0 + t) * 32 + (l & 31);
            const int row = rl ? (k < nr ? rl[k] : 0) : k;
            float x[16 * S];
            const float *xr = a.Xr + ((size_t)p * a.Rmax + row) * a.D;
            if (k < nr && a.D == 16 * S && ((uintptr_t)xr & 15) == 0) {
#pragma unroll
                for (int q = 0; q < 4 * S; ++q) {
                    const float4 v = reinterpret_cast<const float4 *>(xr)[q];
                    x[4 * q] = v.x * sc; x[4 * q + 1] = v.y * sc; x[4 * q + 2] = v.z * sc; x[4 * q + 3] = v.w * sc;
                }
            } else if (k < nr) {
#pragma unroll
                for (int q = 0; q < 16 * S; ++q) x[q] = q < a.D ? xr[q] * sc : 0.0f;
            } else {
#pragma unroll
                for (int q = 0; q < 16 * S; ++q) x[q] = 0.0f;  // rows past the count write nothing
            }
            f16x8 fr[NM];
            row_frags<S>(x, a.D, h, a.role, a.cs, fr);
#pragma unroll
            for (int c = 0; c < NB; ++c) A[t][c] = fr[kOne ? (c < S ? c : 2 * S) : c];
            // the bias (see above): 1.0 (3-term) or 64 (1-term) opposite the image's 2^15
            const _Float16 bv = (_Float16)(kOne ? 64.0f : 1.0f);
            if (h == 0) {
                if (a.role == 0) A[t][NB - 1][6] = bv;
                else A[t][NB - 1][7] = bv;
            }
            if constexpr (kOne) {
                double ea = 0.0;
#pragma unroll
                for (int q = 0; q < 16 * S; ++q) {
                    const double e = (double)(x[q] - (float)(_Float16)x[q]);
                    ea = ea + e * e;
                }
                rex[t] = split_err_norm(ea);
                asm volatile("" : "+v"(rex[t]));  // here, not sunk to its use after the loop (the rows stay live)
            } else {
                rex[t] = 0.0f;
            }
        }
    }
    unsigned b1[RT][16], b2[RT][16];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) { b1[t][r] = 0x7f800000u; b2[t][r] = 0x7f800000u; }
    const f16x8 *bsrc = a.Bp + (size_t)p * a.ntc * NM * 64 + l;
    auto issue = [&](int grp, int bufi) {
        for (int c = wid; c < G * NB; c += W) {
            const int g = c / NB, cc = c - g * NB;
            const int sch = kOne ? (cc < S ? cc : 2 * S) : cc;  // the stored chunk
            const f16x8 *src = bsrc + ((size_t)(grp * G + g) * NM + sch) * 64;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)src,
                (__attribute__((address_space(3))) void *)(Bs + bufi * kB + c * 64), 16, 0, 0);
        }
    };
    // row tile t's slots take the values of column tiles ct (x) and ct + 1 (y)
    auto epilogue = [&](const f32x16 (&x)[2], int t, unsigned ct) {
        asm("" : "+s"(ct));
        const unsigned ct1 = ct + 1u;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            // pass 1: the tile numbers in the low bits; pass 2: values only
            const unsigned cx = kIdx ? (__float_as_uint(x[0][r]) & keep) | ct : __float_as_uint(x[0][r]);
            const unsigned cy = kIdx ? (__float_as_uint(x[1][r]) & keep) | ct1 : __float_as_uint(x[1][r]);
            // the median as v_med3_f32 (the same order on these non-negative
            // patterns; an integer median shares min(b1, cx) with the min3
            // below and costs a v_min more)
            const unsigned md = __float_as_uint(
                __builtin_amdgcn_fmed3f(__uint_as_float(b1[t][r]), __uint_as_float(cx), __uint_as_float(cy)));
            b2[t][r] = umin2(b2[t][r], md);
            b1[t][r] = umin2(b1[t][r], umin2(cx, cy));
            asm("" : "+v"(b2[t][r]));  // no b2 min chain across steps (it held 32 more VGPRs and spilled)
        }
    };
    // executed chunk c -> the register / LDS chunk holding its operands
    auto ach = [](int c) { return kOne ? c : amap(c, S); };
    auto bch = [](int c) { return kOne ? c : bmap(c, S); };
    f32x16 acc[RT][2];
    // the first phase A finds a harmless pending epilogue: +inf with code 0
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[1][c][r] = __builtin_inff();
    unsigned pend = 0u;
    const f32x16 zero = {};
    // VALU per phase (two tiles' epilogues): 80; spread over the phase's MFMAs
    constexpr int kVA = PCR_VA;
    constexpr int kVB = PCR_VB;
    if (g0 < ngroups) issue(g0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int grp = g0; grp < ngroups; ++grp) {
        const int buf = (grp - g0) & 1;
        if (grp + 1 < ngroups) issue(grp + 1, buf ^ 1);
        const f16x8 *Bb = Bs + buf * kB + l;
        // the step's B fragments, read in MFMA order (the first MFMAs wait for
        // the first reads only): the group's first step reads them at its
        // start, every later step at the end of the previous step's phase B
        f16x8 Bf[2][NB];
#pragma unroll
        for (int c = 0; c < NB; ++c)
#pragma unroll
            for (int u = 0; u < 2; ++u) Bf[u][c] = Bb[(u * NB + c) * 64];
#pragma unroll
        for (int st = 0; st < G / 2; ++st) {
            const unsigned ct = (unsigned)(grp * G + 2 * st);
            // phase A
#pragma unroll
            for (int c = 0; c < NX; ++c)
#pragma unroll
                for (int u = 0; u < 2; ++u)
                    acc[0][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[0][ach(c)], Bf[u][bch(c)],
                                                                       c == 0 ? zero : acc[0][u], 0, 0, 0);
            epilogue(acc[1], 1, pend);
            if (st == 0) SGB(0x100, 2 * NB, 0);
            SGB(0x002, kRow8Head, 0);
#pragma unroll
            for (int i = 0; i < 2 * NX; ++i) {
                SGB(0x008, 1, 0);
                SGB(0x002, kVA, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            // phase B
#pragma unroll
            for (int c = 0; c < NX; ++c)
#pragma unroll
                for (int u = 0; u < 2; ++u)
                    acc[1][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[1][ach(c)], Bf[u][bch(c)],
                                                                       c == 0 ? zero : acc[1][u], 0, 0, 0);
            epilogue(acc[0], 0, ct);
            if (st + 1 < G / 2) {  // the next step's fragments, behind this phase's last MFMA
#pragma unroll
                for (int c = 0; c < NB; ++c)
#pragma unroll
                    for (int u = 0; u < 2; ++u) Bf[u][c] = Bb[((2 * st + 2 + u) * NB + c) * 64];
            }
            SGB(0x008, 2, 0);
#pragma unroll
            for (int i = 0; i < 2 * NX - 2; ++i) {
                SGB(0x002, kVB, 0);
                SGB(0x008, 1, 0);
            }
            if (st + 1 < G / 2) SGB(0x100, 2 * NB, 0);
            SGB(0x002, 16, 0);
            __builtin_amdgcn_sched_barrier(0);
            pend = ct;
        }
        // the next group's DMA has landed for every wave, and every wave is done
        // reading this buffer before the group after next overwrites it
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    epilogue(acc[1], 1, pend);
    // Row merge through LDS (the B buffers are free): each lane stores its 16
    // slots (b1, b2), then lane L takes row L & 31 and half of its 32 column
    // lanes (16 entries in column order: on equal patterns -- same value, same
    // tile code -- the lower column lane stays), and the two halves combine by
    // one exchange.  Unsigned order = the screen's order (all values >= 0 or
    // +inf).  Stride 17: the stores and the row reads spread over the banks.
    uint2 *tl = reinterpret_cast<uint2 *>(Bs) + (size_t)wid * 64 * 17;
    const int R = l & 31, hR = (R >> 2) & 1, rR = (R & 3) + 4 * (R >> 3), j0 = 16 * h;
#pragma unroll
    for (int t = 0; t < RT; ++t) {  // every wave runs both (the barriers), rows past nr write nothing
        const int qt = qt0 + t;
        __syncthreads();  // (t = 0: every wave is past its last B read; t = 1: the row reads)
#pragma unroll
        for (int r = 0; r < 16; ++r) tl[l * 17 + r] = make_uint2(b1[t][r], b2[t][r]);
        __syncthreads();
        unsigned B1 = 0x7f800000u, B2 = 0x7f800000u;
        int jw = j0;
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            const uint2 e = tl[(hR * 32 + j0 + jj) * 17 + rR];
            B2 = umin2(umin2(B2, e.y), umax2(B1, e.x));
            const bool take = e.x < B1;
            B1 = take ? e.x : B1;
            jw = take ? j0 + jj : jw;
        }
        {   // lanes L < 32 hold column lanes 0..15: the partner's (16..31) win strictly below
            const unsigned o1 = (unsigned)__shfl_xor((int)B1, 32, 64), o2 = (unsigned)__shfl_xor((int)B2, 32, 64);
            const int oj = __shfl_xor(jw, 32, 64);
            B2 = umin2(umin2(B2, o2), umax2(B1, o1));
            const bool take = o1 < B1;
            B1 = take ? o1 : B1;
            jw = take ? oj : jw;
        }
        const int mi1 = (int)(B1 & ctmask) * 32 + jw;
        const int k = qt * 32 + R;
        if (h != 0 || k >= nr) continue;
        const int row = rl ? rl[k] : k;  // the original row index
        if (csl > 1) {  // this slice's partial, merged by featnn_slicemerge
            a.part[((size_t)p * csl + sl) * a.Rmax + k] = make_uint4(B1, B2, (unsigned)mi1, 0u);
            continue;
        }
        if (row_tail<kIdx, kOne, NX>(a, p, row, m, B1, B2, mi1, rex[t], __builtin_ldexp(1.0, a.ctbits - 23)))
            a.list[(size_t)p * a.Rmax + atomicAdd(a.count + p, 1)] = row;
    }
}

// featnn_row8's column slices (list mode, csl > 1) merged: per listed row the
// smallest B1 over the slices (the values carry the column tile code: no two
// are equal across slices), B2 the second smallest of the union, then the
// row's certification and outputs as the unsliced kernel's tail
template <int S, bool kIdx>
__global__ __launch_bounds__(256) void featnn_slicemerge(RowArgs5 a) {
    constexpr int NX = 3 * S + 1;
    const int p = blockIdx.y, k = blockIdx.x * 256 + threadIdx.x;
    const int *rl = a.rlist + (size_t)p * a.Rmax;
    if (k >= a.rcount[p]) return;
    unsigned B1 = 0x7f800000u, B2 = 0x7f800000u, mi = 0u;
    for (int s2 = 0; s2 < a.csl; ++s2) {
        const uint4 q = a.part[((size_t)p * a.csl + s2) * a.Rmax + k];
        B2 = umin2(umin2(B2, q.y), umax2(B1, q.x));
        mi = q.x < B1 ? q.z : mi;
        B1 = umin2(B1, q.x);
    }
    const int row = rl[k];
    if (row_tail<kIdx, false, NX>(a, p, row, count_of(a.n_cols, p, a.Cmax), B1, B2, (int)mi, 0.0f,
                                  __builtin_ldexp(1.0, a.ctbits - 23)))
        a.list[(size_t)p * a.Rmax + atomicAdd(a.count + p, 1)] = row;
}

// ---------------------------------------------------------------------------
// Round 6: the 1-term screens without a per-value index (featnn_row9, then
// featnn_regroup9).  featnn_row8 spends 2.5 VALU per screened value -- the
// column code OR-ed into the low bits (1) and the running top-2 (1.5) -- i.e.
// 40 VALU per 32 x 32 tile beside 3 MFMAs (96 pipe cycles): the 1-term pass
// is VALU-issue bound (~190 issue cycles per tile).  featnn_row9 swaps the
// MFMA's operands (the column fragments as A, the row's as B: the tile's
// transpose), so a lane holds ONE row and 16 columns of each column tile
// (register r: column 8 (r / 4) + 4 h + (r % 4), h the lane half).  A lane's
// 32 values of a step (two column tiles) form a group, and the sweep keeps
// per lane only
//   B1 -- the smallest value,
//   B2 -- the second smallest GROUP minimum,
//   I  -- the step of B1's group:
// 16 v_min3 + 5 VALU per step and row tile (10.5 per tile): the loop is
// MFMA-pipe bound.  The lane halves merge at the end (a row's other half is
// another set of groups).  What the sweep does not know -- the argmin's column
// and the second smallest value INSIDE the winning group -- featnn_regroup9
// recovers by re-running the identical MFMA chain (same operands, same order:
// bit-identical values) for the winning step only: a pair's rows bucketed by
// that step, one 32-row tile per bucket segment (~1 % of the sweep's MFMAs).
// Then second = min(B2, the group's own second) exactly, the values carry no
// code bits (pk = 0), and the certification and outputs are featnn_row8's
// (row_tail, its kCT bound).
// The norms are not an MFMA: the columns' terms ct_j = f32(|y_j|^2 + B)
// (feat_colterms, B the pair's) are the MFMA chain's accumulator input, so a
// tile costs S = 2 MFMAs instead of S + 1 and the values are ct_j - 2 x.y_j
// (the row's |x|^2 left out: a constant per row).  A lane's 16 C values per
// column tile come from the LDS copy of the group's terms or by DPP row
// broadcasts of one float per lane (see the sweep).
// ---------------------------------------------------------------------------

// The 1-term row operand of one row (lane half h) built from its f32 values:
// its -2 f16(x) chunks exactly as the packs store them (row_frags) -- one
// 128-byte line per row where the packed image spreads it over S lines: the
// regroup gathers rows.  The sweep and the regroup both build it here, so
// their MFMA chains agree bit for bit.  (No norm chunk: featnn_row9 takes the
// columns' |y|^2 + B as the MFMA's accumulator input and leaves |x|^2 out.)
template <int S>
__device__ __forceinline__ void row_operand1(const RowArgs5 &a, int p, int row, bool valid, int h,
                                             f16x8 (&A)[S]) {
    const float sc = __uint_as_float(a.sc[p]);
    float x[16 * S];
    const float *xr = a.Xr + ((size_t)p * a.Rmax + row) * a.D;
    if (valid && a.D == 16 * S && ((uintptr_t)xr & 15) == 0) {
#pragma unroll
        for (int q = 0; q < 4 * S; ++q) {
            const float4 v = reinterpret_cast<const float4 *>(xr)[q];
            x[4 * q] = v.x * sc; x[4 * q + 1] = v.y * sc; x[4 * q + 2] = v.z * sc; x[4 * q + 3] = v.w * sc;
        }
    } else if (valid) {
#pragma unroll
        for (int q = 0; q < 16 * S; ++q) x[q] = q < a.D ? xr[q] * sc : 0.0f;
    } else {
#pragma unroll
        for (int q = 0; q < 16 * S; ++q) x[q] = 0.0f;
    }
    // both lane halves' elements at compile-time indices, then the half's pick
    // (an index by h is a select chain over the row)
    auto seg = [&](int k) {
        const _Float16 hi = (_Float16)x[k];
        return k < a.D ? (a.role == 0 ? (_Float16)(-2.0f * (float)hi) : hi) : (_Float16)0.0f;
    };
#pragma unroll
    for (int c = 0; c < S; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const _Float16 v0 = seg(16 * c + j), v1 = seg(16 * c + 8 + j);
            A[c][j] = h ? v1 : v0;
        }
}

// a lane's 16 column terms of column tile ct (register r: column
// 8 (r / 4) + 4 h + (r % 4)), from 32 floats per tile
__device__ __forceinline__ f32x16 colterms(const float *tile32, int h) {
    f32x16 c;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float4 v = *reinterpret_cast<const float4 *>(tile32 + 8 * j + 4 * h);
        c[4 * j] = v.x; c[4 * j + 1] = v.y; c[4 * j + 2] = v.z; c[4 * j + 3] = v.w;
    }
    return c;
}

__device__ __forceinline__ unsigned fbits(float v) { return __float_as_uint(v); }

// min of a lane's 32 values of one step (two column tiles): three v_min3 chains
__device__ __forceinline__ unsigned group_min32(const f32x16 &x, const f32x16 &y) {
    unsigned c0 = umin2(umin2(fbits(x[0]), fbits(x[1])), fbits(x[2]));
    unsigned c1 = umin2(umin2(fbits(x[11]), fbits(x[12])), fbits(x[13]));
    unsigned c2 = umin2(umin2(fbits(y[6]), fbits(y[7])), fbits(y[8]));
#pragma unroll
    for (int r = 3; r < 11; r += 2) c0 = umin2(umin2(c0, fbits(x[r])), fbits(x[r + 1]));
    c1 = umin2(umin2(c1, fbits(x[14])), fbits(x[15]));
#pragma unroll
    for (int r = 0; r < 6; r += 2) c1 = umin2(umin2(c1, fbits(y[r])), fbits(y[r + 1]));
#pragma unroll
    for (int r = 9; r < 15; r += 2) c2 = umin2(umin2(c2, fbits(y[r])), fbits(y[r + 1]));
    c2 = umin2(c2, fbits(y[15]));
    return umin2(umin2(c0, c1), c2);
}

// kIdx: pass 1 / pass 2 (the same code; two names for the profiles)
template <int S, int G, bool kIdx>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void featnn_row9(RowArgs5 a) {
    constexpr int W = 8, RT = 2;          // waves per workgroup, row tiles per wave
    constexpr int NM = 2 * S + 1;         // stored k-chunks of the packed images
    constexpr int NB = S;                 // executed chunks: the f16 segment
    constexpr int kT = G * NB * 64;       // f16x8 of a B buffer's fragments
    constexpr int kB = kT + G * 8;        // + the group's column terms (G x 32 floats)
    static_assert(G % 8 == 0 && S <= 2, "column tiles in pairs; the terms in whole 1 KB DMA pieces");
    constexpr int kTC = G / 8;            // the group's terms: 1 KB pieces
    __shared__ __attribute__((aligned(16))) f16x8 Bs[2 * kB];
    const int b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const int ppx = (a.P + 7) >> 3;
    const int p = a.rbmajor ? (slot % ppx) * 8 + xcd : (slot / a.nrb) * 8 + xcd;
    const int rb = a.rbmajor ? slot / ppx : slot - (slot / a.nrb) * a.nrb;
    if (p >= a.P) return;  // whole block
    const int *rl = a.rlist ? a.rlist + (size_t)p * a.Rmax : nullptr;
    const int nr = rl ? a.rcount[p] : count_of(a.n_rows, p, a.Rmax);
    if (rb * W * RT * 32 >= nr) return;  // whole block: no rows here
    const int wid = threadIdx.x >> 6, l = threadIdx.x & 63, h = l >> 5;
    const int m = count_of(a.n_cols, p, a.Cmax);
    const int qt0 = (rb * W + wid) * RT;  // this wave's first row tile
    const int ntc = (m + 31) >> 5;
    const int ngroups = (ntc + G - 1) / G;
    f16x8 A[RT][NB];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
        const int k = (qt0 + t) * 32 + (l & 31);
        row_operand1<S>(a, p, rl ? (k < nr ? rl[k] : 0) : k, k < nr, h, A[t]);
    }
    // per row tile: B1, B2, I as above; pm the min of the current step's
    // first column tile (the group's first half)
    unsigned B1[RT], B2[RT], I[RT], pm[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) { B1[t] = 0x7f800000u; B2[t] = 0x7f800000u; I[t] = 0u; pm[t] = 0x7f800000u; }
    const f16x8 *bsrc = a.Bp + (size_t)p * a.ntc * NM * 64 + l;
    const float *csrc = a.cct + (size_t)p * a.ntc * 32 + 4 * l;
    auto issue = [&](int grp, int bufi) {
        for (int c = wid; c < G * NB + kTC; c += W) {
            if (c >= G * NB) {  // the group's column terms: G x 128 B, 16 B per lane and piece
                const int tc = c - G * NB;
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(csrc + (size_t)grp * G * 32 + tc * 256),
                    (__attribute__((address_space(3))) void *)(Bs + bufi * kB + kT + tc * 64), 16, 0, 0);
                continue;
            }
            const int g = c / NB, cc = c - g * NB;
            const f16x8 *src = bsrc + ((size_t)(grp * G + g) * NM + cc) * 64;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)src,
                (__attribute__((address_space(3))) void *)(Bs + bufi * kB + c * 64), 16, 0, 0);
        }
    };
    // min of a lane's 16 values of one column tile and c0 (two v_min3 chains)
    auto min16 = [](const f32x16 &x, unsigned c0) {
        unsigned c1 = umin2(umin2(fbits(x[8]), fbits(x[9])), fbits(x[10]));
        c0 = umin2(umin2(c0, fbits(x[0])), fbits(x[1]));
        c1 = umin2(umin2(c1, fbits(x[11])), fbits(x[12]));
        c0 = umin2(umin2(c0, fbits(x[2])), fbits(x[3]));
        c1 = umin2(umin2(c1, fbits(x[13])), fbits(x[14]));
        c0 = umin2(umin2(c0, fbits(x[4])), fbits(x[5]));
        c0 = umin2(umin2(c0, fbits(x[6])), fbits(x[7]));
        return umin2(umin2(c1, fbits(x[15])), c0);
    };
    // row tile t's group of step st closed by its second column tile y
    auto close = [&](const f32x16 &y, int t, unsigned st) {
        const unsigned mn = min16(y, pm[t]);
        // 2nd smallest of {B1, B2, mn}: their median (the full pattern, so it
        // selects to one v_med3_u32)
        const unsigned n2 = umax2(umin2(B1[t], B2[t]), umin2(umax2(B1[t], B2[t]), mn));
        I[t] = mn < B1[t] ? st : I[t];
        B1[t] = umin2(B1[t], mn);
        B2[t] = n2;
    };
    // A tile's 16 column terms per lane (the MFMA's C): registers [0, 4 KL) as
    // KL ds_read_b128 of the LDS copy, the rest from ONE float per lane -- lane
    // l holds column 8 (n / 4) + (n % 4) + 4 h of the tile (n = l % 16), so the
    // DPP row broadcast of row position r gives every lane its register r's
    // column (one v_mov_dpp per register).  Measured (C4, featnn_bench alone):
    // pass 1 1.15 ms with KL = 0, 1.19 with KL = 4 (4 KB of LDS reads per wave
    // and column tile), the mixes 1.21 - 1.24; pass 2 0.77 with KL = 4 against
    // 0.80 with KL = 0.
    const int cl = 8 * ((l & 15) >> 2) + (l & 3) + 4 * h;
#ifndef PCR_CT_LDS1
#define PCR_CT_LDS1 0
#endif
#ifndef PCR_CT_LDS2
#define PCR_CT_LDS2 4
#endif
    constexpr int KL = kIdx ? PCR_CT_LDS1 : PCR_CT_LDS2;
    constexpr int kCR = KL + (KL < 4 ? 1 : 0), kCV = 16 - 4 * KL;  // LDS reads / VALU per tile's terms
    // registers [4 KL, 16) of a tile's terms from the lane's float v
    auto cterms = [&](f32x16 &c, int v) {
#define PCR_BC(r) if ((r) >= 4 * KL) c[r] = __int_as_float(__builtin_amdgcn_mov_dpp(v, 0x150 + (r), 0xf, 0xf, false))
        PCR_BC(0); PCR_BC(1); PCR_BC(2); PCR_BC(3); PCR_BC(4); PCR_BC(5); PCR_BC(6); PCR_BC(7);
        PCR_BC(8); PCR_BC(9); PCR_BC(10); PCR_BC(11); PCR_BC(12); PCR_BC(13); PCR_BC(14); PCR_BC(15);
#undef PCR_BC
    };
    // Schedule per step (two column tiles u = 0, 1; both row tiles in each
    // phase), so one tile's 16 column terms are live at a time:
    //   A: tile u = 0's 4 MFMAs (C = its terms) | the previous step's closes
    //   B: tile u = 1's 4 MFMAs                  | this step's first halves (pm)
    // Each phase reads the next phase's fragments and terms behind its MFMAs.
    f32x16 acc[RT][2];
    // the first phase A closes a harmless pending group: +inf
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][1][r] = __builtin_inff();
    unsigned pend = 0u;
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int grp = 0; grp < ngroups; ++grp) {
        const int buf = grp & 1;
        if (grp + 1 < ngroups) issue(grp + 1, buf ^ 1);
        const f16x8 *Bb = Bs + buf * kB + l;
        const float *Cb = reinterpret_cast<const float *>(Bs + buf * kB + kT);
        const int *Cv = reinterpret_cast<const int *>(Cb) + cl;
        auto cnext = [&](int u) {
            f32x16 c;
#pragma unroll
            for (int j = 0; j < KL; ++j) {
                const float4 v = *reinterpret_cast<const float4 *>(Cb + 32 * u + 8 * j + 4 * h);
                c[4 * j] = v.x; c[4 * j + 1] = v.y; c[4 * j + 2] = v.z; c[4 * j + 3] = v.w;
            }
            if constexpr (KL < 4) cterms(c, Cv[32 * u]);
            return c;
        };
        f16x8 Bf[NB];
        f32x16 Cf;
#pragma unroll
        for (int c = 0; c < NB; ++c) Bf[c] = Bb[c * 64];
        Cf = cnext(0);
        __builtin_amdgcn_sched_barrier(0);  // the group's first reads: a region of their own
#pragma unroll
        for (int st = 0; st < G / 2; ++st) {
            const unsigned stp = (unsigned)(grp * (G / 2) + st);
            // phase A
#pragma unroll
            for (int c = 0; c < NB; ++c)
#pragma unroll
                for (int t = 0; t < RT; ++t)
                    acc[t][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(Bf[c], A[t][c], c == 0 ? Cf : acc[t][0], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < RT; ++t) close(acc[t][1], t, pend);
#pragma unroll
            for (int c = 0; c < NB; ++c) Bf[c] = Bb[((2 * st + 1) * NB + c) * 64];
            Cf = cnext(2 * st + 1);
            SGB(0x002, 2, 0);
#pragma unroll
            for (int i = 0; i < NB * RT; ++i) {
                SGB(0x008, 1, 0);
                SGB(0x002, 5, 0);
            }
            SGB(0x100, NB + kCR, 0);
            SGB(0x002, 6 + kCV, 0);
            __builtin_amdgcn_sched_barrier(0);
            // phase B
#pragma unroll
            for (int c = 0; c < NB; ++c)
#pragma unroll
                for (int t = 0; t < RT; ++t)
                    acc[t][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(Bf[c], A[t][c], c == 0 ? Cf : acc[t][1], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < RT; ++t) pm[t] = min16(acc[t][0], 0x7f800000u);
            if (st + 1 < G / 2) {
#pragma unroll
                for (int c = 0; c < NB; ++c) Bf[c] = Bb[((2 * st + 2) * NB + c) * 64];
                Cf = cnext(2 * st + 2);
            }
#pragma unroll
            for (int i = 0; i < NB * RT; ++i) {
                SGB(0x008, 1, 0);
                SGB(0x002, 4, 0);
            }
            if (st + 1 < G / 2) SGB(0x100, NB + kCR, 0);
            if (st + 1 < G / 2 && kCV) SGB(0x002, kCV, 0);
            __builtin_amdgcn_sched_barrier(0);
            pend = stp;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
#pragma unroll
    for (int t = 0; t < RT; ++t) close(acc[t][1], t, pend);
    // the row's two lane halves: the smaller B1 wins (the lower half on a tie:
    // a zero gap, uncertified either way); the second smallest of the union.
    // The row goes to its winning step's bucket as (row, B1, B2, half); a row
    // that one_term_fails, or past a full bucket, goes to the 3-term screen's
    // list instead (and its record is marked for featnn_finish9 to skip)
    const int nst = a.ntc >> 1;
#pragma unroll
    for (int t = 0; t < RT; ++t) {
        const unsigned o1 = (unsigned)__shfl_xor((int)B1[t], 32, 64);
        const unsigned o2 = (unsigned)__shfl_xor((int)B2[t], 32, 64);
        const unsigned oi = (unsigned)__shfl_xor((int)I[t], 32, 64);
        const unsigned s2 = umin2(umax2(B1[t], o1), umin2(B2[t], o2));
        const bool mine = B1[t] < o1 || (B1[t] == o1 && h == 0);
        const unsigned w1 = mine ? B1[t] : o1;
        const unsigned wst = min(mine ? I[t] : oi, (unsigned)(nst - 1));
        const int k = (qt0 + t) * 32 + (l & 31);
        if (h == 0 && k < nr) {
            // re-read, not kept from the operand build across the sweep (registers)
            const int row = rl ? reinterpret_cast<const volatile int *>(rl)[k] : k;
            const size_t bk = (size_t)p * nst + wst;
            const bool early = one_term_fails<kIdx, S>(a, p, row, w1, s2, a.rre[(size_t)p * a.ntr * 32 + row],
                                                       a.rct[(size_t)p * a.ntr * 32 + row]);
            const int rank = early ? a.bcap : atomicAdd(a.bcnt + bk, 1);
            if (rank < a.bcap) {
                a.blist[bk * a.bcap + rank] = make_uint4((unsigned)row, w1, s2, mine ? 0u : 1u);
            } else {
                a.rec[(size_t)p * a.Rmax + row] = make_uint4(0u, 0u, 0u, 1u);
                a.list[(size_t)p * a.Rmax + atomicAdd(a.count + p, 1)] = row;
            }
        }
    }
}

// featnn_row9's second half (one launch per pass).  A pair's tiles: each
// bucket's rows in 32-row tiles, in bucket order.  Grid (blocks per pair, P):
// a block puts the pair's tiles-per-bucket prefix in LDS once, its waves take
// tiles w, w + 4 gridDim.x, ... (a few each); one MFMA chain over a tile's
// two column tiles (from the packed image) gives every row of the tile its
// winning group's 32 values again (its operand rebuilt from the f32 row, as
// the sweep built it), and the row's (column, B1, B2) record goes to
// featnn_finish9.  (Run inside the sweep, on a workgroup's own 512 rows, the
// regroup cost more: pass 1 2.0 ms against 1.29 + 0.2 -- ~126 chains of ~4
// rows per workgroup and the registers it kept live.)
constexpr int kRegroupMaxSteps = 4096;
template <int S, bool kIdx>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void featnn_regroup9(RowArgs5 a) {
    constexpr int NM = 2 * S + 1, NB = S;
    // the pair's per-step tile prefix and row counts, 2 (steps + 1) ints of
    // dynamic LDS (a static 4097-entry pair held 32 KB and four blocks per CU)
    extern __shared__ int rg_lds[];
    __shared__ int wsum[4];
    const int nst = a.ntc >> 1;
    int *ts = rg_lds, *cn = rg_lds + nst + 1;
    // XCD-aware: a pair's blocks on one XCD (its rows and column image in that L2)
    const int nbp = gridDim.x / (8 * ((a.P + 7) >> 3));  // blocks per pair
    const int bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3;
    const int p = (slot / nbp) * 8 + xcd, bx = slot % nbp;
    if (p >= a.P) return;
    const int t = threadIdx.x, wid = t >> 6, l = t & 63, h = l >> 5;
    const int *bc = a.bcnt + (size_t)p * nst;
    // exclusive prefix of the tiles per bucket: each wave scans a quarter
    const int seg = (nst + 3) >> 2, s0 = min(nst, wid * seg), s1 = min(nst, s0 + seg);
    int run = 0;
    for (int c0 = s0; c0 < s1; c0 += 64) {
        const int i = c0 + l;
        const int ci = i < s1 ? min(bc[i], a.bcap) : 0;
        const int ti = (ci + 31) >> 5;
        int x = ti;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (l >= o) x += y;
        }
        if (i < s1) {
            ts[i] = run + x - ti;
            cn[i] = ci;
        }
        run += __shfl(x, 63, 64);
    }
    if (l == 0) wsum[wid] = run;
    __syncthreads();
    int add = 0;
    for (int ww = 0; ww < wid; ++ww) add += wsum[ww];
    for (int i = s0 + l; i < s1; i += 64) ts[i] += add;
    if (t == 0) ts[nst] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    const int ntiles = ts[nst];
    const f16x8 *bimg = a.Bp + (size_t)p * a.ntc * NM * 64 + l;
    const float *ctp = a.cct + (size_t)p * a.ntc * 32;
    const uint4 *bl = a.blist + (size_t)p * nst * a.bcap;
    // tile q's bucket, its rows' entries (the next tile's loaded while this one runs)
    auto locate = [&](int q, int &b, bool &valid, uint4 &e) {
        int lo = 0, hi = nst;  // ts[lo] <= q < ts[hi]
        while (hi - lo > 1) {
            const int md = (lo + hi) >> 1;
            if (ts[md] <= q) lo = md;
            else hi = md;
        }
        b = lo;
        const int o = (q - ts[b]) * 32 + (l & 31);
        valid = o < cn[b];
        e = valid ? bl[(size_t)b * a.bcap + o] : make_uint4(0u, 0u, 0u, 0u);
    };
    const int qs = nbp * 4;
    int q = bx * 4 + wid, b = 0;
    bool valid = false;
    uint4 e = make_uint4(0u, 0u, 0u, 0u);
    if (q < ntiles) locate(q, b, valid, e);
    for (; q < ntiles; q += qs) {
        int bn = 0;
        bool vn = false;
        uint4 en = make_uint4(0u, 0u, 0u, 0u);
        if (q + qs < ntiles) locate(q + qs, bn, vn, en);
        const int row = (int)e.x;
        f16x8 Bf[2][NB];
        f32x16 acc[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
            for (int c = 0; c < NB; ++c) Bf[u][c] = bimg[((size_t)(2 * b + u) * NM + c) * 64];
            acc[u] = colterms(ctp + (size_t)(2 * b + u) * 32, h);
        }
        f16x8 A[NB];
        row_operand1<S>(a, p, row, valid, h, A);
#pragma unroll
        for (int c = 0; c < NB; ++c)
#pragma unroll
            for (int u = 0; u < 2; ++u)
                acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(Bf[u][c], A[c], acc[u], 0, 0, 0);
        if (valid && (int)e.w == h) {
            // the winner's column (the first in column order among equal
            // patterns) and the group's second smallest value
            unsigned t2 = 0xffffffffu;
            int pos = -1;
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const unsigned v = fbits(acc[u][r]);
                    const bool hit = pos < 0 && v == e.y;
                    t2 = hit ? t2 : umin2(t2, v);
                    pos = hit ? 32 * (2 * b + u) + 8 * (r >> 2) + 4 * h + (r & 3) : pos;
                }
            // a winner not found again (it cannot be: the same chain) is left uncertified
            const unsigned B2 = pos < 0 ? e.y : umin2(e.z, t2);
            a.rec[(size_t)p * a.Rmax + row] = make_uint4((unsigned)(pos < 0 ? 64 * b : pos), e.y, B2, 0u);
        }
        b = bn; valid = vn; e = en;
    }
}

// the rows' certification and outputs (row_tail) in row order, from the
// regroup's (column, B1, B2) records: coalesced, where the regroup visits rows
// in bucket order.  A record marked 1 is a row the sweep gave to the 3-term
// screen.  A row that fails here -- its winning group's own second value
// closed the gap, rare -- goes to a.llist: pass 1 the exact rescan's list (the
// 3-term screen runs beside this kernel), pass 2 none (the resolve sends a
// column whose top-2 gap is too small to the exact column rescan).  1024 rows per block, the listed ones appended with
// one global atomic per block: one counter per pair, the P counters in a few
// cache lines -- per-row atomics from this short kernel serialised there
// (~4 cycles each, 0.15 ms for C4's 73k rows).
template <int S, bool kIdx>
__global__ __launch_bounds__(256) void featnn_finish9(RowArgs5 a) {
    constexpr int R = 4;
    __shared__ int wcnt[4], base;
    const int p = blockIdx.y, t = threadIdx.x, l = t & 63, w = t >> 6;
    const int *rl = a.rlist ? a.rlist + (size_t)p * a.Rmax : nullptr;
    const int nr = rl ? a.rcount[p] : count_of(a.n_rows, p, a.Rmax);
    const int k0 = blockIdx.x * 256 * R;
    if (k0 >= nr) return;  // whole block
    const int m = count_of(a.n_cols, p, a.Cmax);
    int rows[R];
    bool put[R];
    uint4 rc[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int k = k0 + i * 256 + t;
        rows[i] = k < nr ? (rl ? rl[k] : k) : -1;
        rc[i] = rows[i] >= 0 ? a.rec[(size_t)p * a.Rmax + rows[i]] : make_uint4(0u, 0u, 0u, 1u);
    }
    int mine = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        put[i] = false;
        if (rc[i].w == 0u)
            put[i] = row_tail<kIdx, true, S, true>(a, p, rows[i], m, rc[i].y, rc[i].z, (int)rc[i].x,
                                                   a.rre[(size_t)p * a.ntr * 32 + rows[i]], 0.0,
                                                   a.rct[(size_t)p * a.ntr * 32 + rows[i]]);
        mine += put[i] ? 1 : 0;
    }
    // block-wide exclusive offsets of the listed rows
    int x = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (l >= o) x += y;
    }
    if (l == 63) wcnt[w] = x;
    __syncthreads();
    if (t == 0) {
        const int tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
        base = tot && a.llist ? atomicAdd(a.lcount + p, tot) : 0;
    }
    __syncthreads();
    if (!a.llist) return;
    int off = base + x - mine;
    for (int ww = 0; ww < w; ++ww) off += wcnt[ww];
#pragma unroll
    for (int i = 0; i < R; ++i)
        if (put[i]) a.llist[(size_t)p * a.Rmax + off++] = rows[i];
}

struct MutArgs {
    const int32_t *nn12, *n_src, *n_tgt;
    int Nmax, Mmax, mutual, ransac_n, Kt, D, ntm;
    int *used;        // [P][Mmax + 1]: 1 = j in J (2: listed for the rescan), 3: listed, not in J
    int *pos;         // [P][Mmax + 1] scan scratch
    int *jlist, *nj;  // [P][Mmax], [P]: the rows of pass 2, ascending
    const double *v12;
    const float *e12;
    const float4 *wq;   // (w1, w2, e2, the bias in w1 / w2)
    const unsigned *fmax;
    const int32_t *nns; // the screened argmins J is built from (never overwritten by the rescans)
    const float *F, *G; // the f32 clouds and the scale the packs used: the exact distance of a
    const unsigned *mx; // candidate whose screened value is too coarse for its column's gap
    int *flag;        // [P][Nmax + 1]: mutual 0 / 1, 2 = decided by the exact column
    int *list21, *cnt21;
    const int32_t *nn21x;
    int32_t *corres, *n_corres;
};

// J = {nn12[i]} of each pair, ascending (one workgroup per pair).  kLds: the
// flags and their scan in LDS ((Mmax + 1) ints of dynamic LDS), the used flags
// written once, coalesced, for featmut_resolve; else all in the HBM scratch.
template <bool kLds>
__global__ __launch_bounds__(1024) void featmut_jbuild(MutArgs a) {
    extern __shared__ int jsh[];
    const int p = blockIdx.x;
    const int n = count_of(a.n_src, p, a.Nmax), m = count_of(a.n_tgt, p, a.Mmax);
    int *ug = a.used + (size_t)p * (a.Mmax + 1);
    int *u = kLds ? jsh : ug;
    int *ps = kLds ? jsh : a.pos + (size_t)p * (a.Mmax + 1);
    int *jl = a.jlist + (size_t)p * a.Mmax;
    const int32_t *nn = a.nns + (size_t)p * a.Nmax;
    for (int j = threadIdx.x; j < m; j += 1024) u[j] = 0;
    __syncthreads();
    if constexpr (kLds) {
        for (int i = threadIdx.x; i < n; i += 1024) {
            const int j = nn[i];
            if (j >= 0 && j < m) jsh[j] = 1;
        }
        __syncthreads();
        for (int j = threadIdx.x; j < m; j += 1024) ug[j] = jsh[j];
        // in place: flags -> exclusive starts (the scan reads each flag before it
        // writes that position's start; a flag is set iff start[j + 1] > start[j])
        block_exclusive_scan_1024(jsh, jsh, m, false);
        __syncthreads();
        for (int j = threadIdx.x; j < m; j += 1024)
            if (jsh[j + 1] > jsh[j]) jl[jsh[j]] = j;
        if (threadIdx.x == 0) a.nj[p] = jsh[m];
        return;
    }
    for (int i = threadIdx.x; i < n; i += 1024) {
        const int j = nn[i];
        if (j >= 0 && j < m) u[j] = 1;  // plain stores of one value: no race on the result
    }
    __syncthreads();
    for (int j = threadIdx.x; j < m; j += 1024) ps[j] = u[j];
    __syncthreads();
    block_exclusive_scan_1024(ps, ps, m, false);
    for (int j = threadIdx.x; j < m; j += 1024)
        if (u[j]) jl[ps[j]] = j;
    if (threadIdx.x == 0) a.nj[p] = ps[m];
}

// decide each candidate from the pass-2 values, list the undecidable columns
// (once each) for the exact rescan
__global__ __launch_bounds__(256) void featmut_resolve(MutArgs a) {
    const int p = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    const int n = count_of(a.n_src, p, a.Nmax), m = count_of(a.n_tgt, p, a.Mmax);
    if (i >= n) return;
    const size_t oi = (size_t)p * a.Nmax + i;
    const int j = a.nn12[oi];
    int f = 0;
    int *uj = a.used + (size_t)p * (a.Mmax + 1) + j;
    const double e1 = (double)a.e12[oi];  // 0: rescanned (or a zero bound)
    if (j >= 0 && j < m && e1 == 0.0 && (*uj == 0 || *uj == 3)) {
        // J was built from the screened argmins, beside the exact row rescan:
        // a rescanned row's exact argmin j may have no pass-2 values (pass-1
        // certified rows kept the argmin J was built from).  Its exact column
        // argmin decides (listed once: used 0 -> 3)
        f = 2;
        if (atomicCAS(uj, 0, 3) == 0) a.list21[(size_t)p * a.Mmax + atomicAdd(a.cnt21 + p, 1)] = j;
    } else if (j >= 0 && j < m) {
        const size_t oj = (size_t)p * a.Mmax + j;
        const float4 q = a.wq[oj];  // biased values (exact in f64), the bound, the bias
        const double w1 = (double)q.x - (double)q.w, w2 = (double)q.y - (double)q.w, e2 = (double)q.z;
        const double vi = a.v12[oi];
        // slack: the f64 sums of a rescanned value vs the exact real distance
        const double sl = 1e-9 * (__builtin_fabs(w1) + __builtin_fabs(vi));
        bool done = false;
        if (w2 - w1 > 2.0 * (e2 + e1 + sl)) {
            f = (vi <= w1 + e2 + e1 + sl) ? 1 : 0;
            done = true;
        } else if (e1 != 0.0) {
            // the row's screened value is too coarse for this column's gap (the
            // 1-term screen's bound): its exact distance, the oracle's f64 sum in
            // the rescan's units, decides when the gap alone allows
            const float *fr = a.F + oi * a.D, *gr = a.G + oj * a.D;
            double acc = 0.0;
            for (int k = 0; k < a.D; ++k) {
                const double df = (double)fr[k] - (double)gr[k];
                acc = acc + df * df;
            }
            const double sc = (double)__uint_as_float(a.mx[p]);
            const double vx = acc * sc * sc;
            const double slx = 1e-9 * (__builtin_fabs(w1) + __builtin_fabs(vx));
            if (w2 - w1 > 2.0 * (e2 + slx)) {
                f = (vx <= w1 + e2 + slx) ? 1 : 0;
                done = true;
            }
        }
        if (!done) {
            f = 2;
            if (atomicCAS(uj, 1, 2) == 1)
                a.list21[(size_t)p * a.Mmax + atomicAdd(a.cnt21 + p, 1)] = j;
        }
    }
    a.flag[(size_t)p * (a.Nmax + 1) + i] = f;
}

// the flags (undecided ones from the exact column argmin) -> corres_build's
// ordered compaction and fallback (one workgroup per pair)
__global__ __launch_bounds__(1024) void featmut_corres(MutArgs a) {
    const int p = blockIdx.x;
    const int n = count_of(a.n_src, p, a.Nmax), m = count_of(a.n_tgt, p, a.Mmax);
    const int32_t *a12 = a.nn12 + (size_t)p * a.Nmax;
    int *f = a.flag + (size_t)p * (a.Nmax + 1);
    int32_t *co = a.corres + (size_t)p * a.Nmax * 2;
    if (a.mutual) {
        for (int i = threadIdx.x; i < n; i += 1024) {
            const int v = f[i];
            if (v == 2) f[i] = (a.nn21x[(size_t)p * a.Mmax + a12[i]] == i) ? 1 : 0;
        }
    } else {
        for (int i = threadIdx.x; i < n; i += 1024) f[i] = 0;
    }
    (void)m;
    __syncthreads();
    block_exclusive_scan_1024(f, f, n, false);
    const int total = f[n];
    const bool use_mutual = a.mutual && total >= 3 * a.ransac_n;
    if (use_mutual) {
        for (int i = threadIdx.x; i < n; i += 1024) {
            const int pos = f[i];
            if (f[i + 1] != pos) { co[2 * pos] = i; co[2 * pos + 1] = a12[i]; }
        }
    } else {
        for (int i = threadIdx.x; i < n; i += 1024) { co[2 * i] = i; co[2 * i + 1] = a12[i]; }
    }
    if (threadIdx.x == 0) a.n_corres[p] = use_mutual ? total : n;
}

}  // namespace

// packed operands, norms and per-pair maxima of both clouds (shared by the
// dual screen and the mutual path)
struct V5Buf {
    int S, NM, NX, W, nrb, ntn, ntm, ctbits;  // S chunks per D-segment, NM stored, NX executed
    Split5 sp;
    f16x8 *Ap, *Bp;
    float *fnr, *gnr;
    unsigned *gmax, *fmax, *mx;
    int *cnt12, *cnt21, *list12, *list21;
    unsigned *gemax, *femax;  // per pair max |x - f16(x)| of the column (G) / row (F) images
    int *fbc12, *fbc21, *fbl12, *fbl21;  // the rows a 1-term screen left for the 3-term one
    float *fre, *gre;                    // per row |x - f16(x)| of F / G (scaled, rounded up)
    float *fct, *gct;                    // per row f32(|x|^2 + B) of F / G (featnn_row9's column terms)
    float *cbias;                        // [P] their B (feat_colterms)
};

static int v5_prepare(const float *F, const float *G, int P, int Nmax, int Mmax, int D,
                      const int32_t *n_src, const int32_t *n_tgt, hipStream_t s, V5Buf &v) {
    v.S = cdiv(D, 16);
    v.NM = 2 * v.S + 1;
    v.NX = 3 * v.S + 1;
    v.sp = split5_params(D);
    v.W = 8;                                          // waves (32-row tiles) per workgroup
    v.nrb = cdiv(cdiv(Nmax, 32), v.W);                // dual screen row blocks
    // row tiles, padded to whole blocks of the dual screen (8 tiles) and of the
    // row screens (8 waves x row_tiles(S) tiles; the sentinel rows are valid encodings)
    v.ntn = cdiv(cdiv(Nmax, 32), 16) * 16;
    v.ntm = cdiv(cdiv(Mmax, 32), std::max(kRow8G, kRow9G)) * std::max(kRow8G, kRow9G);  // column tiles, whole groups
    v.ctbits = 1;
    while ((1 << v.ctbits) < std::max(v.ntm, v.ntn)) ++v.ctbits;
    PCR_REQUIRE(v.ctbits <= 16, PCR_ERR_ARG, "feature_match: N=%d / M=%d too large", Nmax, Mmax);
    const int NM = v.NM, ntn = v.ntn, ntm = v.ntm;
    const size_t ap = (size_t)P * ntn * NM * 64, bp = (size_t)P * ntm * NM * 64;  // f16x8
    const size_t nn_n = (size_t)P * ntn * 32, nn_m = (size_t)P * ntm * 32;
    const size_t bytes =
        16 * (ap + bp) + 4 * (3 * (nn_n + nn_m) + 9 * (size_t)P + 2 * (size_t)P * (Nmax + Mmax) + 19 * (size_t)P);
    char *ws = (char *)workspace(2, bytes + 256);
    PCR_REQUIRE(ws, PCR_ERR_NOMEM, "feature_match: %s", pcr_last_error());
    v.Ap = (f16x8 *)ws;
    v.Bp = v.Ap + ap;
    v.fnr = (float *)(v.Bp + bp);
    v.gnr = v.fnr + nn_n;
    v.fre = v.gnr + nn_m;
    v.gre = v.fre + nn_n;
    v.fct = v.gre + nn_m;
    v.gct = v.fct + nn_n;
    // [0,P): max|y|  [P,2P): max|x|  [2P,3P): the scale used  [3P,4P): cnt12  [4P,5P): cnt21
    // [5P,6P): gemax  [6P,7P): femax  [7P,8P): fbc12  [8P,9P): fbc21 (feat_sample clears
    // all but the scale)
    v.gmax = (unsigned *)(v.gct + nn_m);
    v.fmax = v.gmax + P;
    v.mx = v.gmax + 2 * P;
    v.cnt12 = (int *)(v.gmax + 3 * P);
    v.cnt21 = v.cnt12 + P;
    v.gemax = v.gmax + 5 * P;
    v.femax = v.gmax + 6 * P;
    v.fbc12 = (int *)(v.gmax + 7 * P);
    v.fbc21 = v.fbc12 + P;
    v.list12 = v.fbc21 + P;                    // per pair, stride Nmax
    v.list21 = v.list12 + (size_t)P * Nmax;    // per pair, stride Mmax
    v.fbl12 = v.list21 + (size_t)P * Mmax;     // per pair, stride Nmax
    v.fbl21 = v.fbl12 + (size_t)P * Nmax;      // per pair, stride Mmax
    unsigned *mxp = (unsigned *)(v.fbl21 + (size_t)P * Mmax);  // [P][2][zr] partial maxima (repair)
    unsigned *smax = mxp + 2 * (size_t)P * 8;                     // [P] sample maxima
    int *bad = (int *)(smax + P);                                  // [P] repair flags
    v.cbias = (float *)(bad + P);                                  // [P] featnn_row9's B
    prof_begin(s, kProfFeatPack);
    hipLaunchKernelGGL(feat_sample, dim3(P), dim3(256), 0, s, F, n_src, Nmax, G, n_tgt, Mmax, D, smax, v.gmax,
                       bad, P);
    PCR_LAUNCH_CHECK();
    // the repair passes: few blocks walking the flags (empty in the common case)
    const int R = std::min(P, kRepairR), zr = 8;
    for (int rep = 0; rep < 2; ++rep) {
        PackCtl pc{smax, mxp, zr, P, rep, bad, v.mx};
        if (rep) {
            hipLaunchKernelGGL(feat_maxabs, dim3(R, 2, zr), dim3(1024), 0, s, F, n_src, Nmax, G, n_tgt, Mmax, D,
                               mxp, v.gmax, bad, P);
            PCR_LAUNCH_CHECK();
        }
        const int gy = rep ? R : P;
        PackIO io{{F, G}, {n_src, n_tgt}, {Nmax, Mmax}, {ntn, ntm}, {v.Ap, v.Bp}, {v.fnr, v.gnr}, {v.fmax, v.gmax},
                  {v.femax, v.gemax}, {v.fre, v.gre}, {v.fct, v.gct}};
        const dim3 grid(cdiv(std::max(ntn, ntm), 4), gy, 2);
        if (D == 32) hipLaunchKernelGGL(feat_pack5r<32>, grid, dim3(256), 0, s, io, v.sp, pc);  // register-resident
        else hipLaunchKernelGGL(feat_pack5, grid, dim3(256), 0, s, io, D, v.S, v.sp, pc);
        PCR_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(feat_colterms, dim3(cdiv(std::max(ntn, ntm) * 32, 256), P, 2), dim3(256), 0, s, v.fct, v.gct,
                       ntn, ntm, v.fmax, v.gmax, v.cbias);
    PCR_LAUNCH_CHECK();
    prof_end(s, kProfFeatPack);
    return PCR_OK;
}

static RescanArgs5 rescan_args(const float *F, const float *G, const int32_t *n_src,
                               const int32_t *n_tgt, int Nmax, int Mmax, int D) {
    RescanArgs5 ra;
    ra.F = F; ra.G = G; ra.n_src = n_src; ra.n_tgt = n_tgt; ra.Nmax = Nmax; ra.Mmax = Mmax;
    ra.D = D;
    ra.list12 = ra.list21 = nullptr;
    ra.cnt12 = ra.cnt21 = nullptr;
    ra.nn12 = ra.nn21 = nullptr;
    ra.cap = 256;
    ra.sd = nullptr;
    ra.sj = nullptr;
    ra.v12 = nullptr; ra.e12 = nullptr; ra.mx = nullptr; ra.T = 0;
    return ra;
}

// exact f64 rescan of the listed rows of both directions (a direction with a
// zero count costs its empty blocks only)
static int run_rescan(RescanArgs5 &ra, int P, int D, hipStream_t s) {
    const bool v4 = (D % 4) == 0 && ((uintptr_t)ra.F & 15) == 0 && ((uintptr_t)ra.G & 15) == 0;
    // candidate slices per (pair, direction): ~8192 blocks whatever the batch --
    // a pair's list is short (C4: 27 rows on average, 45 at most, one or two
    // 32-row batches), so a block is a short chain of dependent candidate
    // loads and more, shorter slices finish sooner (256 pairs: 4 / 8 / 16
    // slices 0.575 / 0.489 / 0.471 ms per step)
    const int S = std::max(1, std::min(16, 4096 / std::max(P, 1)));
    if (S > 1) {
        char *rw = (char *)workspace(6, (sizeof(double) + sizeof(int)) * (size_t)P * 2 * ra.cap * S + 64);
        PCR_REQUIRE(rw, PCR_ERR_NOMEM, "feature_match: %s", pcr_last_error());
        ra.sd = (double *)rw;
        ra.sj = (int *)(ra.sd + (size_t)P * 2 * ra.cap * S);
    }
    const dim3 rg(P, 2, S);
    if (getenv("PCR_RESCAN_DEBUG")) {  // diagnostic: the per-pair list lengths (host sync)
        for (int d = 0; d < 2; ++d) {
            const int *c = d ? ra.cnt21 : ra.cnt12;
            if (!c) continue;
            std::vector<int> h((size_t)P);
            PCR_HIP_CHECK(hipMemcpyAsync(h.data(), c, sizeof(int) * (size_t)P, hipMemcpyDeviceToHost, s));
            PCR_HIP_CHECK(hipStreamSynchronize(s));
            long long tot = 0;
            int mx = 0, over = 0;
            for (int v : h) { tot += v; mx = std::max(mx, v); over += v > ra.cap ? 1 : 0; }
            std::sort(h.begin(), h.end());
            fprintf(stderr, "rescan dir %d: rows %lld, max %d, p50 %d, p90 %d, p99 %d, pairs over cap %d\n", d, tot,
                    mx, h[P / 2], h[(P * 9) / 10], h[(P * 99) / 100], over);
        }
    }
    prof_begin(s, kProfFeatRescan);
    const int dv = cdiv(D, 16) * 16;
#define PCR_R3(DVV)                                                                    \
    if (dv == DVV) {                                                                    \
        if (v4) hipLaunchKernelGGL((featnn_rescan3<DVV, true>), rg, dim3(256), 0, s, ra); \
        else hipLaunchKernelGGL((featnn_rescan3<DVV, false>), rg, dim3(256), 0, s, ra);  \
    }
    PCR_R3(16) PCR_R3(32) PCR_R3(48) PCR_R3(64)
#undef PCR_R3
    PCR_LAUNCH_CHECK();
    if (S > 1) {
        hipLaunchKernelGGL(featnn_rescan_merge, dim3(P, 2), dim3(256), 0, s, ra, S);
        PCR_LAUNCH_CHECK();
    }
    prof_end(s, kProfFeatRescan);
    return PCR_OK;
}

static int feature_match_v5(const float *F, const float *G, int P, int Nmax, int Mmax, int D,
                            const int32_t *n_src, const int32_t *n_tgt, int32_t *nn12,
                            int32_t *nn21, hipStream_t s) {
    V5Buf v;
    int rc = v5_prepare(F, G, P, Nmax, Mmax, D, n_src, n_tgt, s, v);
    if (rc != PCR_OK) return rc;
    const int W = v.W, nrb = v.nrb, ntm = v.ntm;
    DualArgs5 d;
    d.Ap = v.Ap; d.Bp = v.Bp; d.fnr = v.fnr; d.gnr = v.gnr; d.fmax = v.fmax; d.gmax = v.gmax;
    d.n_src = n_src; d.n_tgt = n_tgt; d.P = P; d.Nmax = Nmax; d.Mmax = Mmax; d.ntn = v.ntn;
    d.ntm = ntm; d.nrb = nrb; d.D = D; d.nn12 = nn12; d.list12 = v.list12;
    d.count12 = v.cnt12;
    // the dual screen's row code: column tiles only
    d.ctbits = 1;
    while ((1 << d.ctbits) < ntm) ++d.ctbits;
    const size_t cpn = (size_t)P * nrb * ntm * 32;
    char *cw = (char *)workspace(11, cpn * 8 + 64);
    PCR_REQUIRE(cw, PCR_ERR_NOMEM, "feature_match: %s", pcr_last_error());
    d.cp1 = (float *)cw;
    d.cp2 = d.cp1 + cpn;
    d.cpi = nullptr;
    const long long nblk = 8LL * nrb * cdiv(P, 8);  // XCD-aware 1-D grid
    PCR_REQUIRE(nblk < (1LL << 31), PCR_ERR_ARG, "feature_match: grid too large");
    prof_begin(s, kProfFeatScreen);
    {
        switch (v.S) {
#define PCR_D7CASE(K)                                                                        \
    case K:                                                                                  \
        hipLaunchKernelGGL((featnn_dual7<K, (K <= 2 ? 8 : 4)>), dim3((unsigned)nblk),          \
                           dim3(512), 0, s, d);                                              \
        break;
            PCR_D7CASE(1) PCR_D7CASE(2) PCR_D7CASE(3) PCR_D7CASE(4)
#undef PCR_D7CASE
            default: set_error("feature dim too large for the f16 split screen"); return PCR_ERR_ARG;
        }
    }
    PCR_LAUNCH_CHECK();
    prof_end(s, kProfFeatScreen);
    hipLaunchKernelGGL(featnn_colmerge5, dim3(cdiv(Mmax, 256), P), dim3(256), 0, s, d, nn21, v.list21,
                       v.cnt21, 16 * v.NX, W);
    PCR_LAUNCH_CHECK();
    RescanArgs5 ra = rescan_args(F, G, n_src, n_tgt, Nmax, Mmax, D);
    ra.list12 = v.list12; ra.list21 = v.list21; ra.cnt12 = v.cnt12; ra.cnt21 = v.cnt21;
    ra.nn12 = nn12; ra.nn21 = nn21;
    return run_rescan(ra, P, D, s);
}

// row tiles per wave of the row screens (featnn_row7)
// (two up to D = 32; one above, where two tiles' accumulators and fragments
// spilled at S = 4: 256 VGPRs + 179 spilled)
constexpr int row_tiles(int S) { return S <= 2 ? 2 : 1; }
// column tiles per LDS group of the row screens (featnn_row7's G)
constexpr int row_group(int S) { return S <= 2 ? 8 : 4; }

// row tiles per wave of pass 2 at S = 2: one (128 VGPRs, four waves per SIMD
// instead of two, at twice the B-fragment reads: 1.58 vs 1.64 ms); pass 1 at
// S <= 2 is featnn_row8; other S: row_tiles
static int pass_tiles(int S, bool pass2) { return (S == 2 && pass2) ? 1 : row_tiles(S); }

// one featnn_row8 launch over a grid for all Rmax rows (list mode: the blocks
// past the pair's count exit at once)
template <bool kIdx, bool kOne>
static int launch_row8(const RowArgs5 &r0, int S, hipStream_t s) {
    RowArgs5 r = r0;
    r.nrb = cdiv(cdiv(r.Rmax, 32), 8 * 2);  // 8 waves x 2 row tiles per workgroup
    const int csl = r.rbmajor ? r.csl : 1;
    const long long nblk = 8LL * r.nrb * csl * cdiv(r.P, 8);  // XCD-aware 1-D grid
    PCR_REQUIRE(nblk < (1LL << 31), PCR_ERR_ARG, "feature_corres: grid too large");
    if (S == 1) hipLaunchKernelGGL((featnn_row8<1, kRow8G, kIdx, kOne>), dim3((unsigned)nblk), dim3(512), 0, s, r);
    else hipLaunchKernelGGL((featnn_row8<2, kRow8G, kIdx, kOne>), dim3((unsigned)nblk), dim3(512), 0, s, r);
    PCR_LAUNCH_CHECK();
    if (csl > 1) {
        const dim3 mg(cdiv(r.Rmax, 256), r.P);
        if (S == 1) hipLaunchKernelGGL((featnn_slicemerge<1, kIdx>), mg, dim3(256), 0, s, r);
        else hipLaunchKernelGGL((featnn_slicemerge<2, kIdx>), mg, dim3(256), 0, s, r);
        PCR_LAUNCH_CHECK();
    }
    return PCR_OK;
}

// column slices of the 3-term screens' list mode: a pair's short list is
// one workgroup per slice -- at 256 pairs one slice (the chip is full), at
// 32 pairs 8 (one block per pair left 224 CUs idle: ~0.2 ms per launch)
static int list_slices(int P) { return std::max(1, std::min(8, 256 / std::max(P, 1))); }

// PCR_FEAT_ROW9=0: the round-6 featnn_row8 1-term passes (A/B; read per call)
static bool feat_row9() {
    const char *e = getenv("PCR_FEAT_ROW9");
    return !(e && e[0] == '0');
}

template <bool kIdx>
static int launch_row9(const RowArgs5 &r0, int S, hipStream_t s) {
    RowArgs5 r = r0;
    r.nrb = cdiv(cdiv(r.Rmax, 32), 8 * 2);  // 8 waves x 2 row tiles per workgroup
    const long long nblk = 8LL * r.nrb * cdiv(r.P, 8);  // XCD-aware 1-D grid
    PCR_REQUIRE(nblk < (1LL << 31), PCR_ERR_ARG, "feature_corres: grid too large");
    constexpr int G = kIdx ? kRow9G1 : kRow9G;
    if (S == 1) hipLaunchKernelGGL((featnn_row9<1, G, kIdx>), dim3((unsigned)nblk), dim3(512), 0, s, r);
    else hipLaunchKernelGGL((featnn_row9<2, G, kIdx>), dim3((unsigned)nblk), dim3(512), 0, s, r);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

template <bool kIdx>
static int launch_regroup9(const RowArgs5 &r, int S, hipStream_t s) {
    // a pair has at most one tile per 32 rows plus one per bucket: ~6 per
    // wave (PCR_REGROUP_TPB: tiles per 4-wave block; 4 / 6 / 12 / 24 measured
    // 0.36 / 0.34 / 0.30 / 0.29 ms per C4 step); 1-D, a pair's blocks on one XCD
    static const int tpb = [] {
        const char *e = getenv("PCR_REGROUP_TPB");
        const int v = e ? atoi(e) : 24;
        return v >= 4 ? v : 24;
    }();
    const int nbp = cdiv(cdiv(r.Rmax, 32) + r.ntc / 2, tpb);
    const dim3 grid((unsigned)(8LL * nbp * cdiv(r.P, 8)));
    const dim3 fgrid(cdiv(r.Rmax, 1024), r.P);
    const size_t sm = sizeof(int) * (2 * (size_t)(r.ntc / 2) + 1);
    if (S == 1) {
        hipLaunchKernelGGL((featnn_regroup9<1, kIdx>), grid, dim3(256), sm, s, r);
        hipLaunchKernelGGL((featnn_finish9<1, kIdx>), fgrid, dim3(256), 0, s, r);
    } else {
        hipLaunchKernelGGL((featnn_regroup9<2, kIdx>), grid, dim3(256), sm, s, r);
        hipLaunchKernelGGL((featnn_finish9<2, kIdx>), fgrid, dim3(256), 0, s, r);
    }
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

// a 3-term fallback screen (list mode), in its profile slot
template <bool kIdx>
static int launch_fallback(const RowArgs5 &r, int S, hipStream_t q, int slot) {
    prof_begin(q, slot);
    const int rc = launch_row8<kIdx, false>(r, S, q);
    prof_end(q, slot);
    return rc;
}

// side(q) then main() on s; with PCR_FEAT_BESIDE=1, side(q) on the second
// side stream beside main() on s, joined back into s.  Measured (featnn_bench,
// mutual): 256 pairs 3.42 ms either way, 32 pairs 0.778 beside vs 0.755 ms in
// order -- the 3-term screen and the regroup compete for the same CUs, so the
// default is in order
template <class Side, class Main>
static int beside(hipStream_t s, Side side, Main main) {
    static const bool off = [] {
        const char *e = getenv("PCR_FEAT_BESIDE");
        return !(e && e[0] == '1');
    }();
    hipStream_t q = s;
    hipEvent_t ef = nullptr, ej = nullptr;
    int rc = off ? PCR_OK : side_stream(&q, &ef, &ej, 2);
    if (rc != PCR_OK) return rc;
    if (q != s) {
        PCR_HIP_CHECK(hipEventRecord(ef, s));
        PCR_HIP_CHECK(hipStreamWaitEvent(q, ef, 0));
    }
    if ((rc = side(q)) != PCR_OK) return rc;
    if (q != s) PCR_HIP_CHECK(hipEventRecord(ej, q));
    prof_begin(s, kProfFeatRegroup);
    rc = main();
    prof_end(s, kProfFeatRegroup);
    if (rc != PCR_OK) return rc;
    if (q != s) PCR_HIP_CHECK(hipStreamWaitEvent(s, ej, 0));
    return PCR_OK;
}

// the 1-term screens in front of the 3-term ones (S <= 2): on by default,
// PCR_FEAT_ONE=0 for the round-5 path (A/B, the parity tests; read per call)
static bool feat_one_term() {
    const char *e = getenv("PCR_FEAT_ONE");
    return !(e && e[0] == '0');
}

// one row screen launch (pass 1: kIdx, F rows; pass 2: the J rows of G)
template <bool kIdx>
static int launch_row7(const RowArgs5 &r, int S, hipStream_t s, int rt) {
    const long long nblk = 8LL * r.nrb * cdiv(r.P, 8);  // XCD-aware 1-D grid
    PCR_REQUIRE(nblk < (1LL << 31), PCR_ERR_ARG, "feature_match: grid too large");
    if (rt == 1 && row_tiles(S) != 1 && S == 2) {
        hipLaunchKernelGGL((featnn_row7<2, row_group(2), kIdx, 1>), dim3((unsigned)nblk), dim3(512), 0, s, r);
        PCR_LAUNCH_CHECK();
        return PCR_OK;
    }
    switch (S) {
#define PCR_R7CASE(K)                                                                            \
    case K:                                                                                      \
        hipLaunchKernelGGL((featnn_row7<K, row_group(K), kIdx, row_tiles(K)>), dim3((unsigned)nblk), \
                           dim3(512), 0, s, r);                                                  \
        break;
        PCR_R7CASE(1) PCR_R7CASE(2) PCR_R7CASE(3) PCR_R7CASE(4)
#undef PCR_R7CASE
        default: set_error("feature dim too large for the f16 split screen"); return PCR_ERR_ARG;
    }
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

// the mutual path (see featnn_row7): nn12 and the correspondences without the
// column screen of every target
static int feature_corres_v5(const float *F, const float *G, int P, int Nmax, int Mmax, int D,
                             const int32_t *n_src, const int32_t *n_tgt, int mutual, int ransac_n,
                             int32_t *nn12, int32_t *corres, int32_t *n_corres, hipStream_t s) {
    V5Buf v;
    int rc = v5_prepare(F, G, P, Nmax, Mmax, D, n_src, n_tgt, s, v);
    if (rc != PCR_OK) return rc;
    const int ntn = v.ntn, ntm = v.ntm;
    // scratch: v12 [P][Nmax] f64 | e12 [P][Nmax] f32 | wq [P][Mmax] float4 | used, pos
    // [P][Mmax+1] | jlist, nn21x [P][Mmax] | flag [P][Nmax+1] | nj, zero [P] | nns [P][Nmax]
    const size_t pn = (size_t)P * Nmax, pm = (size_t)P * Mmax;
    // featnn_row9's buckets (a pass's rows by winning step): 4x a bucket's mean
    // row count, at least 64 rows; a fuller bucket sends rows to the 3-term screen
    const int nst1 = ntm / 2, nst2 = ntn / 2;
    const int cap1 = std::max(64, 4 * cdiv(Nmax, nst1)), cap2 = std::max(64, 4 * cdiv(Mmax, nst2));
    const size_t pb = (size_t)P * std::max(nst1, nst2);
    const size_t pl = (size_t)P * std::max((size_t)nst1 * cap1, (size_t)nst2 * cap2);
    const size_t pr = (size_t)P * std::max(Nmax, Mmax);
    const int fsl = list_slices(P);
    const size_t pt = fsl > 1 ? (size_t)fsl * pr : 0;  // the sliced 3-term screens' partials
    const size_t bytes = 8 * pn + 4 * pn + 16 * pm + 8 * (pm + P) + 8 * pm + 4 * (pn + P) + 8 * (size_t)P + 4 * pn + 16 +
                         16 * (pl + pr + pt) + 4 * pb + 16;

    bool fresh = false;
    char *ws = (char *)workspace(33, bytes + 256, &fresh);
    PCR_REQUIRE(ws, PCR_ERR_NOMEM, "feature_corres: %s", pcr_last_error());
    MutArgs ma;
    double *v12 = (double *)ws;
    float *e12 = (float *)(v12 + pn);
    float4 *wq = reinterpret_cast<float4 *>(((uintptr_t)(e12 + pn) + 15) & ~(uintptr_t)15);
    ma.used = (int *)(wq + pm);
    ma.pos = ma.used + pm + P;
    ma.jlist = ma.pos + pm + P;
    int *nn21x = ma.jlist + pm;
    ma.flag = nn21x + pm;
    ma.nj = ma.flag + pn + P;
    int *zero = ma.nj + P;
    int32_t *nns = zero + P;
    uint4 *blist = reinterpret_cast<uint4 *>(((uintptr_t)(nns + pn) + 15) & ~(uintptr_t)15);
    uint4 *rec = blist + pl;
    uint4 *part = rec + pr;
    int *bcnt = reinterpret_cast<int *>(part + pt);
    const bool one = v.S <= 2 && feat_one_term();
    // (the regroup keeps a pair's per-step prefix in LDS)
    const bool use9 = one && feat_row9() && std::max(ntm, ntn) / 2 <= kRegroupMaxSteps;
    // a constant zero count per pair (read only): cleared when the slot is new
    // or was last used for fewer pairs
    static thread_local const void *z_ptr = nullptr;
    static thread_local int z_cnt = 0;
    if (fresh || z_ptr != (const void *)zero || z_cnt < P) {
        PCR_HIP_CHECK(hipMemsetAsync(zero, 0, sizeof(int) * (size_t)P, s));
        z_ptr = zero;
        z_cnt = P;
    }
    ma.nn12 = nn12; ma.n_src = n_src; ma.n_tgt = n_tgt; ma.Nmax = Nmax; ma.Mmax = Mmax;
    ma.mutual = mutual; ma.ransac_n = ransac_n; ma.Kt = 16 * v.NX; ma.D = D; ma.ntm = ntm;
    ma.v12 = v12; ma.e12 = e12; ma.wq = wq; ma.fmax = v.fmax;
    ma.nns = v.S <= 2 ? nns : nn12;  // featnn_row7 (S > 2) writes no copy
    ma.F = F; ma.G = G; ma.mx = v.mx;
    ma.list21 = v.list21; ma.cnt21 = v.cnt21; ma.nn21x = nn21x;
    ma.corres = corres; ma.n_corres = n_corres;
    // pass 1: F rows x all G columns
    RowArgs5 r;
    r.Ap = v.Ap; r.Bp = v.Bp; r.rnr = v.fnr; r.cmax = v.gmax; r.n_rows = n_src; r.n_cols = n_tgt;
    r.rlist = nullptr; r.rcount = nullptr; r.P = P; r.Rmax = Nmax; r.Cmax = Mmax; r.ntr = ntn;
    const int rt1 = pass_tiles(v.S, false);
    r.ntc = ntm; r.nrb = cdiv(cdiv(Nmax, 32), v.W * rt1); r.D = D; r.ctbits = 1;
    while ((1 << r.ctbits) < ntm) ++r.ctbits;
    r.nn = nn12; r.v = v12; r.e = e12; r.list = v.list12; r.count = v.cnt12;
    r.wq = nullptr;
    r.Xr = F; r.sc = v.mx; r.role = 0; r.cs = v.sp.cs;  // featnn_row8 builds its rows from F
    r.cemax = v.gemax; r.nns = nns; r.fbdiag = 0; r.rbmajor = 0;
    r.rre = v.fre; r.bcnt = bcnt; r.blist = blist; r.bcap = cap1; r.rec = rec;
    r.cct = v.gct; r.rct = v.fct; r.cbias = v.cbias;
    r.csl = 1; r.part = part; r.llist = nullptr; r.lcount = nullptr;
    if (prep_event && prep_at == 2) {
        PCR_HIP_CHECK(hipEventRecord(prep_event, s));
        if (prep_fn && (rc = prep_fn(prep_ctx)) != PCR_OK) return rc;
        prep_fn = nullptr;
    }
    prof_begin(s, kProfFeatScreen);
    if (one) {  // two column tiles per step (featnn_row8), 1-term; the rows it leaves to the 3-term
        r.list = v.fbl12; r.count = v.fbc12;
        RowArgs5 r1 = r;
        r1.rlist = v.fbl12; r1.rcount = v.fbc12; r1.list = v.list12; r1.count = v.cnt12; r1.fbdiag = 1;
        r1.rbmajor = 1; r1.csl = fsl;
        if (use9) {  // featnn_row9's sweep, then the winners' groups again (regroup + finish)
            PCR_HIP_CHECK(hipMemsetAsync(bcnt, 0, sizeof(int) * (size_t)P * nst1, s));
            if ((rc = launch_row9<true>(r, v.S, s)) != PCR_OK) return rc;
            prof_end(s, kProfFeatScreen);
            // the 3-term screen of the rows the sweep listed, beside the regroup
            RowArgs5 rg = r;
            rg.llist = v.list12; rg.lcount = v.cnt12;
            if ((rc = beside(s, [&](hipStream_t q) { return launch_fallback<true>(r1, v.S, q, kProfFeatScreen1b); },
                             [&] { return launch_regroup9<true>(rg, v.S, s); })) != PCR_OK)
                return rc;
        } else {
            if ((rc = launch_row8<true, true>(r, v.S, s)) != PCR_OK) return rc;
            prof_end(s, kProfFeatScreen);
            if ((rc = launch_fallback<true>(r1, v.S, s, kProfFeatScreen1b)) != PCR_OK) return rc;
        }
    } else if (v.S <= 2) {  // the 3-term screen only
        if ((rc = launch_row8<true, false>(r, v.S, s)) != PCR_OK) return rc;
        prof_end(s, kProfFeatScreen);
    } else {
        rc = launch_row7<true>(r, v.S, s, rt1);
        if (rc != PCR_OK) return rc;
        prof_end(s, kProfFeatScreen);
    }
    if (prep_event && prep_at == 1) {
        PCR_HIP_CHECK(hipEventRecord(prep_event, s));
        if (prep_fn && (rc = prep_fn(prep_ctx)) != PCR_OK) return rc;
        prep_fn = nullptr;
    }
    RescanArgs5 ra = rescan_args(F, G, n_src, n_tgt, Nmax, Mmax, D);
    ra.list12 = v.list12; ra.list21 = v.list21; ra.cnt12 = v.cnt12; ra.cnt21 = zero;
    ra.nn12 = nn12; ra.nn21 = nn21x;
    ra.v12 = v12; ra.e12 = e12; ra.mx = v.mx; ra.T = v.sp.T;
    // mutual: the exact rescan of the uncertified rows runs on a side stream
    // beside J's build and pass 2, which read none of its results (J from the
    // screened argmins; featmut_resolve, after the join, sends a rescanned
    // row's new argmin outside J to the exact column rescan).  Large batches
    // only: at 32-128 pairs it gained nothing.  The side stream is the
    // pipeline's prep stream (its grid builds are enqueued first, prep_fn)
    hipStream_t rs = s;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    if (mutual && P >= 192) {
        rc = side_stream(&rs, &ev_fork, &ev_join, 1);
        if (rc != PCR_OK) return rc;
        PCR_HIP_CHECK(hipEventRecord(ev_fork, s));
        PCR_HIP_CHECK(hipStreamWaitEvent(rs, ev_fork, 0));
    }
    rc = run_rescan(ra, P, D, rs);
    if (rc != PCR_OK) return rc;
    if (rs != s) PCR_HIP_CHECK(hipEventRecord(ev_join, rs));
    if (mutual) {
        // the LDS form when its dynamic (Mmax + 1) ints fit beside the kernel's
        // static LDS (the block scan's wave totals) in 64 KB
        const size_t jsm = sizeof(int) * ((size_t)Mmax + 1);
        static size_t jstatic = [] {
            hipFuncAttributes fa{};
            return hipFuncGetAttributes(&fa, (const void *)featmut_jbuild<true>) == hipSuccess
                       ? fa.sharedSizeBytes : (size_t)1024;
        }();
        if (jsm + jstatic <= 64 * 1024) {
            PCR_HIP_CHECK(hipFuncSetAttribute((const void *)featmut_jbuild<true>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));
            hipLaunchKernelGGL(featmut_jbuild<true>, dim3(P), dim3(1024), jsm, s, ma);
        } else {
            hipLaunchKernelGGL(featmut_jbuild<false>, dim3(P), dim3(1024), 0, s, ma);
        }
        PCR_LAUNCH_CHECK();
        // pass 2: the rows J of G (B-role fragments as the register operand) x all F
        // columns (A-role fragments streamed): the same products, values only
        RowArgs5 r2 = r;
        r2.Ap = v.Bp; r2.Bp = v.Ap; r2.rnr = v.gnr; r2.cmax = v.fmax; r2.n_rows = n_tgt;
        r2.n_cols = n_src; r2.rlist = ma.jlist; r2.rcount = ma.nj; r2.Rmax = Mmax; r2.Cmax = Nmax;
        const int rt2 = pass_tiles(v.S, true);
        r2.ntr = ntm; r2.ntc = ntn; r2.nrb = cdiv(cdiv(Mmax, 32), v.W * rt2);
        r2.nn = nullptr; r2.v = nullptr; r2.e = nullptr; r2.list = nullptr; r2.count = nullptr;
        r2.nns = nullptr;
        r2.wq = wq;
        r2.Xr = G; r2.sc = v.mx; r2.role = 1; r2.cs = v.sp.cs;
        r2.cemax = v.femax;
        prof_begin(s, kProfFeatScreen2);
        if (one) {  // values only, 1-term; the columns whose gap it cannot use go to the 3-term
            r2.list = v.fbl21; r2.count = v.fbc21;
            RowArgs5 r2b = r2;
            r2b.rlist = v.fbl21; r2b.rcount = v.fbc21; r2b.list = nullptr; r2b.count = nullptr; r2b.fbdiag = 2;
            r2b.rbmajor = 1; r2b.csl = fsl;
            if (use9) {
                r2.rre = v.gre; r2.bcap = cap2; r2.cct = v.fct; r2.rct = v.gct;
                PCR_HIP_CHECK(hipMemsetAsync(bcnt, 0, sizeof(int) * (size_t)P * nst2, s));
                if ((rc = launch_row9<false>(r2, v.S, s)) != PCR_OK) return rc;
                prof_end(s, kProfFeatScreen2);
                RowArgs5 rg2 = r2;
                rg2.llist = nullptr; rg2.lcount = nullptr;
                if ((rc = beside(s, [&](hipStream_t q) { return launch_fallback<false>(r2b, v.S, q, kProfFeatScreen2b); },
                                 [&] { return launch_regroup9<false>(rg2, v.S, s); })) != PCR_OK)
                    return rc;
            } else {
                if ((rc = launch_row8<false, true>(r2, v.S, s)) != PCR_OK) return rc;
                prof_end(s, kProfFeatScreen2);
                if ((rc = launch_fallback<false>(r2b, v.S, s, kProfFeatScreen2b)) != PCR_OK) return rc;
            }
        } else if (v.S <= 2) {
            if ((rc = launch_row8<false, false>(r2, v.S, s)) != PCR_OK) return rc;
            prof_end(s, kProfFeatScreen2);
        } else {
            rc = launch_row7<false>(r2, v.S, s, rt2);
            if (rc != PCR_OK) return rc;
            prof_end(s, kProfFeatScreen2);
        }
        if (rs != s) PCR_HIP_CHECK(hipStreamWaitEvent(s, ev_join, 0));
        hipLaunchKernelGGL(featmut_resolve, dim3(cdiv(Nmax, 256), P), dim3(256), 0, s, ma);
        PCR_LAUNCH_CHECK();
        RescanArgs5 rb = rescan_args(F, G, n_src, n_tgt, Nmax, Mmax, D);
        rb.list12 = v.list12; rb.list21 = v.list21; rb.cnt12 = zero; rb.cnt21 = v.cnt21;
        rb.nn12 = nn12; rb.nn21 = nn21x;
        rc = run_rescan(rb, P, D, s);
        if (rc != PCR_OK) return rc;
    }
    hipLaunchKernelGGL(featmut_corres, dim3(P), dim3(1024), 0, s, ma);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

int corres_impl(const int32_t *nn12, const int32_t *nn21, const int32_t *n_src,
                const int32_t *n_tgt, int P, int Nmax, int Mmax, int mutual, int ransac_n,
                int32_t *corres, int32_t *n_corres, hipStream_t s);

int feature_corres_impl(const float *F, const float *G, int P, int Nmax, int Mmax, int D,
                        const int32_t *n_src, const int32_t *n_tgt, int mutual, int ransac_n,
                        int32_t *nn12, int32_t *corres, int32_t *n_corres, hipStream_t s) {
    PCR_REQUIRE(D >= 1 && D <= 128, PCR_ERR_ARG, "feature_corres: D=%d unsupported (1..128)", D);
    if (D <= 64)
        return feature_corres_v5(F, G, P, Nmax, Mmax, D, n_src, n_tgt, mutual, ransac_n, nn12, corres,
                                 n_corres, s);
    // 64 < D <= 128: both directions from the f32 screen, then the filter
    int32_t *nn21 = (int32_t *)workspace(34, sizeof(int32_t) * (size_t)P * Mmax + 64);
    PCR_REQUIRE(nn21, PCR_ERR_NOMEM, "feature_corres: %s", pcr_last_error());
    int rc = feature_match_f32(F, G, P, Nmax, Mmax, D, n_src, n_tgt, nn12, nn21, s);
    if (rc != PCR_OK) return rc;
    return corres_impl(nn12, nn21, n_src, n_tgt, P, Nmax, Mmax, mutual, ransac_n, corres, n_corres, s);
}

int feature_match_impl(const float *F, const float *G, int P, int Nmax, int Mmax, int D,
                       const int32_t *n_src, const int32_t *n_tgt, int32_t *nn12, int32_t *nn21,
                       hipStream_t s) {
    PCR_REQUIRE(D >= 1 && D <= 128, PCR_ERR_ARG, "feature_match: D=%d unsupported (1..128)", D);
    if (D <= 64) return feature_match_v5(F, G, P, Nmax, Mmax, D, n_src, n_tgt, nn12, nn21, s);
    return feature_match_f32(F, G, P, Nmax, Mmax, D, n_src, n_tgt, nn12, nn21, s);
}

int corres_impl(const int32_t *nn12, const int32_t *nn21, const int32_t *n_src,
                const int32_t *n_tgt, int P, int Nmax, int Mmax, int mutual, int ransac_n,
                int32_t *corres, int32_t *n_corres, hipStream_t s) {
    int *scratch = (int *)workspace(3, sizeof(int) * (size_t)P * (Nmax + 1));
    PCR_REQUIRE(scratch, PCR_ERR_NOMEM, "corres: %s", pcr_last_error());
    hipLaunchKernelGGL(corres_build, dim3(P), dim3(1024), 0, s, nn12, nn21, n_src, n_tgt, Nmax, Mmax,
                       mutual, ransac_n, scratch, corres, n_corres);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

}  // namespace pcr

extern "C" int pcr_feature_match(const float *src_feat, const float *tgt_feat, int32_t P,
                                 int32_t Nmax, int32_t Mmax, int32_t D, const int32_t *n_src,
                                 const int32_t *n_tgt, int32_t *nn12, int32_t *nn21,
                                 pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(P >= 0 && Nmax >= 0 && Mmax >= 0, PCR_ERR_ARG, "feature_match: negative size");
    if (P == 0 || Nmax == 0 || Mmax == 0) return PCR_OK;
    PCR_REQUIRE(src_feat && tgt_feat && nn12 && nn21, PCR_ERR_ARG, "feature_match: null pointer");
    PCR_REQUIRE(P <= 65535, PCR_ERR_ARG, "feature_match: P=%d > 65535", P);
    return pcr::feature_match_impl(src_feat, tgt_feat, P, Nmax, Mmax, D, n_src, n_tgt, nn12, nn21,
                                   pcr::as_stream(stream));
}

extern "C" int pcr_feature_correspondences(const float *src_feat, const float *tgt_feat, int32_t P,
                                           int32_t Nmax, int32_t Mmax, int32_t D, const int32_t *n_src,
                                           const int32_t *n_tgt, int32_t mutual_filter, int32_t ransac_n,
                                           int32_t *nn12, int32_t *corres, int32_t *n_corres,
                                           pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(P >= 0 && Nmax >= 0 && Mmax >= 0, PCR_ERR_ARG, "feature_corres: negative size");
    if (P == 0 || Nmax == 0) return PCR_OK;
    PCR_REQUIRE(src_feat && tgt_feat && nn12 && corres && n_corres, PCR_ERR_ARG,
                "feature_corres: null pointer");
    PCR_REQUIRE(P <= 65535, PCR_ERR_ARG, "feature_corres: P=%d > 65535", P);
    hipStream_t s = pcr::as_stream(stream);
    if (Mmax == 0) {  // no target: nn12 = 0 (the reference loop never runs), no mutual pair
        PCR_HIP_CHECK(hipMemsetAsync(nn12, 0, sizeof(int32_t) * (size_t)P * Nmax, s));
        int32_t *nn21 = (int32_t *)pcr::workspace(34, 64);
        PCR_REQUIRE(nn21, PCR_ERR_NOMEM, "feature_corres: %s", pcr_last_error());
        return pcr::corres_impl(nn12, nn21, n_src, n_tgt, P, Nmax, 0, mutual_filter, ransac_n, corres,
                                n_corres, s);
    }
    return pcr::feature_corres_impl(src_feat, tgt_feat, P, Nmax, Mmax, D, n_src, n_tgt, mutual_filter,
                                    ransac_n, nn12, corres, n_corres, s);
}

// debug: copy the mutual path's scratch (v12 | e12 | wq (16-B aligned) | used | pos | jlist |
// nn21x | flag | nj, feature_corres_v5's layout) of the last call to dst
extern "C" int pcr_featmut_debug_copy(void *dst, int64_t bytes, pcr_stream_t stream) {
    pcr::clear_error();
    void *src = pcr::workspace(33, 16);
    PCR_REQUIRE(src && dst && bytes >= 0, PCR_ERR_ARG, "featmut_debug_copy: bad arguments");
    PCR_HIP_CHECK(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, pcr::as_stream(stream)));
    return PCR_OK;
}

extern "C" int pcr_correspondences(const int32_t *nn12, const int32_t *nn21, int32_t P,
                                   int32_t Nmax, int32_t Mmax, const int32_t *n_src,
                                   const int32_t *n_tgt, int32_t mutual_filter, int32_t ransac_n,
                                   int32_t *corres, int32_t *n_corres, pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(P >= 0 && Nmax >= 0 && Mmax >= 0, PCR_ERR_ARG, "correspondences: negative size");
    if (P == 0) return PCR_OK;
    PCR_REQUIRE(nn12 && nn21 && corres && n_corres, PCR_ERR_ARG, "correspondences: null pointer");
    return pcr::corres_impl(nn12, nn21, n_src, n_tgt, P, Nmax, Mmax, mutual_filter, ransac_n,
                            corres, n_corres, pcr::as_stream(stream));
}

extern "C" int pcr_featnn_fallback_rows(int64_t *rows12, int64_t *cols21, int32_t reset) {
    pcr::clear_error();
    unsigned long long v[2] = {0, 0};
    PCR_HIP_CHECK(hipDeviceSynchronize());
    PCR_HIP_CHECK(hipMemcpyFromSymbol(v, HIP_SYMBOL(pcr::g_featnn_fallback_rows), sizeof(v)));
    if (rows12) *rows12 = (int64_t)v[0];
    if (cols21) *cols21 = (int64_t)v[1];
    if (reset) {
        const unsigned long long z[2] = {0, 0};
        PCR_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(pcr::g_featnn_fallback_rows), z, sizeof(z)));
    }
    return PCR_OK;
}

extern "C" int pcr_featnn_rescan_rows(int64_t *rows12, int64_t *rows21, int32_t reset) {
    pcr::clear_error();
    unsigned long long v[2] = {0, 0};
    PCR_HIP_CHECK(hipDeviceSynchronize());
    PCR_HIP_CHECK(hipMemcpyFromSymbol(v, HIP_SYMBOL(pcr::g_featnn_rescan_rows), sizeof(v)));
    if (rows12) *rows12 = (int64_t)v[0];
    if (rows21) *rows21 = (int64_t)v[1];
    if (reset) {
        const unsigned long long z[2] = {0, 0};
        PCR_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(pcr::g_featnn_rescan_rows), z, sizeof(z)));
    }
    return PCR_OK;
}
