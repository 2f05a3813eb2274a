// a5 for 64 < D <= 128: the f32 screen of the feature-space 1-NN (the D <= 64
// product shapes run the f16 x3 split screen in featnn.hip).  Same contract
// (oracle_featnn: exact f64 argmin, lowest index on ties) and the same
// certify-or-rescan structure: augmented f32 operands on v_mfma_f32_32x32x2_f32
// give both directions' distances in one launch, every uncertified row /
// column is recomputed exactly in f64 (featnn_rescan2).
#include "featnn_common.h"
#include "scan.h"

namespace pcr {
namespace {

// ---------------------------------------------------------------------------
// v3: augmented operands.  Row operand A_i = [-2 f_i, 1, |f_i|^2], column
// operand B_j = [g_j, |g_j|^2, 1] (k-step S2 carries the norms), so the MFMA
// chain (C = 0) yields the full squared distance d_ij for BOTH directions: no
// VALU adds, no per-tile global loads.  B tiles are staged into LDS with
// global_load_lds (lane-linear 256-B rows), double-buffered: the DMA of group
// k+1 flies while group k computes; one vmcnt(0) + barrier per group also
// publishes the column partials.  All LDS in one array.
// Error: every product is exact or a single rounding; |partial sums| <=
// (|f|+|g|)^2, K+3 roundings -> bound 4(K+2)u(|f|+|g|)^2 kept with the extra
// x2 margin of the certification (see featnn_screen).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void feat_pack_aug(const float *X, const int32_t *n, int Nmax,
                                                    int D, int S2a, int ntiles, int role, float *Xp,
                                                    float *nrm, unsigned *gmax) {
    // role 0: rows (A = -2x, then [1, |x|^2]); role 1: cols (B = x, then [|x|^2, 1])
    const int p = blockIdx.y, t = blockIdx.x, l = threadIdx.x;
    const int cnt = count_of(n, p, Nmax);
    const int row = t * 32 + (l & 31), h = l >> 5;
    const bool valid = row < cnt;
    const float *x = X + ((size_t)p * Nmax + (valid ? row : 0)) * D;
    double acc = 0.0;
    if (valid)
        for (int k = 0; k < D; ++k) acc = acc + (double)x[k] * (double)x[k];
    const float sq = valid ? (float)acc : __builtin_inff();
    float *dst = Xp + (((size_t)p * ntiles + t) * S2a) * 64 + l;
    for (int s = 0; s < S2a - 1; ++s) {
        const int k = 2 * s + h;
        const float v = (valid && k < D) ? x[k] : 0.0f;
        dst[(size_t)s * 64] = role == 0 ? -2.0f * v : v;
    }
    dst[(size_t)(S2a - 1) * 64] = (role == 0) ? (h == 0 ? 1.0f : sq) : (h == 0 ? sq : 1.0f);
    if (h == 0) {
        const float r = valid ? (float)__builtin_sqrt(acc) : 0.0f;
        nrm[(size_t)p * ntiles * 32 + row] = r;
        if (valid) atomicMax(gmax + p, __float_as_uint(r));
    }
}

struct DualArgs3 {
    const float *Ap, *Bp;          // augmented packed rows / cols
    const float *fnr, *gnr;        // |f|, |g|
    const unsigned *fmax, *gmax;
    const int32_t *n_src, *n_tgt;
    int Nmax, Mmax, ntn, ntm, nrb;
    int32_t *nn12;
    int *list12, *count12;
    float *cp1, *cp2;
    int *cpi;
};

template <int KCH, int G>
__global__ __launch_bounds__(512) void featnn_dual3(DualArgs3 a) {
    constexpr int S2a = 8 * KCH + 1;
    constexpr int kB = G * S2a * 64;           // floats per B buffer
    constexpr int kP = G * 8 * 32;             // entries per partial buffer
    __shared__ __attribute__((aligned(16))) float smem[2 * kB + 2 * 3 * kP];
    float *Bs = smem;                          // [2][G][S2a][64]
    float *Pc1 = smem + 2 * kB;                // [2][G][8][32]
    float *Pc2 = Pc1 + 2 * kP;
    int *Pci = reinterpret_cast<int *>(Pc2 + 2 * kP);
    const int p = blockIdx.y, rb = blockIdx.x;
    const int wid = threadIdx.x >> 6, l = threadIdx.x & 63, h = l >> 5;
    const int n = count_of(a.n_src, p, a.Nmax), m = count_of(a.n_tgt, p, a.Mmax);
    const int qt = rb * 8 + wid;
    const bool active = qt * 32 < n;
    const int ntc = (m + 31) >> 5;
    const int ngroups = (ntc + G - 1) / G;

    float A[S2a];
    const float *qp = a.Ap + (((size_t)p * a.ntn + (active ? qt : 0)) * S2a) * 64 + l;
#pragma unroll
    for (int s = 0; s < S2a; ++s) A[s] = qp[(size_t)s * 64];
    if (!active) {  // padded rows: +inf distance (A's |f|^2 slot) keeps them out
#pragma unroll
        for (int s = 0; s < S2a - 1; ++s) A[s] = 0.0f;
        A[S2a - 1] = h == 0 ? 1.0f : __builtin_inff();
    }
    float b1[16], b2[16];
    int i1[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) { b1[r] = __builtin_inff(); b2[r] = __builtin_inff(); i1[r] = 0; }

    const float *bsrc = a.Bp + ((size_t)p * a.ntm * S2a) * 64 + l;
    auto issue = [&](int grp, int bufi) {
        // G*S2a rows of 256 B; wave w issues rows w, w+8, ...
        for (int c = wid; c < G * S2a; c += 8) {
            const int g = c / S2a, srow = c - g * S2a;
            const int ct = min(grp * G + g, ntc - 1);
            const float *src = bsrc + ((size_t)ct * S2a + srow) * 64;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)src,
                (__attribute__((address_space(3))) void *)(Bs + bufi * kB + (g * S2a + srow) * 64), 4,
                0, 0);
        }
    };
    const size_t cpoff = ((size_t)p * a.nrb + rb) * (size_t)a.ntm * 32;
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int grp = 0; grp < ngroups; ++grp) {
        const int buf = grp & 1;
        if (grp + 1 < ngroups) issue(grp + 1, buf ^ 1);
        const float *Bb = Bs + buf * kB + l;
        f32x16 acc[G];
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[g][r] = 0.0f;
#pragma unroll
        for (int s = 0; s < S2a; ++s)
#pragma unroll
            for (int g = 0; g < G; ++g)
                acc[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(A[s], Bb[(g * S2a + s) * 64], acc[g], 0, 0, 0);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int ct = grp * G + g;
            const int j = ct * 32 + (l & 31);
            // column direction: 4 independent chains (q = r & 3, rows increasing
            // along each), merged with the index tie-break
            float c1[4], c2[4];
            int ci[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) { c1[q] = __builtin_inff(); c2[q] = __builtin_inff(); ci[q] = 0; }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float v = acc[g][r];
                b2[r] = __builtin_amdgcn_fmed3f(b1[r], b2[r], v);
                const bool c = v < b1[r];
                b1[r] = c ? v : b1[r];
                i1[r] = c ? j : i1[r];
                const int q = r & 3;
                c2[q] = __builtin_amdgcn_fmed3f(c1[q], c2[q], v);
                const bool cc = v < c1[q];
                c1[q] = cc ? v : c1[q];
                ci[q] = cc ? (qt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) : ci[q];
            }
            top2_merge(c1[0], ci[0], c2[0], c1[1], ci[1], c2[1]);
            top2_merge(c1[2], ci[2], c2[2], c1[3], ci[3], c2[3]);
            top2_merge(c1[0], ci[0], c2[0], c1[2], ci[2], c2[2]);
            float cc1 = c1[0], cc2 = c2[0];
            int cci = ci[0];
            const float o1 = __shfl_xor(cc1, 32, 64), o2 = __shfl_xor(cc2, 32, 64);
            const int oi = __shfl_xor(cci, 32, 64);
            top2_merge(cc1, cci, cc2, o1, oi, o2);
            if (h == 0) {
                const int e = (buf * G + g) * 256 + wid * 32 + l;
                Pc1[e] = cc1;
                Pc2[e] = cc2;
                Pci[e] = cci;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const int t = threadIdx.x;
        if (t < G * 32) {
            const int g = t >> 5, col = t & 31, ct = grp * G + g;
            if (ct < ntc) {
                const int e0 = (buf * G + g) * 256 + col;
                float m1 = Pc1[e0], m2 = Pc2[e0];
                int mi = Pci[e0];
#pragma unroll
                for (int w = 1; w < 8; ++w)
                    top2_merge(m1, mi, m2, Pc1[e0 + 32 * w], Pci[e0 + 32 * w], Pc2[e0 + 32 * w]);
                const size_t o = cpoff + (size_t)ct * 32 + col;
                a.cp1[o] = m1;
                a.cp2[o] = m2;
                a.cpi[o] = mi;
            }
        }
    }
    if (!active) return;
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
    a.nn12[(size_t)p * a.Nmax + row] = mi1;
    const double Gm = (double)__uint_as_float(a.gmax[p]);
    const double qn = (double)a.fnr[(size_t)p * a.ntn * 32 + row];
    const double K = 2.0 * S2a;
    const double bound = 4.0 * (K + 2.0) * 5.9604644775390625e-08 * (qn + Gm) * (qn + Gm);
    if (!((double)mb2 - (double)mb1 > bound)) a.list12[atomicAdd(a.count12, 1)] = p * a.Nmax + row;
}

__global__ void featnn_colmerge3(DualArgs3 a, int32_t *nn21, int *list21, int *count21, int S2a) {
    const int p = blockIdx.y;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int m = count_of(a.n_tgt, p, a.Mmax);
    if (j >= m) return;
    const int n = count_of(a.n_src, p, a.Nmax);
    const int nrb_used = (((n + 31) >> 5) + 7) >> 3;
    float b1 = __builtin_inff(), b2 = __builtin_inff();
    int i1 = 0;
    for (int rb = 0; rb < nrb_used; ++rb) {
        const size_t o = ((size_t)p * a.nrb + rb) * (size_t)a.ntm * 32 + j;
        top2_merge(b1, i1, b2, a.cp1[o], a.cpi[o], a.cp2[o]);
    }
    nn21[(size_t)p * a.Mmax + j] = i1;
    const double F = (double)__uint_as_float(a.fmax[p]);
    const double gn = (double)a.gnr[(size_t)p * a.ntm * 32 + j];
    const double K = 2.0 * S2a;
    const double bound = 4.0 * (K + 2.0) * 5.9604644775390625e-08 * (gn + F) * (gn + F);
    if (!((double)b2 - (double)b1 > bound)) list21[atomicAdd(count21, 1)] = p * a.Mmax + j;
}

// exact f64 rescan (v3/v4 modes), one 256-thread block per listed row: the
// query row is broadcast from LDS, each thread streams its candidates as
// float4 rows with two independent chains in flight; lowest index wins ties.
template <bool V4>
__global__ __launch_bounds__(256) void featnn_rescan2(const float *Q, const float *C, int Nqmax,
                                                      int Ncmax, int D, const int32_t *ncnt,
                                                      const int *list, const int *list_count,
                                                      int32_t *nn) {
    __shared__ double qs[512];
    __shared__ double wb[4];
    __shared__ int wj[4];
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const int count = *list_count;
    for (int e = blockIdx.x; e < count; e += gridDim.x) {
        const int code = list[e];
        const int p = code / Nqmax, row = code - p * Nqmax;
        const int nc = count_of(ncnt, p, Ncmax);
        const float *q = Q + ((size_t)p * Nqmax + row) * D;
        for (int k = tid; k < D; k += 256) qs[k] = (double)q[k];
        __syncthreads();
        const float *cb = C + (size_t)p * Ncmax * D;
        double best = __builtin_inf();
        int bj = 0x7fffffff;
        auto dist = [&](int j) {
            const float *c = cb + (size_t)j * D;
            double acc = 0.0;
            if (V4) {
                const float4 *c4 = reinterpret_cast<const float4 *>(c);
                for (int k = 0; k < D; k += 4) {
                    const float4 v = c4[k >> 2];
                    double df = qs[k] - (double)v.x;
                    acc = acc + df * df;
                    df = qs[k + 1] - (double)v.y;
                    acc = acc + df * df;
                    df = qs[k + 2] - (double)v.z;
                    acc = acc + df * df;
                    df = qs[k + 3] - (double)v.w;
                    acc = acc + df * df;
                }
            } else {
                for (int k = 0; k < D; ++k) {
                    const double df = qs[k] - (double)c[k];
                    acc = acc + df * df;
                }
            }
            return acc;
        };
        int j = tid;
        for (; j + 256 < nc; j += 512) {
            const double d0 = dist(j), d1 = dist(j + 256);
            if (d0 < best) { best = d0; bj = j; }
            if (d1 < best) { best = d1; bj = j + 256; }
        }
        if (j < nc) {
            const double d0 = dist(j);
            if (d0 < best) { best = d0; bj = j; }
        }
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const double ob = __shfl_xor(best, o, 64);
            const int oj = __shfl_xor(bj, o, 64);
            if (ob < best || (ob == best && oj < bj)) { best = ob; bj = oj; }
        }
        if (l == 0) { wb[w] = best; wj[w] = bj; }
        __syncthreads();
        if (tid == 0) {
            best = wb[0];
            bj = wj[0];
            for (int k = 1; k < 4; ++k)
                if (wb[k] < best || (wb[k] == best && wj[k] < bj)) { best = wb[k]; bj = wj[k]; }
            nn[(size_t)p * Nqmax + row] = (bj == 0x7fffffff) ? 0 : bj;
        }
        __syncthreads();
    }
}

}  // namespace

// exact f64 rescans of both directions' ambiguous lists
static int launch_rescans(const float *F, const float *G, int Nmax, int Mmax, int D,
                          const int32_t *n_src, const int32_t *n_tgt, const int *list12,
                          const int *list21, const int *counts, int32_t *nn12, int32_t *nn21,
                          hipStream_t s) {
    PCR_REQUIRE(D <= 512, PCR_ERR_ARG, "feature_match: D=%d > 512", D);
    const bool v4 = (D % 4) == 0 && ((uintptr_t)F & 15) == 0 && ((uintptr_t)G & 15) == 0;
    prof_begin(s, kProfFeatRescan);
    if (v4) {
        hipLaunchKernelGGL(featnn_rescan2<true>, dim3(2048), dim3(256), 0, s, F, G, Nmax, Mmax, D,
                           n_tgt, list12, counts, nn12);
        PCR_LAUNCH_CHECK();
        hipLaunchKernelGGL(featnn_rescan2<true>, dim3(2048), dim3(256), 0, s, G, F, Mmax, Nmax, D,
                           n_src, list21, counts + 1, nn21);
    } else {
        hipLaunchKernelGGL(featnn_rescan2<false>, dim3(2048), dim3(256), 0, s, F, G, Nmax, Mmax, D,
                           n_tgt, list12, counts, nn12);
        PCR_LAUNCH_CHECK();
        hipLaunchKernelGGL(featnn_rescan2<false>, dim3(2048), dim3(256), 0, s, G, F, Mmax, Nmax, D,
                           n_src, list21, counts + 1, nn21);
    }
    PCR_LAUNCH_CHECK();
    prof_end(s, kProfFeatRescan);
    return PCR_OK;
}

int feature_match_f32(const float *F, const float *G, int P, int Nmax, int Mmax, int D,
                      const int32_t *n_src, const int32_t *n_tgt, int32_t *nn12, int32_t *nn21,
                      hipStream_t s) {
    const int KCH = cdiv(D, 16);
    const int S2a = 8 * KCH + 1;
    const int ntn = cdiv(Nmax, 32), ntm = cdiv(Mmax, 32) + 8;  // +8 padded (+inf) tiles
    const size_t ap = (size_t)P * ntn * S2a * 64, bp = (size_t)P * ntm * S2a * 64;
    const size_t nn_n = (size_t)P * ntn * 32, nn_m = (size_t)P * ntm * 32;
    const size_t bytes = 4 * (ap + bp + nn_n + nn_m + 2 * (size_t)P + 2 + (size_t)P * (Nmax + Mmax));
    char *ws = (char *)workspace(2, bytes + 256);
    PCR_REQUIRE(ws, PCR_ERR_NOMEM, "feature_match: %s", pcr_last_error());
    float *Ap = (float *)ws;
    float *Bp = Ap + ap;
    float *fnr = Bp + bp;
    float *gnr = fnr + nn_n;
    unsigned *gmax = (unsigned *)(gnr + nn_m);  // [0,P): max|g|  [P,2P): max|f|
    int *list_count = (int *)(gmax + 2 * P);
    int *list = list_count + 2;
    int *list21 = list + (size_t)P * Nmax;
    PCR_HIP_CHECK(hipMemsetAsync(gmax, 0, sizeof(unsigned) * 2 * P + 2 * sizeof(int), s));
    hipLaunchKernelGGL(feat_pack_aug, dim3(ntn, P), dim3(64), 0, s, F, n_src, Nmax, D, S2a, ntn, 0,
                       Ap, fnr, gmax + P);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(feat_pack_aug, dim3(ntm, P), dim3(64), 0, s, G, n_tgt, Mmax, D, S2a, ntm, 1,
                       Bp, gnr, gmax);
    PCR_LAUNCH_CHECK();
    DualArgs3 d;
    d.Ap = Ap; d.Bp = Bp; d.fnr = fnr; d.gnr = gnr; d.fmax = gmax + P; d.gmax = gmax;
    d.n_src = n_src; d.n_tgt = n_tgt; d.Nmax = Nmax; d.Mmax = Mmax; d.ntn = ntn; d.ntm = ntm;
    d.nrb = cdiv(ntn, 8); d.nn12 = nn12; d.list12 = list; d.count12 = list_count;
    const size_t cpn = (size_t)P * d.nrb * ntm * 32;
    char *cw = (char *)workspace(11, cpn * 12 + 64);
    PCR_REQUIRE(cw, PCR_ERR_NOMEM, "feature_match: %s", pcr_last_error());
    d.cp1 = (float *)cw;
    d.cp2 = d.cp1 + cpn;
    d.cpi = (int *)(d.cp2 + cpn);
    const dim3 g(d.nrb, P);
    prof_begin(s, kProfFeatScreen);
    {
        switch (KCH) {
#define PCR_D3CASE(K, GG) \
    case K: hipLaunchKernelGGL((featnn_dual3<K, GG>), g, dim3(512), 0, s, d); break;
            PCR_D3CASE(1, 4) PCR_D3CASE(2, 4) PCR_D3CASE(3, 3) PCR_D3CASE(4, 2)
            PCR_D3CASE(5, 2) PCR_D3CASE(6, 2) PCR_D3CASE(7, 1) PCR_D3CASE(8, 1)
#undef PCR_D3CASE
            default: set_error("feature dim too large"); return PCR_ERR_ARG;
        }
    }
    PCR_LAUNCH_CHECK();
    prof_end(s, kProfFeatScreen);
    hipLaunchKernelGGL(featnn_colmerge3, dim3(cdiv(Mmax, 256), P), dim3(256), 0, s, d, nn21, list21,
                       list_count + 1, S2a);
    PCR_LAUNCH_CHECK();
    return launch_rescans(F, G, Nmax, Mmax, D, n_src, n_tgt, list, list21, list_count, nn12, nn21, s);
}

}  // namespace pcr
