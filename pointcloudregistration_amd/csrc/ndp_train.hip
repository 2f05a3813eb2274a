// f4: the fused NDP level training step -- one level's warp
// forward with saved activations, the warp backward, the weight gradients and
// the loss around the Chamfer pass -- as libpcr kernels, so an optimisation
// iteration of c2p-net/deformationpyramid/model/registration.py:208-262 is
//   ndp_train_fwd -> nnd Chamfer fwd (a1) -> ndp_chamfer_glue -> nnd Chamfer
//   bwd (a2) -> ndp_train_bwd -> ndp_wgrad -> ndp_wgrad_reduce
//   -> pcr_ndp_control -> pcr_adam_masked
// with no PyTorch autograd on the path.  Semantics: NDPLayer.forward
// (nets.py:111-140, motion SE3, rotation axis_angle, rigid_body.py:89-119) in
// f32, its gradient by the chain rule written out below, nn.Linear weight
// gradients dW = sum_p delta_p (x) a_p, bias gradients sum_p delta_p, and the
// loss of :231-244 (truncated Chamfer means + w_reg * mean BCE(s, 0)).
//
// Layouts (N points of the level):
//   activations H_l, deltas D_l, positional encoding, branch data: FEATURE-major
//   [F][N] f32 -- lane j of a wave writes point j of a 32-point tile, so every
//   save and load is a coalesced 128-byte row segment, and the weight-gradient
//   GEMMs (K = points) read contiguous rows.
//   aux [8][N]: r (3, = 1e-3 o_r), y = R x + t (3), s (nonrigidity), 0.
//   dO [8][N]: dL/d(branch pre-activation): rot (3), trn (3), nr (1), 0.
// MFMA mapping (ndp_tile.h): a 32-feature x 32-point tile is 16 accumulator
// registers, a layer a chain of exact-f32 v_mfma_f32_32x32x2_f32 whose B operand
// is the previous layer's tile; a workgroup of 4 waves owns 32 points, wave w
// feature tile w of every layer, the tiles exchanged through LDS (a 20k-point
// level runs 2,500 waves, not the 625 of one wave per 32 points).  The backward
// products use the transposed weights (A[i][k] = W[k][i], lanes read
// consecutive columns: coalesced).  Weight gradients are split-K GEMMs over
// 128-point chunks with per-chunk partials reduced in a fixed order
// (deterministic).
#include "pcr_internal.h"
#include "ndp_tile.h"
#include "ndp_ctl.h"
#include <cstdlib>

namespace pcr {
namespace {

using ndpt::chain;
using ndpt::f32x16;
using ndpt::frow;
using ndpt::publish;
using ndpt::TileX;

constexpr int kMaxHid = 4;
constexpr int kNT = 4;  // width 128: 4 feature tiles, 4 waves per workgroup

struct TrainArgs {
    const float *x;                 // (N, 3) level input
    int N, W, nhid, m, k0;          // nhid = depth - 1
    const float *w_in, *b_in;       // (W, 6), (W)
    const float *w_hid[kMaxHid], *b_hid[kMaxHid];  // (W, W), (W)
    const float *w_rot, *b_rot, *w_trn, *b_trn, *w_nr, *b_nr;
    float *pe;                      // [6][N]
    float *H;                       // [nhid + 1][W][N]: H_0 = relu(input), H_l = relu(hidden l)
    float *aux;                     // [8][N]
    float *x_out;                   // (N, 3)
    // backward
    const float *g;                 // (N, 3) dL/dx'
    double bce_scale;               // w_reg / N when the level has the nonrigidity branch, else 0
    float *dO;                      // [8][N]
    float *D;                       // [nhid + 1][W][N]: dL/d(pre-activation) of layer l
    // Chamfer subset (optional): inv[p] = k when inds[k] == p (inds unique), else -1;
    // the forward also writes x'[inds] to xs (K, 3), and the backward reads dL/dx'
    // of point p from gsub[inv[p]] (zero off the subset) instead of g
    const int32_t *inv;
    float *xs;
    const float *gsub;
    const long long *gacc;          // or: the subset gradient in 2^-44 fixed point (ndp_chamfer.hip)
    int gacc_k;                     // its K (replica stride)
    const double *gate;             // f4 early stop (pcr_internal.h), or null
};

__device__ __forceinline__ float sgn_mask(float a, float d) { return a > 0.0f ? d : 0.0f; }

// ---- forward of one level, saving what the backward needs -------------------
__global__ __launch_bounds__(64 * kNT) void ndp_train_fwd(TrainArgs a) {
    if (gated_off(a.gate)) return;
    constexpr int W = 32 * kNT;
    __shared__ TileX X[kNT];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, h = l >> 5, j = l & 31;
    const int pt = blockIdx.x * 32 + j;
    const bool valid = pt < a.N;
    const int N = a.N;
    float x0 = 0.f, x1 = 0.f, x2 = 0.f;
    if (valid) { x0 = a.x[3 * pt]; x1 = a.x[3 * pt + 1]; x2 = a.x[3 * pt + 2]; }
    const float wf = __builtin_ldexpf(1.0f, a.m + a.k0);
    float pe[3];
    {
        const float v0 = x0 * wf, v1 = x1 * wf, v2 = x2 * wf;
        pe[0] = h ? cosf(v0) : sinf(v0);
        pe[1] = h ? cosf(v1) : sinf(v1);
        pe[2] = h ? cosf(v2) : sinf(v2);
        if (valid && w == 0)
            for (int s = 0; s < 3; ++s) a.pe[(size_t)(2 * s + h) * N + pt] = pe[s];
    }
    f32x16 H;
#pragma unroll
    for (int r = 0; r < 16; ++r) H[r] = a.b_in[32 * w + frow(r, h)];
    {
        const float *wr = a.w_in + (32 * w + j) * 6;
#pragma unroll
        for (int s = 0; s < 3; ++s) H = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[2 * s + h], pe[s], H, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) H[r] = fmaxf(H[r], 0.0f);
    auto save = [&](int layer) {
        if (!valid) return;
        float *base = a.H + ((size_t)layer * W + 32 * w) * N + pt;
#pragma unroll
        for (int r = 0; r < 16; ++r) base[(size_t)frow(r, h) * N] = H[r];
    };
    save(0);
    for (int hl = 0; hl < a.nhid; ++hl) {
        publish(X[w], l, H);
        __syncthreads();
        const float *wr = a.w_hid[hl] + (size_t)(32 * w + j) * W;
        const float *bm = a.b_hid[hl];
        f32x16 Hn;
#pragma unroll
        for (int r = 0; r < 16; ++r) Hn[r] = bm[32 * w + frow(r, h)];
        Hn = chain<kNT>(X, l, [&](int it, int r) { return wr[32 * it + frow(r, h)]; }, Hn);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; ++r) H[r] = fmaxf(Hn[r], 0.0f);
        save(hl + 1);
    }
    publish(X[w], l, H);
    __syncthreads();
    if (w != 0) return;  // branch head and warp: wave 0 (no barrier follows)
    const bool has_nr = a.w_nr != nullptr;
    const float *br = j < 3 ? a.w_rot + j * W
                    : j < 6 ? a.w_trn + (j - 3) * W
                    : (j == 6 && has_nr) ? a.w_nr : nullptr;
    f32x16 Bo;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int q = frow(r, h);
        Bo[r] = q < 3 ? a.b_rot[q] : q < 6 ? a.b_trn[q - 3] : (q == 6 && has_nr) ? a.b_nr[0] : 0.0f;
    }
    Bo = chain<kNT>(X, l, [&](int it, int r) { return br ? br[32 * it + frow(r, h)] : 0.0f; }, Bo);
    const float o0 = Bo[0], o1 = Bo[1], o2 = Bo[2], o3 = Bo[3];
    const float p0 = __shfl_xor(o0, 32, 64), p1 = __shfl_xor(o1, 32, 64);
    const float p2 = __shfl_xor(o2, 32, 64), p3 = __shfl_xor(o3, 32, 64);
    const float rr0 = h ? p0 : o0, rr1 = h ? p1 : o1, rr2 = h ? p2 : o2;
    const float tt0 = h ? p3 : o3, tt1 = h ? o0 : p0, tt2 = h ? o1 : p1;
    const float nrr = h ? o2 : p2;
    const float t0 = 0.001f * tt0, t1 = 0.001f * tt1, t2 = 0.001f * tt2;
    const float r0 = 0.001f * rr0, r1 = 0.001f * rr1, r2 = 0.001f * rr2;
    const float th = sqrtf((r0 * r0 + r1 * r1) + r2 * r2);
    const float w0 = r0 / th, w1 = r1 / th, w2 = r2 / th;
    const float K[3][3] = {{0.f, -w2, w1}, {w2, 0.f, -w0}, {-w1, w0, 0.f}};
    const float sn = sinf(th), cs = 1.0f - cosf(th);
    float R[3][3];
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int v = 0; v < 3; ++v) {
            const float kk = (K[u][0] * K[0][v] + K[u][1] * K[1][v]) + K[u][2] * K[2][v];
            R[u][v] = ((u == v ? 1.0f : 0.0f) + sn * K[u][v]) + cs * kk;
        }
    const float y0 = ((R[0][0] * x0 + R[0][1] * x1) + R[0][2] * x2) + t0;
    const float y1 = ((R[1][0] * x0 + R[1][1] * x1) + R[1][2] * x2) + t1;
    const float y2 = ((R[2][0] * x0 + R[2][1] * x1) + R[2][2] * x2) + t2;
    float n0 = y0, n1 = y1, n2 = y2, s = 0.0f;
    if (has_nr) {
        s = 1.0f / (1.0f + expf(-(0.001f * nrr)));
        n0 = x0 + s * (y0 - x0);
        n1 = x1 + s * (y1 - x1);
        n2 = x2 + s * (y2 - x2);
    }
    if (valid && h == 0) {
        a.x_out[3 * pt] = n0; a.x_out[3 * pt + 1] = n1; a.x_out[3 * pt + 2] = n2;
        const float v[8] = {r0, r1, r2, y0, y1, y2, s, 0.0f};
#pragma unroll
        for (int k = 0; k < 8; ++k) a.aux[(size_t)k * N + pt] = v[k];
        if (a.xs) {
            const int k = a.inv[pt];
            if (k >= 0) { a.xs[3 * k] = n0; a.xs[3 * k + 1] = n1; a.xs[3 * k + 2] = n2; }
        }
    }
}

// ---- backward of one level: dL/dx' -> branch gradients -> layer deltas -----
__global__ __launch_bounds__(64 * kNT) void ndp_train_bwd(TrainArgs a) {
    if (gated_off(a.gate)) return;
    constexpr int W = 32 * kNT;
    __shared__ TileX X[kNT];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, h = l >> 5, j = l & 31;
    const int pt = blockIdx.x * 32 + j;
    const bool valid = pt < a.N;
    const int N = a.N;
    const bool has_nr = a.w_nr != nullptr;
    // per-point branch gradients: computed once per workgroup by wave 0 (its two
    // half-waves split the gradient replicas) and broadcast through LDS to the
    // four waves (each had recomputed them, 96 gradient words per lane)
    __shared__ float sdO[8][32];
    float dO[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (w == 0) {
        const float x[3] = {valid ? a.x[3 * pt] : 0.f, valid ? a.x[3 * pt + 1] : 0.f, valid ? a.x[3 * pt + 2] : 0.f};
        float g[3] = {0.f, 0.f, 0.f};
        if (a.inv && a.gacc) {
            // the two-word fixed point of ndp_chamfer.hip: header word = flag bit 0,
            // (s + 2048) << 8; hi words at 2^-s, lo words (after all hi) at 2^-(s+40);
            // half h sums replicas h, h + 2, ... (integer sums: exact, any order)
            const int k = valid ? a.inv[pt] : -1;
            const long long hw = a.gacc[0];
            const float bad = (hw & 1) ? __builtin_nanf("") : 0.0f;
            int sh = (int)(hw >> 8) - 2048;
            if (sh >= 1000) sh -= 1000;  // diagnostics: hi words only (PCR_NDP_FIXSHIFT)
            const size_t lo = (size_t)3 * PCR_NDP_GACC_REPLICAS * a.gacc_k;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                long long vh = 0, vl = 0;
                if (k >= 0)
#pragma unroll
                    for (int r = h; r < PCR_NDP_GACC_REPLICAS; r += 2) {
                        const size_t o = 1 + 3 * ((size_t)r * a.gacc_k + k) + c;
                        vh += a.gacc[o];
                        vl += a.gacc[o + lo];
                    }
                vh += __shfl_xor(vh, 32, 64);
                vl += __shfl_xor(vl, 32, 64);
                const double v = __builtin_ldexp((double)vh, -sh) + __builtin_ldexp((double)vl, -sh - 40);
                g[c] = k >= 0 ? (float)v + bad : 0.0f;
            }
        } else if (!valid) {
        } else if (a.inv) {
            const int k = a.inv[pt];
            g[0] = k >= 0 ? a.gsub[3 * k] : 0.0f;
            g[1] = k >= 0 ? a.gsub[3 * k + 1] : 0.0f;
            g[2] = k >= 0 ? a.gsub[3 * k + 2] : 0.0f;
        } else {
            g[0] = a.g[3 * pt]; g[1] = a.g[3 * pt + 1]; g[2] = a.g[3 * pt + 2];
        }
        float aux[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) aux[k] = valid ? a.aux[(size_t)k * N + pt] : 0.f;
        const float r0 = aux[0], r1 = aux[1], r2 = aux[2];
        const float y[3] = {aux[3], aux[4], aux[5]};
        if (has_nr) {
            // x' = x + s (y - x), s = sigmoid(1e-3 o_n); BCE(s, 0) = -log(1 - s), mean
            const float s = aux[6];
            const float ds = ((g[0] * (y[0] - x[0]) + g[1] * (y[1] - x[1])) + g[2] * (y[2] - x[2])) +
                             (float)a.bce_scale / (1.0f - s);
            dO[6] = 0.001f * (ds * (s * (1.0f - s)));
            g[0] *= s; g[1] *= s; g[2] *= s;
        }
        // y = R x + t
        dO[3] = 0.001f * g[0]; dO[4] = 0.001f * g[1]; dO[5] = 0.001f * g[2];
        const float th = sqrtf((r0 * r0 + r1 * r1) + r2 * r2);
        const float w[3] = {r0 / th, r1 / th, r2 / th};
        const float K[3][3] = {{0.f, -w[2], w[1]}, {w[2], 0.f, -w[0]}, {-w[1], w[0], 0.f}};
        const float sn = sinf(th), cs0 = cosf(th), cs = 1.0f - cs0;
        float G[3][3], KK[3][3];
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
            for (int v = 0; v < 3; ++v) {
                G[u][v] = g[u] * x[v];
                KK[u][v] = (K[u][0] * K[0][v] + K[u][1] * K[1][v]) + K[u][2] * K[2][v];
            }
        // R = I + sin(th) K + (1 - cos(th)) K^2
        float dth = 0.0f;
        float dK[3][3];
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
            for (int v = 0; v < 3; ++v) {
                dth += G[u][v] * (cs0 * K[u][v] + sn * KK[u][v]);
                // d<G, K K>/dK = G K^T + K^T G
                float gkt = 0.0f, ktg = 0.0f;
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    gkt += G[u][q] * K[v][q];
                    ktg += K[q][u] * G[q][v];
                }
                dK[u][v] = sn * G[u][v] + cs * (gkt + ktg);
            }
        const float gw[3] = {dK[2][1] - dK[1][2], dK[0][2] - dK[2][0], dK[1][0] - dK[0][1]};
        const float gww = (gw[0] * w[0] + gw[1] * w[1]) + gw[2] * w[2];
#pragma unroll
        for (int c = 0; c < 3; ++c) dO[c] = 0.001f * ((gw[c] - gww * w[c]) / th + dth * w[c]);
        if (!valid)
#pragma unroll
            for (int k = 0; k < 8; ++k) dO[k] = 0.0f;
        if (h == 0) {  // (w is the rotation axis here)
#pragma unroll
            for (int k = 0; k < 8; ++k) sdO[k][j] = dO[k];
            if (valid)
                for (int k = 0; k < 8; ++k) a.dO[(size_t)k * N + pt] = dO[k];
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) dO[k] = sdO[k][j];
    // delta of the last hidden activation: W_b^T dO (K = 8 branch rows, 4 k-steps)
    const int L = a.nhid;
    auto load_act = [&](int layer, int r) -> float {
        return valid ? a.H[((size_t)layer * W + 32 * w + frow(r, h)) * N + pt] : 0.0f;
    };
    auto branch_w = [&](int q, int col) -> float {  // W_b[q][col], q = branch row 0..7
        if (q < 3) return a.w_rot[q * W + col];
        if (q < 6) return a.w_trn[(q - 3) * W + col];
        if (q == 6 && has_nr) return a.w_nr[col];
        return 0.0f;
    };
    f32x16 Dt;
#pragma unroll
    for (int r = 0; r < 16; ++r) Dt[r] = 0.0f;
#pragma unroll
    for (int s = 0; s < 4; ++s)  // k = 2s + h: B[k][j] = dO[k] of point j
        Dt = __builtin_amdgcn_mfma_f32_32x32x2f32(branch_w(2 * s + h, 32 * w + j),
                                                  h ? dO[2 * s + 1] : dO[2 * s], Dt, 0, 0, 0);
    // rows of the transposed product: A[i][k] = W[k][i] -> lane j gives W[k][32 w + j]
    for (int layer = L; layer >= 0; --layer) {
        // mask by the layer's ReLU: delta of the pre-activation
#pragma unroll
        for (int r = 0; r < 16; ++r) Dt[r] = sgn_mask(load_act(layer, r), Dt[r]);
        if (valid) {
            float *base = a.D + ((size_t)layer * W + 32 * w) * N + pt;
#pragma unroll
            for (int r = 0; r < 16; ++r) base[(size_t)frow(r, h) * N] = Dt[r];
        }
        if (layer == 0) break;
        publish(X[w], l, Dt);
        __syncthreads();
        const float *Wm = a.w_hid[layer - 1];  // layer l = relu(W_{l-1} H_{l-1} + b)
        f32x16 Dn;
#pragma unroll
        for (int r = 0; r < 16; ++r) Dn[r] = 0.0f;
        Dn = chain<kNT>(X, l, [&](int it, int r) {
            return Wm[(size_t)(32 * it + frow(r, h)) * W + 32 * w + j]; }, Dn);
        __syncthreads();
        Dt = Dn;
    }
}

// ---- weight gradients: dW[o][i] = sum_p D[o][p] X[i][p] (split-K) ------------
struct WgradJob {
    const float *D;   // [FO][N]
    const float *X;   // [FI][N]
    int FO, FI;       // actual rows (<= 128)
    float *part;      // [nchunk][FO][FI] then [nchunk][FO] bias partials
};
struct WgradArgs {
    WgradJob job[8];
    int N, chunk;     // points per chunk (multiple of 64)
    const double *gate;
};

constexpr int kWgT = 64;  // points per LDS stage

// 16 waves: wave t owns output tile t of the job (a 128 x 128 weight is 4 x 4
// tiles); the chains and the bias sums keep their point order
__global__ __launch_bounds__(1024) void ndp_wgrad(WgradArgs a) {
    if (gated_off(a.gate)) return;
    __shared__ float Ds[128][kWgT + 1], Xs[128][kWgT + 1];
    const WgradJob jb = a.job[blockIdx.y];
    const int c = blockIdx.x, nchunk = gridDim.x;
    const int p0 = c * a.chunk, p1 = min(a.N, p0 + a.chunk);
    const int tid = threadIdx.x, wid = tid >> 6, l = tid & 63, h = l >> 5, jj = l & 31;
    const int nti = (jb.FI + 31) >> 5, ntile = ((jb.FO + 31) >> 5) * nti;
    const bool own = wid < ntile;
    const int to = own ? wid / nti : 0, ti = own ? wid - to * nti : 0;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
    float bsum = 0.0f;  // bias partial of output row tid (tid < FO)
    for (int pb = p0; pb < p1; pb += kWgT) {
        const int np = min(kWgT, p1 - pb);
        __syncthreads();
        for (int e = tid; e < 128 * kWgT; e += 1024) {
            const int row = e / kWgT, col = e - row * kWgT;
            const bool in = col < np;
            Ds[row][col] = (row < jb.FO && in) ? jb.D[(size_t)row * a.N + pb + col] : 0.0f;
            Xs[row][col] = (row < jb.FI && in) ? jb.X[(size_t)row * a.N + pb + col] : 0.0f;
        }
        __syncthreads();
        if (tid < jb.FO) {
#pragma unroll 8
            for (int k = 0; k < np; ++k) bsum += Ds[tid][k];
        }
        if (own)
            for (int s = 0; s < kWgT / 2; ++s) {
                const int k = 2 * s + h;
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Ds[32 * to + jj][k], Xs[32 * ti + jj][k], acc,
                                                           0, 0, 0);
            }
    }
    // D[o][i]: lane (jj, h) holds rows frow(r, h) of column jj
    if (own) {
        const int col = 32 * ti + jj;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = 32 * to + frow(r, h);
            if (row < jb.FO && col < jb.FI)
                jb.part[((size_t)c * jb.FO + row) * jb.FI + col] = acc[r];
        }
    }
    if (tid < jb.FO)
        jb.part[(size_t)nchunk * jb.FO * jb.FI + (size_t)c * jb.FO + tid] = bsum;
}

struct ReduceJob {
    const float *part;
    int FO, FI;
    float *gw, *gb;   // [FO][FI], [FO]
};
struct ReduceArgs {
    ReduceJob job[8];
    int nchunk;
    const double *gate;
};

// four lanes per output element: lane q sums the chunks c = q (mod 4) in chunk
// order, then the four sums are combined as (s0 + s1) + (s2 + s3) by two xor
// shuffles (f32 addition commutes exactly, so every lane holds the same bits):
// a fixed order, four times the loads in flight of one lane per element (the
// single-lane loop was a chain of ~20 dependent load batches per element)
__global__ __launch_bounds__(256) void ndp_wgrad_reduce(ReduceArgs a) {
    if (gated_off(a.gate)) return;
    const ReduceJob jb = a.job[blockIdx.y];
    const int e = blockIdx.x * 64 + (threadIdx.x >> 2), q = threadIdx.x & 3;
    const int nw = jb.FO * jb.FI;
    const float *src = nullptr;
    size_t stride = 0;
    if (e < nw) {
        src = jb.part + e;
        stride = (size_t)nw;
    } else if (e < nw + jb.FO) {
        src = jb.part + (size_t)a.nchunk * nw + (e - nw);
        stride = (size_t)jb.FO;
    }
    float s = 0.0f;
    if (src) {
#pragma unroll 8
        for (int c = q; c < a.nchunk; c += 4) s += src[(size_t)c * stride];
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (q != 0 || !src) return;
    if (e < nw) jb.gw[e] = s;
    else jb.gb[e - nw] = s;
}

// ---- the level loss around the Chamfer pass (registration.py:231-244): the
// truncated Chamfer means with their gradients dL/dd1 = 1/K, dL/dd2 = 1/M
// (0 where truncated), + w_reg * mean(-max(log(1 - s), -100)), and the loss
// log entry; one workgroup, fixed reduction order ------------------------------
struct GlueArgs {
    const float *d1, *d2, *s;  // (K), (M), nonrigidity (N) or null (no BCE term)
    int K, M, N, log_last;
    float trunc, w_reg, g1, g2;
    float *gd1, *gd2, *loss, *log;
    long long *ctr;
    const double *gate = nullptr;
};

__global__ __launch_bounds__(1024) void ndp_chamfer_glue(GlueArgs a) {
    if (gated_off(a.gate)) return;
    __shared__ float red[3][16];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    float s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
    for (int i = t; i < a.K; i += 1024) {
        const float d = a.d1[i];
        const bool in = !(d >= a.trunc);  // torch.where(d >= trunc, 0, d): NaN stays
        s1 += in ? d : 0.0f;
        if (a.gd1) a.gd1[i] = in ? a.g1 : 0.0f;
    }
    for (int i = t; i < a.M; i += 1024) {
        const float d = a.d2[i];
        const bool in = !(d >= a.trunc);
        s2 += in ? d : 0.0f;
        if (a.gd2) a.gd2[i] = in ? a.g2 : 0.0f;
    }
    if (a.s)
        for (int i = t; i < a.N; i += 1024) {
            const float v = logf(1.0f - a.s[i]);
            s3 += v < -100.0f ? -100.0f : v;  // clamp(min=-100), NaN stays
        }
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        s1 += __shfl_xor(s1, o, 64);
        s2 += __shfl_xor(s2, o, 64);
        s3 += __shfl_xor(s3, o, 64);
    }
    if (lane == 0) { red[0][wv] = s1; red[1][wv] = s2; red[2][wv] = s3; }
    __syncthreads();
    if (t != 0) return;
    float S1 = 0.0f, S2 = 0.0f, S3 = 0.0f;
    for (int w = 0; w < 16; ++w) { S1 += red[0][w]; S2 += red[1][w]; S3 += red[2][w]; }
    float L = S1 / (float)a.K + S2 / (float)a.M;
    if (a.s) L = L + a.w_reg * (-S3 / (float)a.N);
    *a.loss = L;
    const long long c = *a.ctr;
    a.log[c < a.log_last ? c : a.log_last] = L;
    *a.ctr = c + 1;
}

// ---- the same loss over kLossBlocks workgroups (fixed index ranges, partials
// summed in block order by the last block to finish), with the early-stop rule
// applied by that block: one launch for the glue and pcr_ndp_control ----------
constexpr int kLossBlocks = 32;

struct LossArgs {
    GlueArgs g;
    double *state;  // or null (no rule)
    double ratio, stop_loss;
    int max_break;
    float *part;    // [3][kLossBlocks]
    unsigned *done; // zero between launches (the last block resets it)
};

__global__ __launch_bounds__(256) void ndp_loss_kernel(LossArgs a) {
    const GlueArgs &g = a.g;
    if (gated_off(g.gate)) return;
    __shared__ float red[3][4];
    __shared__ bool last;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6, b = blockIdx.x;
    auto range = [&](int n, int &lo, int &hi) {
        const int per = (n + kLossBlocks - 1) / kLossBlocks;
        lo = min(n, b * per);
        hi = min(n, lo + per);
    };
    float s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
    int lo, hi;
    range(g.K, lo, hi);
    for (int i = lo + t; i < hi; i += 256) {
        const float d = g.d1[i];
        s1 += !(d >= g.trunc) ? d : 0.0f;  // torch.where(d >= trunc, 0, d): NaN stays
    }
    range(g.M, lo, hi);
    for (int i = lo + t; i < hi; i += 256) {
        const float d = g.d2[i];
        s2 += !(d >= g.trunc) ? d : 0.0f;
    }
    if (g.s) {
        range(g.N, lo, hi);
        for (int i = lo + t; i < hi; i += 256) {
            const float v = logf(1.0f - g.s[i]);
            s3 += v < -100.0f ? -100.0f : v;  // clamp(min=-100), NaN stays
        }
    }
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        s1 += __shfl_xor(s1, o, 64);
        s2 += __shfl_xor(s2, o, 64);
        s3 += __shfl_xor(s3, o, 64);
    }
    if (lane == 0) { red[0][wv] = s1; red[1][wv] = s2; red[2][wv] = s3; }
    __syncthreads();
    if (t == 0) {
        a.part[b] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
        a.part[kLossBlocks + b] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
        a.part[2 * kLossBlocks + b] = ((red[2][0] + red[2][1]) + red[2][2]) + red[2][3];
        __threadfence();
        last = atomicAdd(a.done, 1u) == kLossBlocks - 1;
    }
    __syncthreads();
    if (!last || t != 0) return;
    __threadfence();
    float S1 = 0.0f, S2 = 0.0f, S3 = 0.0f;
    for (int k = 0; k < kLossBlocks; ++k) {
        S1 += __hip_atomic_load(a.part + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        S2 += __hip_atomic_load(a.part + kLossBlocks + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        S3 += __hip_atomic_load(a.part + 2 * kLossBlocks + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    float L = S1 / (float)g.K + S2 / (float)g.M;
    if (g.s) L = L + g.w_reg * (-S3 / (float)g.N);
    *g.loss = L;
    const long long c = *g.ctr;
    g.log[c < g.log_last ? c : g.log_last] = L;
    *g.ctr = c + 1;
    *a.done = 0;
    if (a.state) ndp_control_rule(L, a.state, a.ratio, a.max_break, a.stop_loss);
}

}  // namespace
}  // namespace pcr

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
static int fill_train(const pcr_ndp_train *t, pcr::TrainArgs &a) {
    PCR_REQUIRE(t, PCR_ERR_ARG, "ndp_train: null descriptor");
    PCR_REQUIRE(t->N >= 0 && t->width == 128, PCR_ERR_ARG, "ndp_train: width %d (only 128)", t->width);
    PCR_REQUIRE(t->depth >= 1 && t->depth - 1 <= pcr::kMaxHid, PCR_ERR_ARG, "ndp_train: depth %d", t->depth);
    const pcr_ndp_level &L = t->level;
    PCR_REQUIRE(L.w_in && L.b_in && L.w_rot && L.b_rot && L.w_trn && L.b_trn && (!L.w_nr || L.b_nr),
                PCR_ERR_ARG, "ndp_train: null weight");
    a = pcr::TrainArgs{};
    a.x = t->x; a.N = t->N; a.W = t->width; a.nhid = t->depth - 1; a.m = L.m; a.k0 = t->k0;
    a.w_in = L.w_in; a.b_in = L.b_in;
    for (int k = 0; k < a.nhid; ++k) {
        PCR_REQUIRE(t->w_hid[k] && t->b_hid[k], PCR_ERR_ARG, "ndp_train: null hidden layer %d", k);
        a.w_hid[k] = t->w_hid[k];
        a.b_hid[k] = t->b_hid[k];
    }
    a.w_rot = L.w_rot; a.b_rot = L.b_rot; a.w_trn = L.w_trn; a.b_trn = L.b_trn;
    a.w_nr = L.w_nr; a.b_nr = L.b_nr;
    a.pe = t->pe; a.H = t->H; a.aux = t->aux; a.x_out = t->x_out;
    a.g = t->g; a.bce_scale = t->bce_scale; a.dO = t->dO; a.D = t->D;
    a.inv = t->inv; a.xs = t->xs; a.gsub = t->gsub; a.gacc = t->gacc; a.gacc_k = t->gacc_k;
    a.gate = pcr::current_gate();
    return PCR_OK;
}

extern "C" int pcr_ndp_train_forward(const pcr_ndp_train *t, pcr_stream_t stream) {
    pcr::clear_error();
    pcr::TrainArgs a;
    int rc = fill_train(t, a);
    if (rc != PCR_OK) return rc;
    if (a.N == 0) return PCR_OK;
    PCR_REQUIRE(a.x && a.pe && a.H && a.aux && a.x_out, PCR_ERR_ARG, "ndp_train_forward: null buffer");
    PCR_REQUIRE(!a.xs || a.inv, PCR_ERR_ARG, "ndp_train_forward: xs without inv");
    hipLaunchKernelGGL(pcr::ndp_train_fwd, dim3((a.N + 31) / 32), dim3(64 * pcr::kNT), 0,
                       pcr::as_stream(stream), a);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

extern "C" int pcr_ndp_train_backward(const pcr_ndp_train *t, float *part, int32_t chunk,
                                      float *const *grads, pcr_stream_t stream) {
    pcr::clear_error();
    pcr::TrainArgs a;
    int rc = fill_train(t, a);
    if (rc != PCR_OK) return rc;
    if (a.N == 0) return PCR_OK;
    PCR_REQUIRE((a.inv ? (a.gsub != nullptr || a.gacc != nullptr) : a.g != nullptr) && a.dO && a.D && part && grads, PCR_ERR_ARG,
                "ndp_train_backward: null buffer");
    PCR_REQUIRE(chunk >= 64 && chunk % 64 == 0, PCR_ERR_ARG, "ndp_train_backward: chunk %d", chunk);
    hipStream_t s = pcr::as_stream(stream);
    hipLaunchKernelGGL(pcr::ndp_train_bwd, dim3((a.N + 31) / 32), dim3(64 * pcr::kNT), 0, s, a);
    PCR_LAUNCH_CHECK();
    // jobs: input layer (W x 6 over pe), hidden layers, branches (7 x W over H_last)
    const int W = a.W, N = a.N, nchunk = (N + chunk - 1) / chunk;
    pcr::WgradArgs wa{};
    pcr::ReduceArgs ra{};
    wa.N = N; wa.chunk = chunk; ra.nchunk = nchunk;
    wa.gate = a.gate; ra.gate = a.gate;
    int nj = 0;
    size_t off = 0;
    auto add = [&](const float *D, const float *X, int FO, int FI, float *gw, float *gb) {
        wa.job[nj] = pcr::WgradJob{D, X, FO, FI, part + off};
        ra.job[nj] = pcr::ReduceJob{part + off, FO, FI, gw, gb};
        off += (size_t)nchunk * ((size_t)FO * FI + FO);
        ++nj;
    };
    // grads: [0] w_in [1] b_in, then per hidden layer (w, b), then w_branch (8 x W rows
    // rot 0-2, trn 3-5, nr 6), b_branch (8)
    add(a.D, a.pe, W, 6, grads[0], grads[1]);
    for (int k = 0; k < a.nhid; ++k)
        add(a.D + (size_t)(k + 1) * W * N, a.H + (size_t)k * W * N, W, W, grads[2 + 2 * k],
            grads[3 + 2 * k]);
    add(a.dO, a.H + (size_t)a.nhid * W * N, 7, W, grads[2 + 2 * a.nhid], grads[3 + 2 * a.nhid]);
    hipLaunchKernelGGL(pcr::ndp_wgrad, dim3(nchunk, nj), dim3(1024), 0, s, wa);
    PCR_LAUNCH_CHECK();
    hipLaunchKernelGGL(pcr::ndp_wgrad_reduce, dim3((W * W + W + 63) / 64, nj), dim3(256), 0, s, ra);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

extern "C" int64_t pcr_ndp_train_partial_floats(int32_t N, int32_t width, int32_t depth, int32_t chunk) {
    if (N <= 0 || chunk <= 0) return 0;
    const int64_t nchunk = (N + chunk - 1) / chunk, W = width;
    return nchunk * ((W * 6 + W) + (int64_t)(depth - 1) * (W * W + W) + (7 * W + 7));
}

extern "C" int pcr_ndp_chamfer_glue(const float *d1, int32_t K, const float *d2, int32_t M,
                                    const float *s, int32_t N, double w_reg, double trunc,
                                    float *gd1, float *gd2, float *loss, float *log, int64_t *ctr,
                                    int32_t log_last, pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(K >= 0 && M >= 0 && N >= 0 && log_last >= 0, PCR_ERR_ARG, "ndp_chamfer_glue: negative size");
    PCR_REQUIRE((K == 0 || d1) && (M == 0 || d2) && loss && log && ctr, PCR_ERR_ARG,
                "ndp_chamfer_glue: null buffer");
    pcr::GlueArgs g{d1, d2, s, K, M, N, log_last, (float)trunc, (float)w_reg,
                    (float)(1.0 / (double)K), (float)(1.0 / (double)M), gd1, gd2, loss, log,
                    (long long *)ctr};
    g.gate = pcr::current_gate();
    hipLaunchKernelGGL(pcr::ndp_chamfer_glue, dim3(1), dim3(1024), 0, pcr::as_stream(stream), g);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

extern "C" int64_t pcr_ndp_loss_scratch_bytes(void) {
    return (int64_t)(sizeof(float) * 3 * pcr::kLossBlocks + 64);
}

extern "C" int pcr_ndp_chamfer_loss(const float *d1, int32_t K, const float *d2, int32_t M, const float *s,
                                    int32_t N, double w_reg, double trunc, float *loss, float *log,
                                    int64_t *ctr, int32_t log_last, double *state, double break_threshold_ratio,
                                    int32_t max_break_count, double stop_loss, void *scratch,
                                    pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(K >= 1 && M >= 1 && N >= 0 && log_last >= 0, PCR_ERR_ARG, "ndp_chamfer_loss: bad size");
    PCR_REQUIRE(d1 && d2 && loss && log && ctr && scratch, PCR_ERR_ARG, "ndp_chamfer_loss: null buffer");
    pcr::LossArgs a;
    a.g = pcr::GlueArgs{d1, d2, s, K, M, N, log_last, (float)trunc, (float)w_reg,
                        (float)(1.0 / (double)K), (float)(1.0 / (double)M), nullptr, nullptr, loss, log,
                        (long long *)ctr};
    a.g.gate = pcr::current_gate();
    a.state = state;
    a.ratio = break_threshold_ratio;
    a.stop_loss = stop_loss;
    a.max_break = max_break_count;
    a.part = (float *)scratch;
    a.done = (unsigned *)(a.part + 3 * pcr::kLossBlocks);
    hipLaunchKernelGGL(pcr::ndp_loss_kernel, dim3(pcr::kLossBlocks), dim3(256), 0, pcr::as_stream(stream), a);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}
