// a10: NDP deformation-pyramid warp, all levels fused in one launch
// (c2p-net/deformationpyramid/model/nets.py: Deformation_Pyramid.warp :36-48,
// NDPLayer.forward :111-140, posenc :164-177, get_Rotation axis_angle :144-161
// -> rigid_body.exp_so3/skew :89-95,:113-119, MLP :295-304; SE3 motion).
//
// Per level, for every point: pe = [sin wx, cos wx, sin wy, cos wy, sin wz,
// cos wz] (w = 2^(m+k0)), h = ReLU(W_in pe + b), depth-1 x h = ReLU(W h + b),
// r = 1e-3 (W_rot h + b), t = 1e-3 (W_trn h + b), R = exp_so3(r/|r|, |r|),
// x' = R x + t, and with a nonrigidity branch x' = x + s (x' - x),
// s = sigmoid(1e-3 (W_nr h + b)).  f32 throughout, as the reference.
//
// MI355X design: a workgroup of NT = width/32 waves owns 32 points across all
// levels, wave w computing feature tile w of every layer.  Every layer is a
// chain of exact-f32 v_mfma_f32_32x32x2_f32: the activation tile H (32 features
// x 32 points, features in the 16 accumulator registers, points on lanes) is
// the B operand of the next layer directly -- k-step r of input tile it takes
// the feature row (r&3) + 8(r>>2) + 4(lane>>5) that the lane already holds, and
// the A operand (weights) is read in that permuted k order; the other waves'
// tiles arrive through LDS in that layout (ndp_tile.h), in the chain order of
// one wave holding all tiles, so the split changes no bits while a 20k-point
// cloud runs NT x 625 waves.  Wave 0 runs the branch head and the warp and
// hands the new points to the others through LDS.  Biases seed the
// accumulators.  The weights (nn.Linear layout, ~140 KB per level at width
// 128) stream through L1/L2; a lane's 16 k-steps of one 32-column block share
// one 128-byte line.
#include "pcr_internal.h"
#include "ndp_tile.h"

namespace pcr {
namespace {

using ndpt::chain;
using ndpt::f32x16;
using ndpt::frow;
using ndpt::publish;
using ndpt::TileX;

constexpr int kMaxLevels = 16;

struct NdpLevelDev {
    const float *w_in, *b_in, *w_hid, *b_hid, *w_rot, *b_rot, *w_trn, *b_trn, *w_nr, *b_nr;
    int m;
};

struct NdpArgs {
    const float *x;
    int N, nlev, depth, k0;
    float *x_out, *x_levels, *nonrig;
    NdpLevelDev lv[kMaxLevels];
};

template <int NT>
__global__ __launch_bounds__(64 * NT) void ndp_warp_kernel(NdpArgs a) {
    constexpr int W = 32 * NT;
    __shared__ TileX X[NT];
    __shared__ float xn[3][32];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, h = l >> 5, j = l & 31;
    const int pt = blockIdx.x * 32 + j;
    const bool valid = pt < a.N;
    float x0 = 0.f, x1 = 0.f, x2 = 0.f;
    if (valid) { x0 = a.x[3 * pt]; x1 = a.x[3 * pt + 1]; x2 = a.x[3 * pt + 2]; }
    for (int lv = 0; lv < a.nlev; ++lv) {
        const NdpLevelDev &L = a.lv[lv];
        const float wf = __builtin_ldexpf(1.0f, L.m + a.k0);
        // positional encoding as the input layer's B operand: k = 2s + h
        float pe[3];
        {
            const float v0 = x0 * wf, v1 = x1 * wf, v2 = x2 * wf;
            pe[0] = h ? cosf(v0) : sinf(v0);
            pe[1] = h ? cosf(v1) : sinf(v1);
            pe[2] = h ? cosf(v2) : sinf(v2);
        }
        f32x16 H;
#pragma unroll
        for (int r = 0; r < 16; ++r) H[r] = L.b_in[32 * w + frow(r, h)];
        {
            const float *wr = L.w_in + (32 * w + j) * 6;
#pragma unroll
            for (int s = 0; s < 3; ++s) H = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[2 * s + h], pe[s], H, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) H[r] = fmaxf(H[r], 0.0f);
        for (int hl = 0; hl + 1 < a.depth; ++hl) {
            publish(X[w], l, H);
            __syncthreads();
            const float *wr = L.w_hid + (size_t)hl * W * W + (size_t)(32 * w + j) * W;
            const float *bm = L.b_hid + (size_t)hl * W;
            f32x16 Hn;
#pragma unroll
            for (int r = 0; r < 16; ++r) Hn[r] = bm[32 * w + frow(r, h)];
            Hn = chain<NT>(X, l, [&](int it, int r) { return wr[32 * it + frow(r, h)]; }, Hn);
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 16; ++r) H[r] = fmaxf(Hn[r], 0.0f);
        }
        publish(X[w], l, H);
        __syncthreads();
        if (w == 0) {
            // branches in one 32-row tile: rows 0-2 rotation, 3-5 translation, 6 nonrigidity
            const bool has_nr = L.w_nr != nullptr;
            const float *br = j < 3 ? L.w_rot + j * W
                            : j < 6 ? L.w_trn + (j - 3) * W
                            : (j == 6 && has_nr) ? L.w_nr : nullptr;
            f32x16 Bo;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int q = frow(r, h);
                Bo[r] = q < 3 ? L.b_rot[q] : q < 6 ? L.b_trn[q - 3] : (q == 6 && has_nr) ? L.b_nr[0] : 0.0f;
            }
            Bo = chain<NT>(X, l, [&](int it, int r) { return br ? br[32 * it + frow(r, h)] : 0.0f; }, Bo);
            // rows 0-3 sit in registers 0-3 of the h=0 half, rows 4-7 in the h=1 half
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
            // K = skew(w): [[0,-w2,w1],[w2,0,-w0],[-w1,w0,0]]
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
            float n0 = ((R[0][0] * x0 + R[0][1] * x1) + R[0][2] * x2) + t0;
            float n1 = ((R[1][0] * x0 + R[1][1] * x1) + R[1][2] * x2) + t1;
            float n2 = ((R[2][0] * x0 + R[2][1] * x1) + R[2][2] * x2) + t2;
            float sg = 0.0f;
            if (has_nr) {
                sg = 1.0f / (1.0f + expf(-(0.001f * nrr)));
                n0 = x0 + sg * (n0 - x0);
                n1 = x1 + sg * (n1 - x1);
                n2 = x2 + sg * (n2 - x2);
            }
            if (h == 0) {
                xn[0][j] = n0; xn[1][j] = n1; xn[2][j] = n2;
                if (valid) {
                    if (a.x_levels) {
                        float *o = a.x_levels + ((size_t)lv * a.N + pt) * 3;
                        o[0] = n0; o[1] = n1; o[2] = n2;
                    }
                    if (a.nonrig && has_nr) a.nonrig[(size_t)lv * a.N + pt] = sg;
                }
            }
        }
        __syncthreads();
        x0 = xn[0][j]; x1 = xn[1][j]; x2 = xn[2][j];
    }
    if (valid && h == 0 && w == 0) {
        a.x_out[3 * pt] = x0;
        a.x_out[3 * pt + 1] = x1;
        a.x_out[3 * pt + 2] = x2;
    }
}

}  // namespace
}  // namespace pcr

extern "C" int pcr_ndp_warp(const float *x, int32_t N, const pcr_ndp_level *levels,
                            int32_t n_levels, int32_t width, int32_t depth, int32_t k0,
                            float *x_out, float *x_levels, float *nonrigidity,
                            pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(N >= 0 && n_levels >= 0, PCR_ERR_ARG, "ndp_warp: negative size");
    PCR_REQUIRE(n_levels <= pcr::kMaxLevels, PCR_ERR_ARG, "ndp_warp: %d levels > %d", n_levels,
                pcr::kMaxLevels);
    PCR_REQUIRE(width == 32 || width == 64 || width == 96 || width == 128, PCR_ERR_ARG,
                "ndp_warp: width %d not in {32, 64, 96, 128}", width);
    PCR_REQUIRE(depth >= 1, PCR_ERR_ARG, "ndp_warp: depth must be >= 1");
    if (N == 0) return PCR_OK;
    PCR_REQUIRE(x && x_out && (levels || n_levels == 0), PCR_ERR_ARG, "ndp_warp: null pointer");
    pcr::NdpArgs a;
    a.x = x; a.N = N; a.nlev = n_levels; a.depth = depth; a.k0 = k0;
    a.x_out = x_out; a.x_levels = x_levels; a.nonrig = nonrigidity;
    for (int i = 0; i < n_levels; ++i) {
        const pcr_ndp_level &s = levels[i];
        PCR_REQUIRE(s.w_in && s.b_in && s.w_rot && s.b_rot && s.w_trn && s.b_trn &&
                        (depth == 1 || (s.w_hid && s.b_hid)) && (!s.w_nr || s.b_nr),
                    PCR_ERR_ARG, "ndp_warp: level %d has a null weight", i);
        a.lv[i] = pcr::NdpLevelDev{s.w_in, s.b_in, s.w_hid, s.b_hid, s.w_rot, s.b_rot,
                                   s.w_trn, s.b_trn, s.w_nr, s.b_nr, s.m};
    }
    hipStream_t st = pcr::as_stream(stream);
    const dim3 g((unsigned)((N + 31) / 32));  // 32 points per workgroup, a wave per feature tile
    switch (width / 32) {
        case 1: hipLaunchKernelGGL(pcr::ndp_warp_kernel<1>, g, dim3(64), 0, st, a); break;
        case 2: hipLaunchKernelGGL(pcr::ndp_warp_kernel<2>, g, dim3(128), 0, st, a); break;
        case 3: hipLaunchKernelGGL(pcr::ndp_warp_kernel<3>, g, dim3(192), 0, st, a); break;
        default: hipLaunchKernelGGL(pcr::ndp_warp_kernel<4>, g, dim3(256), 0, st, a); break;
    }
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}
