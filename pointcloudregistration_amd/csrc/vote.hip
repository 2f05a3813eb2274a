// a5 (ii): the level voting of c2p-net/ngenet/models/vote.py:12-37, after the
// three feature-space nearest-neighbour searches (get_coor_points, :6-9, which
// run on the featnn screen).  Per source point i with nearest targets j1, j2, j3
// at the h / m / l feature levels:
//   d12 = sqrt(sum((t[j1] - t[j2])^2)), d13, d23   (f32, numpy's order:
//         ((dx*dx + dy*dy) + dz*dz), correctly rounded sqrt)
//   sel_h = d12 < thr or d13 < thr;  sel_m = d23 < thr   (thr = f32(2 voxel))
//   replace = !sel_h and sel_m:  fs_h[i] <- fs_m[i],  ft_h[j2] <- ft_m[j2]
// Rows written for several i carry the same values (the reference's fancy
// assignment likewise), so the result does not depend on thread order.
#include "pcr_internal.h"

namespace pcr {
namespace {

__device__ __forceinline__ float dist3(const float *a, const float *b) {
    const float dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
    return __fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz)));
}

__global__ void vote_kernel(const float *tgt, int m, const int32_t *ih, const int32_t *im,
                            const int32_t *il, int n, float thr, float *fs_h, const float *fs_m,
                            float *ft_h, const float *ft_m, int D, uint8_t *replaced) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int j1 = ih[i], j2 = im[i], j3 = il[i];
    if (j1 < 0 || j1 >= m || j2 < 0 || j2 >= m || j3 < 0 || j3 >= m) {
        if (replaced) replaced[i] = 0;
        return;
    }
    const float *y1 = tgt + 3 * (size_t)j1, *y2 = tgt + 3 * (size_t)j2, *y3 = tgt + 3 * (size_t)j3;
    const bool sel_h = dist3(y1, y2) < thr || dist3(y1, y3) < thr;
    const bool sel_m = dist3(y2, y3) < thr;
    const bool rep = !sel_h && sel_m;
    if (replaced) replaced[i] = rep ? 1 : 0;
    if (!rep) return;
    for (int k = 0; k < D; ++k) fs_h[(size_t)i * D + k] = fs_m[(size_t)i * D + k];
    for (int k = 0; k < D; ++k) ft_h[(size_t)j2 * D + k] = ft_m[(size_t)j2 * D + k];
}

}  // namespace
}  // namespace pcr

extern "C" int pcr_vote_apply(const float *tgt_xyz, int32_t m, const int32_t *nn_h,
                              const int32_t *nn_m, const int32_t *nn_l, int32_t n, double voxel_size,
                              float *src_feat_h, const float *src_feat_m, float *tgt_feat_h,
                              const float *tgt_feat_m, int32_t D, uint8_t *replaced,
                              pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(n >= 0 && m >= 0 && D >= 0, PCR_ERR_ARG, "vote: negative size");
    if (n == 0) return PCR_OK;
    PCR_REQUIRE(tgt_xyz && nn_h && nn_m && nn_l && src_feat_h && src_feat_m && tgt_feat_h && tgt_feat_m,
                PCR_ERR_ARG, "vote: null pointer");
    const float thr = (float)(voxel_size * 2.0);  // numpy: f32 array < python float
    hipLaunchKernelGGL(pcr::vote_kernel, dim3((n + 255) / 256), dim3(256), 0, pcr::as_stream(stream),
                       tgt_xyz, m, nn_h, nn_m, nn_l, n, thr, src_feat_h, src_feat_m, tgt_feat_h,
                       tgt_feat_m, D, replaced);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}
