// Shared pieces of the NDP MLP kernels (ndp.hip, ndp_train.hip): the 32 x 32
// tile of v_mfma_f32_32x32x2_f32 and the LDS exchange of tiles between the
// waves of a workgroup.
//
// A tile holds 32 features x 32 points in 16 accumulator registers: lane
// (j, h) = (lane & 31, lane >> 5), register r holds feature frow(r, h) of point
// j.  k-step r of a chain whose B operand is a tile consumes the feature rows
// {frow(r, 0), frow(r, 1)} the lanes already hold, so a layer's output tile is
// the next layer's B operand as it is.  A workgroup of NT waves owns 32 points,
// wave w feature tile w of every layer: a layer publishes its tile to LDS and
// reads all NT tiles back in the same register layout (ds_read_b128, lanes
// contiguous).  The chains keep the (input tile, k-step) order of one wave
// holding all NT tiles, so the split changes no bits.
#pragma once
#include <hip/hip_runtime.h>

namespace pcr {
namespace ndpt {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int frow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// X[q][lane] = registers 4q .. 4q+3 of one tile as that lane holds them
typedef float4 TileX[4][64];

__device__ __forceinline__ void publish(TileX &X, int l, const f32x16 &T) {
#pragma unroll
    for (int q = 0; q < 4; ++q) X[q][l] = make_float4(T[4 * q], T[4 * q + 1], T[4 * q + 2], T[4 * q + 3]);
}

// acc + sum over input tiles it < NT and k-steps r < 16 of A(it, r) (x) register
// r of tile it, in (it, r) order
template <int NT, class F>
__device__ __forceinline__ f32x16 chain(const TileX *X, int l, F A, f32x16 acc) {
#pragma unroll
    for (int it = 0; it < NT; ++it)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 v = X[it][q][l];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A(it, 4 * q), v.x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A(it, 4 * q + 1), v.y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A(it, 4 * q + 2), v.z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A(it, 4 * q + 3), v.w, acc, 0, 0, 0);
        }
    return acc;
}

}  // namespace ndpt
}  // namespace pcr
