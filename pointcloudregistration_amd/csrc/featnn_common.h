// Shared by the two feature-NN screens (featnn.hip: f16 x3 split, D <= 64;
// featnn_f32.hip: augmented f32 operands, 64 < D <= 128).
#pragma once
#include "pcr_internal.h"

namespace pcr {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int count_of(const int32_t *n, int p, int Nmax) {
    return n ? min(max(n[p], 0), Nmax) : Nmax;
}

// merge two top-2 states; lowest index wins equal minima.  Branch-free: the
// screen's values are finite or +inf (never NaN), so plain selects are exact.
__device__ __forceinline__ void top2_merge(float &b1, int &i1, float &b2, float o1, int oi, float o2) {
    const bool take = (o1 < b1) | ((o1 == b1) & (oi < i1));
    const float mx = (b1 < o1) ? o1 : b1;
    const float m2 = (o2 < b2) ? o2 : b2;
    const float n2 = (m2 < mx) ? m2 : mx;
    b1 = take ? o1 : b1;
    i1 = take ? oi : i1;
    b2 = n2;
}

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace

// 64 < D <= 128 (featnn_f32.hip)
int feature_match_f32(const float *F, const float *G, int P, int Nmax, int Mmax, int D,
                      const int32_t *n_src, const int32_t *n_tgt, int32_t *nn12, int32_t *nn21,
                      hipStream_t s);

}  // namespace pcr
