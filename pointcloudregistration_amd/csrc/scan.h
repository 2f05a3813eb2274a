// Workgroup-wide (1024 threads, 16 wave64) exclusive scan helpers.
#pragma once
#include <hip/hip_runtime.h>

namespace pcr {

// Exclusive scan of in[0..len) into out[0..len], out[len] = total.  Must be
// called by all 1024 threads of the block.  `in` and `out` may alias.
// `zero_in`: reset in[i] = 0 after reading (turns counts into cursors).
__device__ inline void block_exclusive_scan_1024(int *in, int *out, int len, bool zero_in) {
    __shared__ int warp_tot[16];
    __shared__ int carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int base = 0; base < len; base += 1024) {
        const int i = base + threadIdx.x;
        const int v = (i < len) ? in[i] : 0;
        int x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) warp_tot[wid] = x;
        __syncthreads();
        if (threadIdx.x == 0) {
            int acc = 0;
            for (int w = 0; w < 16; ++w) {
                const int t = warp_tot[w];
                warp_tot[w] = acc;
                acc += t;
            }
        }
        __syncthreads();
        const int excl = carry + warp_tot[wid] + x - v;
        if (i < len) {
            if (zero_in) in[i] = 0;
            out[i] = excl;
        }
        __syncthreads();
        if (threadIdx.x == 1023) carry = excl + v;
        __syncthreads();
    }
    if (threadIdx.x == 0) out[len] = carry;
    __syncthreads();
}

}  // namespace pcr
