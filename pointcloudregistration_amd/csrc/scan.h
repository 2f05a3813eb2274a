// Workgroup-wide (1024 threads, 16 wave64) exclusive scan helpers.
#pragma once
#include <hip/hip_runtime.h>

namespace pcr {

// Exclusive scan of in[0..len) into out[0..len], out[len] = total.  Must be
// called by all 1024 threads of the block.  `in` and `out` may alias.
// `zero_in`: reset in[i] = 0 after reading (turns counts into cursors).
//
// Thread t owns the contiguous span [t*per, (t+1)*per): one pass sums the
// spans (independent loads, several in flight per thread), one block-wide scan
// of the 1024 span sums, one pass writes.  The previous 1024-element rounds
// paid a dependent global load and four barriers per round (31 us for a
// 32K-slot grid of one cloud); this is two load round trips whatever len is.
__device__ inline void block_exclusive_scan_1024(int *in, int *out, int len, bool zero_in) {
    __shared__ int warp_tot[16];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int per = (len + 1023) >> 10;
    const int b0 = min(len, (int)threadIdx.x * per), b1 = min(len, b0 + per);
    int v = 0;
#pragma unroll 8
    for (int i = b0; i < b1; ++i) v += in[i];
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
        out[len] = acc;
    }
    __syncthreads();
    int run = warp_tot[wid] + x - v;
#pragma unroll 8
    for (int i = b0; i < b1; ++i) {
        const int c = in[i];
        if (zero_in) in[i] = 0;
        out[i] = run;
        run += c;
    }
    __syncthreads();
}

}  // namespace pcr
