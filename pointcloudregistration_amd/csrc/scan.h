// Workgroup-wide (1024 threads, 16 wave64) exclusive scan helpers.
#pragma once
#include <hip/hip_runtime.h>

namespace pcr {

// Exclusive scan of in[0..len) into out[0..len], out[len] = total.  Must be
// called by all 1024 threads of the block.  `in` and `out` may alias.
// `zero_in`: reset in[i] = 0 after reading (turns counts into cursors).
//
// Wave w owns the contiguous segment [w*seg, (w+1)*seg) and walks it 64
// consecutive words at a time (coalesced in global memory, one word per bank in
// LDS): one pass sums the segment, one block-wide scan of the 16 segment sums,
// one pass scans 64 words per step with shuffles and writes.  (The previous
// version gave each THREAD a contiguous span: for LDS arrays its reads were
// per-fold bank conflicts -- 32-way for the 32K buckets of the spatial order --
// and in global memory every load touched 64 lines.)
__device__ inline void block_exclusive_scan_1024(int *in, int *out, int len, bool zero_in) {
    __shared__ int warp_tot[16];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int seg = (((len + 15) >> 4) + 63) & ~63;
    const int b0 = min(len, wid * seg), b1 = min(len, b0 + seg);
    int v = 0;
    for (int i = b0 + lane; i < b1; i += 64) v += in[i];
#pragma unroll
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) warp_tot[wid] = v;
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
    int run = warp_tot[wid];
    for (int i0 = b0; i0 < b1; i0 += 64) {
        const int i = i0 + lane;
        const int c = i < b1 ? in[i] : 0;
        int x = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (i < b1) {
            if (zero_in) in[i] = 0;
            out[i] = run + x - c;
        }
        run += __shfl(x, 63, 64);
    }
    __syncthreads();
}

}  // namespace pcr
