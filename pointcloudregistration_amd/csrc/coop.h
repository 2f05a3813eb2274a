// Several workgroups per cloud pair (RANSAC verification, ICP): when a batch has
// fewer pairs than the chip has CUs, a pair's sweeps are split over G
// workgroups that meet at a per-pair barrier in global memory.  The G*P
// workgroups of such a launch are made co-resident by a cooperative launch
// (hipLaunchCooperativeKernel fails instead of hanging when they cannot be), so
// the spin-wait below always terminates.  G = 1 launches never call the barrier.
//
// Cross-XCD visibility: see pair_barrier -- loads after it see every
// workgroup's global stores from before it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pcr {

// bar[0] = arrivals (zero before the first arrival; the last arrival resets
// it, so a completed launch leaves it zero), bar[1] = generation (any start).
// Cost matters (a split sweep meets here several times per iteration): each
// thread only waits for its own stores (vmcnt), thread 0 alone makes them
// device-visible (one release fence = one L2 write-back), arrives and spins with
// RELAXED agent-scope loads (no cache invalidation per poll), and one acquire
// fence after the wake-up invalidates the stale lines for the whole CU.
__device__ inline void pair_barrier(unsigned *bar, int G) {
    __builtin_amdgcn_s_waitcnt(0);  // this thread's global stores have completed
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // L2 write-back
        const unsigned gen = __hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned arrived =
            __hip_atomic_fetch_add(&bar[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (arrived == (unsigned)G - 1u) {
            // the last arriver passes every other arriver's release on (acquire
            // their stores, release them with its own)
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
            __hip_atomic_store(&bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&bar[1], gen + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            while (__hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen)
                __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // drop stale lines
    }
    __syncthreads();
}

// global counters a split sweep shares: chunk index and misses
__device__ __forceinline__ int coop_fetch_add(int *p, int v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int coop_load(const int *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// host: workgroups per pair for a launch of P pairs whose kernel fits `per_cu`
// workgroups per CU (0 = cannot tell): fill the chip, at most gmax, 1 when the
// pairs alone fill it
int coop_groups(int P, int per_cu, int gmax = 8);

// host: workgroups a cooperative launch may use when it fits `per_cu` per CU:
// the chip's share of one of the pcr_set_concurrency(k) launches sharing the
// device (CUs * per_cu / k), so k such launches are co-resident; 0 = cannot tell
int coop_capacity(int per_cu);

// host: launch `fn` with P*G workgroups (cooperative when G > 1)
hipError_t coop_launch(const void *fn, int P, int G, int threads, void **args, size_t lds,
                       hipStream_t s);

}  // namespace pcr
