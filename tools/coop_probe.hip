// Standalone exit probe (no torch, no libpcr; ROCm's own HIP runtime): one
// trivial cooperative launch, then exit.  Built by tools/exit_probe.py's
// caller: hipcc --offload-arch=gfx950 tools/coop_probe.hip -o tools/coop_probe_bin
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int *o) { if (threadIdx.x == 0) o[blockIdx.x] = (int)blockIdx.x; }
int main(int argc, char **argv) {
    const int coop = argc > 1 ? atoi(argv[1]) : 1;
    int *o = nullptr;
    if (hipMalloc(&o, 64 * sizeof(int)) != hipSuccess) return 2;
    void *args[] = {&o};
    hipError_t e = coop ? hipLaunchCooperativeKernel((const void *)k, dim3(64), dim3(256), args, 0, 0)
                        : hipLaunchKernel((const void *)k, dim3(64), dim3(256), args, 0, 0);
    if (e != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 3;
    int h[64];
    hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost);
    printf("standalone %s launch ok: %d\n", coop ? "cooperative" : "plain", h[63]);
    hipFree(o);
    return 0;
}
