// Diagnostics: one trivial launch, cooperative or plain, from inside libpcr
// and nothing else of the library -- tools/exit_probe.py's "coop" / "plain"
// modes isolate the exit-time fault seen under rocprofv3.
#include "pcr_internal.h"

namespace pcr {
namespace {
__global__ __launch_bounds__(256) void probe_kernel(int *out) {
    if (threadIdx.x == 0) out[blockIdx.x] = (int)blockIdx.x;
}
}  // namespace
}  // namespace pcr

extern "C" int pcr_coop_probe(int32_t *out, int32_t blocks, int32_t cooperative, pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(out && blocks >= 1 && blocks <= 256, PCR_ERR_ARG, "coop_probe: 1..256 blocks");
    hipStream_t s = pcr::as_stream(stream);
    void *args[] = {&out};
    if (cooperative)
        PCR_HIP_CHECK(hipLaunchCooperativeKernel((const void *)pcr::probe_kernel, dim3(blocks), dim3(256), args, 0, s));
    else
        PCR_HIP_CHECK(hipLaunchKernel((const void *)pcr::probe_kernel, dim3(blocks), dim3(256), args, 0, s));
    return PCR_OK;
}
