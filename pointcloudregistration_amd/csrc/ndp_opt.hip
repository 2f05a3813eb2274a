// f4: the per-iteration control and optimizer step of the NDP
// level optimisation (c2p-net/deformationpyramid/model/registration.py:196-262),
// as device kernels so a whole iteration -- warp, truncated Chamfer, BCE,
// backward, early-stop rule, Adam -- can be captured once in a HIP graph and
// replayed with no host round trip (the reference reads loss.item() every
// iteration, :246-256).
//
//   ndp_control   the reference's early-stop rule on the device, in f64 on the
//                 f32 loss exactly as Python evaluates it:
//                   if loss < 1e-4: break
//                   if |loss_prev - loss| < loss_prev * ratio: count += 1
//                   if count >= max_break_count: break
//                   loss_prev = loss; (step)
//                 A broken level leaves every later replay a no-op.
//   adam_masked   torch.optim.Adam's update (lerp first moment, addcmul second
//                 moment, bias corrections, addcdiv) for all parameter tensors of
//                 the level in one launch, skipped when the control said break.
// State (device f64[8]): 0 active, 1 break count, 2 loss_prev, 3 steps taken,
// 4 last loss, 5 step flag of this iteration, 6 iterations evaluated.
#include "pcr_internal.h"
#include "ndp_ctl.h"

namespace pcr {
namespace {

__global__ void ndp_control_kernel(const float *loss, double *st, double ratio, int max_break,
                                   double stop_loss) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    ndp_control_rule(*loss, st, ratio, max_break, stop_loss);
}

__global__ __launch_bounds__(256) void adam_masked_kernel(const pcr_adam_tensor *tab,
                                                          const double *st, double lr, double b1,
                                                          double b2, double eps) {
    if (st[5] == 0.0) return;
    const pcr_adam_tensor T = tab[blockIdx.y];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= T.n) return;
    // host-side scalars of torch's _multi_tensor_adam, in f64 then as f32 operands
    double pb1 = 1.0, pb2 = 1.0;
    for (int k = 0; k < (int)st[3]; ++k) {
        pb1 *= b1;
        pb2 *= b2;
    }
    const float step_size = (float)(lr / (1.0 - pb1));
    const float bc2_sqrt = (float)__builtin_sqrt(1.0 - pb2);
    const float g = T.grad[i];
    float m = T.exp_avg[i];
    m = m + (float)(1.0 - b1) * (g - m);                   // lerp_(grad, 1 - beta1), weight < 0.5
    float v = T.exp_avg_sq[i] * (float)b2;
    v = v + (float)(1.0 - b2) * (g * g);                   // addcmul_(grad, grad, 1 - beta2)
    const float denom = __builtin_sqrtf(v) / bc2_sqrt + (float)eps;
    T.param[i] = T.param[i] + (-step_size) * (m / denom);  // addcdiv_(exp_avg, denom, -step_size)
    T.exp_avg[i] = m;
    T.exp_avg_sq[i] = v;
}

}  // namespace
}  // namespace pcr

extern "C" int pcr_ndp_control(const float *loss, double *state, double break_threshold_ratio,
                               int32_t max_break_count, double stop_loss, pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(loss && state, PCR_ERR_ARG, "ndp_control: null pointer");
    hipLaunchKernelGGL(pcr::ndp_control_kernel, dim3(1), dim3(64), 0, pcr::as_stream(stream), loss,
                       state, break_threshold_ratio, (int)max_break_count, stop_loss);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}

extern "C" int pcr_adam_masked(const pcr_adam_tensor *tensors, int32_t n_tensors, int32_t max_numel,
                               const double *state, double lr, double beta1, double beta2,
                               double eps, pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(n_tensors >= 0 && n_tensors <= 65535 && max_numel >= 0, PCR_ERR_ARG,
                "adam_masked: bad sizes");
    if (n_tensors == 0 || max_numel == 0) return PCR_OK;
    PCR_REQUIRE(tensors && state, PCR_ERR_ARG, "adam_masked: null pointer");
    hipLaunchKernelGGL(pcr::adam_masked_kernel, dim3((max_numel + 255) / 256, n_tensors), dim3(256),
                       0, pcr::as_stream(stream), tensors, state, lr, beta1, beta2, eps);
    PCR_LAUNCH_CHECK();
    return PCR_OK;
}
