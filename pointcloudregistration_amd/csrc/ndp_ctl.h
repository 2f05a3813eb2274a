// f4: the reference's early-stop rule (registration.py:246-256) on the device,
// shared by pcr_ndp_control and the fused loss of pcr_ndp_chamfer_loss.
// State (device f64[8]): 0 active, 1 break count, 2 loss_prev, 3 steps taken,
// 4 last loss, 5 step flag of this iteration, 6 iterations evaluated.
#pragma once
#include <hip/hip_runtime.h>

namespace pcr {

// one thread; f64 on the f32 loss exactly as Python evaluates loss.item()
__device__ inline void ndp_control_rule(float loss, double *st, double ratio, int max_break, double stop_loss) {
    if (st[0] == 0.0) {
        st[5] = 0.0;
        return;
    }
    const double L = (double)loss;
    st[6] += 1.0;
    st[4] = L;
    if (L < stop_loss) {
        st[0] = 0.0;
        st[5] = 0.0;
        return;
    }
    if (fabs(st[2] - L) < st[2] * ratio) st[1] += 1.0;
    if (st[1] >= (double)max_break) {
        st[0] = 0.0;
        st[5] = 0.0;
        return;
    }
    st[2] = L;
    st[3] += 1.0;
    st[5] = 1.0;
}

}  // namespace pcr
