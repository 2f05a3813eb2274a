"""ICP microbench on the C4 shape: P pairs x 8192 points, init = ground truth
perturbed like a RANSAC result, d = 0.02 (RANSAC.py refine).  Prints ms per launch
(HIP events) and, with PCR_ICP_TIMING=1, the kernel's phase split (stderr).
usage: python tools/icp_bench.py [P] [G]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloudregistration_amd import registration as reg, synth  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 256
if len(sys.argv) > 2:
    os.environ["PCR_COOP_G"] = sys.argv[2]
B = synth.make_batch(P, n=8192, m=8192, d=4, base_seed=1000, feat_noise=1.0)
rng = np.random.default_rng(1)
init = np.zeros((P, 4, 4))
for p in range(P):
    init[p, :3, :3] = synth.rotation_xyz(*rng.normal(0, 0.004, 3)) @ B.R[p]
    init[p, :3, 3] = B.t[p] + rng.normal(0, 0.002, 3)
    init[p, 3, 3] = 1
S, T = torch.from_numpy(B.src).cuda(), torch.from_numpy(B.tgt).cuda()
I = torch.from_numpy(init).cuda()
prm = reg.IcpParams(0.02)
res = reg.icp_batch(S, T, I, prm, want_corr=False)
torch.cuda.synchronize()
timing = os.environ.pop("PCR_ICP_TIMING", None)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    reg.icp_batch(S, T, I, prm, want_corr=False)
e1.record()
torch.cuda.synchronize()
print(f"P={P} G={os.environ.get('PCR_COOP_G', 'auto')}: {e0.elapsed_time(e1) / 10:.3f} ms/launch, "
      f"iters mean {res.stats[:, 0].float().mean().item():.2f}, fitness mean {res.fitness.mean().item():.3f}")
if timing:
    os.environ["PCR_ICP_TIMING"] = timing
    reg.icp_batch(S, T, I, prm, want_corr=False)
    torch.cuda.synchronize()
