"""Is the C4 step host-bound?  Host time to enqueue one pcr_pipeline_step (the GPU
may lag behind) against the wall time per step once synchronised, for P pairs.
With PCR_HOST_TIMING=1 the library prints its per-stage host times (stderr).
usage: python tools/host_overhead.py [P]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloudregistration_amd import synth  # noqa: E402
from pointcloudregistration_amd.pipeline import PairPipeline, default_params  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 32
B = synth.make_batch(P, n=8192, m=8192, d=32, base_seed=1000, feat_noise=1.0)
pipe = PairPipeline(B.src, B.tgt, B.src_feat, B.tgt_feat, default_params(seed=0),
                    pair_ids=np.arange(P, dtype=np.int32))
timing = os.environ.pop("PCR_HOST_TIMING", None)
for _ in range(3):
    pipe.run()
torch.cuda.synchronize()
K = 20
t0 = time.perf_counter()
for _ in range(K):
    pipe.run()
th = (time.perf_counter() - t0) / K
torch.cuda.synchronize()
tt = (time.perf_counter() - t0) / K
# one step enqueued on an idle GPU: its host time alone
torch.cuda.synchronize()
t1 = time.perf_counter()
pipe.run()
t1h = time.perf_counter() - t1
torch.cuda.synchronize()
t1t = time.perf_counter() - t1
print(f"P={P}: back-to-back host enqueue {th * 1e3:.3f} ms/step, wall {tt * 1e3:.3f} ms/step; "
      f"single step host {t1h * 1e3:.3f} ms, wall {t1t * 1e3:.3f} ms")
if timing:
    os.environ["PCR_HOST_TIMING"] = timing
    pipe.run()
    torch.cuda.synchronize()
