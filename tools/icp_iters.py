"""Diagnostic: per-pair ICP iteration counts of one C4 step (256 pairs), the
distribution and the pairs that hit max_iteration."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloudregistration_amd import pipeline, synth  # noqa: E402

P = int(os.environ.get("PAIRS", "256"))
b = synth.make_batch(P, n=8192, m=8192, d=32, base_seed=1000, first_pair=0, feat_noise=1.0)
pp = pipeline.PairPipeline(b.src, b.tgt, b.src_feat, b.tgt_feat, pipeline.default_params(),
                           pair_ids=np.arange(P, dtype=np.int32))
pp.run()
torch.cuda.synchronize()
it = pp.st_i[:, 0].cpu().numpy().astype(int) if pp.st_i.dim() == 2 else pp.st_i.view(-1, 2)[:, 0].cpu().numpy()
print("icp iterations: mean %.2f max %d" % (it.mean(), it.max()))
print("histogram", np.bincount(it).tolist())
rs = pp.st_r.cpu().numpy().reshape(P, -1)
print("ransac stats first pair", rs[0].tolist())
