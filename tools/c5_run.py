"""C5 flow on the GPU box (bench.measure_c5's pair): per-level NDP replay times and
evaluated iterations; run under rocprofv3 --kernel-trace --stats for the C5
kernel profile (profiles/r03/)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
from pointcloudregistration_amd import c2p, ndp_opt, registration as reg, synth  # noqa: E402

B = synth.make_c5_pair(515, n=20000, m=20000, d=32)
rng = np.random.default_rng(5)


def lv(f):
    return [f] + [(f + rng.normal(0, 0.6, f.shape)).astype(np.float32) for _ in range(2)]


fs, ft = lv(B.src_feat[0]), lv(B.tgt_feat[0])
dev = torch.device("cuda")
S, G = torch.from_numpy(B.src[0]).to(dev), torch.from_numpy(B.tgt[0]).to(dev)
FS = [torch.from_numpy(f).to(dev) for f in fs]
FT = [torch.from_numpy(f).to(dev) for f in ft]
cfg = ndp_opt.NDPConfig(max_break_count=int(os.environ.get("MAX_BREAK", "15")))
for rep in range(int(os.environ.get("REPS", "2"))):
    a, b = [f.clone() for f in FS], [f.clone() for f in FT]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, _, fs_h, ft_h = c2p.vote(S, G, a, b, 0.025)
    prm = reg.RansacParams(max_correspondence_distance=0.025, distance_check=0.025, seed=1)
    br = reg.register_feature_ransac_batch(S, G, fs_h, ft_h, prm, want_mask=False)
    est = reg.transform_batch(S.unsqueeze(0), br.transformation)[0]
    corrs = torch.nonzero(br.corr_tgt[0] >= 0).flatten().cpu().numpy()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    torch.manual_seed(0)
    P = ndp_opt.DeformationPyramid(3, 128, dev, -8, 9, True)
    w, _, _, info = ndp_opt.optimize_deformation_pyramid(est, G, corrs, cfg, NDP=P)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"rep {rep}: rigid {1e3 * (t1 - t0):.1f} ms, ndp {1e3 * (t2 - t1):.1f} ms, inds {len(corrs)}, "
          f"evaluated {[i['evaluated'] for i in info]}, replay_ms "
          f"{[round(i.get('replay_ms', 0), 1) for i in info]}, setup_ms "
          f"{[round(i.get('setup_ms', 0), 1) for i in info]}, capture_ms "
          f"{[round(i.get('capture_ms', 0), 1) for i in info]}, level_ms "
          f"{[round(i.get('level_ms', 0), 1) for i in info]}, fb_cnt {[i.get('fb_cnt') for i in info]}", flush=True)
