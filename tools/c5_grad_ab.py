"""C5 NDP stage: per-level loss deviation from the reference loop's golden
(tests/golden/c5_golden.npz) under different gradient paths of the level
Chamfer -- the data-scaled two-word fixed point (default), round 3's single
2^-44 word (PCR_NDP_FIXSHIFT=44), and the nnd drop-in kernels' f32 sums
(PCR_NDP_CHAMFER=0).  Diagnostics for the Adam-trajectory tolerance of
tests/test_c5_full_gpu.py.

    python tools/c5_grad_ab.py
"""
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pointcloudregistration_amd import c2p, ndp_opt, synth  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden", "c5_golden.npz")
CFG = dict(iters=40, lr=0.01, max_break_count=15, break_threshold_ratio=0.001, w_reg=0.05,
           m=9, k0=-8, depth=3, width=128)


def run(mode_env):
    for k in ("PCR_NDP_FIXSHIFT", "PCR_NDP_CHAMFER"):
        os.environ.pop(k, None)
    os.environ.update(mode_env)
    g = dict(np.load(GOLD))
    n_pts, seed, lseed, rseed, tseed, step = (int(x) for x in g["seeds"])
    B = synth.make_c5_pair(seed, n=n_pts, m=n_pts, d=32)
    rng = np.random.default_rng(lseed)

    def lv(f):
        return [f] + [(f + rng.normal(0, 0.6, f.shape)).astype(np.float32) for _ in range(2)]
    fs, ft = lv(B.src_feat[0]), lv(B.tgt_feat[0])
    torch.manual_seed(tseed)
    P = ndp_opt.DeformationPyramid(CFG["depth"], CFG["width"], torch.device("cpu"), CFG["k0"], CFG["m"], True)
    for layer in P.pyramid:
        layer.to("cuda")
    res = c2p.register_c2p(B.src[0], B.tgt[0], fs, ft, float(g["voxel"]), ndp_config=CFG, NDP=P,
                           seed=rseed, pair_id=0)
    torch.cuda.synchronize()
    out = []
    for lvl in range(CFG["m"]):
        want = g[f"loss/l{lvl}"]
        got = res["info"][lvl]["losses"]
        k = min(len(want), len(got))
        rel = np.abs(got[:k] - want[:k]) / np.abs(want[:k])
        out.append({"level": lvl, "evaluated": [int(len(got)), int(len(want))],
                    "max_rel": float(rel.max()), "chamfer": res["info"][lvl]["chamfer"]})
    w = np.abs(res["warped"].cpu().numpy()[::step] - g["warped"]).max()
    return {"levels": out, "warped_max_abs": float(w)}


if __name__ == "__main__":
    modes = {"two_word": {}, "fix44": {"PCR_NDP_FIXSHIFT": "44"}, "nnd_f32": {"PCR_NDP_CHAMFER": "0"}}
    print(json.dumps({k: run(v) for k, v in modes.items()}, indent=1))
