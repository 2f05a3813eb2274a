"""C5 at its own configuration (BASELINE configs[4]):
c2p-net/testScript.py:161-192 -> deformationpyramid/model/registration.py:149-289
on one 20,000-point pair with NDP m = 9, width 128 (the fused HIP training
kernels, not the torch-autograd MLP), depth 3, 40 iterations and the early-stop
rule of config/NDP.yaml, through c2p.register_c2p.

Golden: tests/golden/c5_golden.npz (make_golden_c5.py):
* the rigid stage from the build's oracle chain -- vote, the exact feature 1-NN
  both ways, the mutual filter, feature RANSAC at d = voxel = 0.025, the f32
  estimate, the unique inlier sources.  Bar: bit-exact (T raw f64 bits, the
  inlier source set, SHA-256 of the voted features and of the estimate);
* the NDP stage from the REFERENCE's own Deformation_Pyramid run through the
  loop of optimize_deformation_pyramid on the CPU (f32), fed the same estimate /
  target / inds, with the same initial weights (the build's mirror under the
  same torch seed: checked by SHA-256).  Tolerances as test_ndp_opt_gpu.py: the
  first loss of every level 2e-6 relative (inputs + weights only; f32 sums in
  another order), every loss 2e-3 relative (Adam's normalised steps amplify f32
  rounding of near-zero gradients) or 4x the reference's own spread at that
  level, whichever is larger (REF_SPREAD), the warped samples and the final warp
  2e-3 absolute (every 10th point; clouds of unit scale), and the same number of
  evaluated iterations per level (the early stop fires at the same iteration).

REF_SPREAD: how far the REFERENCE's own loop moves when only the order of its
f32 sums changes (tools/c5_ref_spread.py: the same loop with the Chamfer subset
permuted, seeds 1 and 2, max per level).  Level 4 sits where any rounding
difference grows ~40x -- the reference against itself differs by 2.07e-3
there, against <= 7.8e-5 at every other level measured; this build's exact
(order-free) gradient lands at 5.0e-3 on that level and <= 2.3e-4 elsewhere,
with the final warp within 5e-6 of the golden.
"""
import hashlib
import os

import numpy as np
import pytest
import torch

from pointcloudregistration_amd import c2p, ndp_opt, synth

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c5_golden.npz")
CFG = dict(iters=40, lr=0.01, max_break_count=15, break_threshold_ratio=0.001, w_reg=0.05,
           m=9, k0=-8, depth=3, width=128)
# max relative loss deviation of the reference against itself per level (levels
# 6-8 not measured: the 2e-3 floor applies)
REF_SPREAD = [4.6e-7, 2.9e-5, 5.5e-5, 5.3e-5, 2.07e-3, 7.8e-5]


def _sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


@pytest.fixture(scope="module")
def c5():
    g = dict(np.load(GOLD))
    n_pts, seed, lseed, rseed, tseed, step = (int(x) for x in g["seeds"])
    B = synth.make_c5_pair(seed, n=n_pts, m=n_pts, d=32)
    rng = np.random.default_rng(lseed)

    def lv(f):
        return [f] + [(f + rng.normal(0, 0.6, f.shape)).astype(np.float32) for _ in range(2)]
    fs, ft = lv(B.src_feat[0]), lv(B.tgt_feat[0])
    assert _sha(B.src[0], B.tgt[0], *fs, *ft) == str(g["inputs_sha"]), "synthetic C5 inputs drifted"
    torch.manual_seed(tseed)
    P = ndp_opt.DeformationPyramid(CFG["depth"], CFG["width"], torch.device("cpu"), CFG["k0"], CFG["m"],
                                   True)
    init = {f"init/l{lvl}/{k}": v.numpy().copy()
            for lvl, layer in enumerate(P.pyramid) for k, v in layer.state_dict().items()}
    assert bool(g["init_from_mirror_seed"]) and _sha(*[init[k] for k in sorted(init)]) == str(g["init_sha"])
    for layer in P.pyramid:
        layer.to("cuda")
    res = c2p.register_c2p(B.src[0], B.tgt[0], fs, ft, float(g["voxel"]), ndp_config=CFG, NDP=P,
                           seed=rseed, pair_id=0)
    torch.cuda.synchronize()
    return g, res, step


def test_c5_rigid_stage_bitexact(c5):
    g, res, _ = c5
    assert res["T"].cpu().numpy().tobytes() == g["T"].tobytes()
    assert np.array_equal(res["corrs"].cpu().numpy(), g["inds"])
    assert _sha(res["source_feats_h"].cpu().numpy(), res["target_feats_h"].cpu().numpy()) == str(g["vote_sha"])
    assert _sha(res["estimate"].cpu().numpy()) == str(g["estimate_sha"])


def test_c5_ndp_stage_vs_reference_loop(c5):
    g, res, step = c5
    info, hist = res["info"], res["hist"]
    assert len(info) == CFG["m"]
    for lvl in range(CFG["m"]):
        # the fused HIP path ran (width 128 MLP kernels, the level Chamfer pass,
        # graph replays) -- not the torch-autograd or nnd fallbacks
        assert info[lvl]["mlp"] == "fused" and info[lvl]["chamfer"] == "fused", info[lvl]
        assert "replay_ms" in info[lvl], lvl
        want = g[f"loss/l{lvl}"]
        got = info[lvl]["losses"]
        assert info[lvl]["evaluated"] == len(want), (lvl, info[lvl]["evaluated"], len(want))
        assert abs(got[0] - want[0]) <= 2e-6 * abs(want[0]), (lvl, got[0], want[0])
        spread = REF_SPREAD[lvl] if lvl < len(REF_SPREAD) else 0.0
        np.testing.assert_allclose(got, want, rtol=max(2e-3, 4.0 * spread))
        np.testing.assert_allclose(hist[lvl][::step], g[f"hist/l{lvl}"], atol=2e-3)
    np.testing.assert_allclose(res["warped"].cpu().numpy()[::step], g["warped"], atol=2e-3)
