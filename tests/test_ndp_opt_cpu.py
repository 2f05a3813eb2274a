"""CPU: the f4 host pieces -- the NDP module mirror reproduces the reference's
Deformation_Pyramid.warp (tests/golden/ndp_golden.npz, generated from
c2p-net/deformationpyramid/model/nets.py), and the config mapping."""
import os

import numpy as np
import torch

from pointcloudregistration_amd import ndp_opt

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_mirror_pyramid_matches_reference_warp():
    g = np.load(os.path.join(GOLD, "ndp_golden.npz"))
    P = ndp_opt.DeformationPyramid(3, 32, "cpu", -8, 3, nonrigidity_est=True)
    for lvl, layer in enumerate(P.pyramid):
        layer.load_state_dict({k: torch.from_numpy(g[f"ndp/l{lvl}/{k}"]) for k in layer.state_dict()})
    with torch.no_grad():
        y, data = P.warp(torch.from_numpy(g["ndp/x"]))
    np.testing.assert_allclose(y.numpy(), g["ndp/y"], atol=1e-6)
    for lvl in range(3):
        np.testing.assert_allclose(data[lvl][0].numpy(), g[f"ndp/level{lvl}"], atol=1e-6)
        if lvl > 0:
            np.testing.assert_allclose(data[lvl][1].numpy(), g[f"ndp/nonrigid{lvl}"], atol=1e-6)
        else:
            assert data[lvl][1] is None


def test_config_from_yaml_like_sources():
    class Obj:
        iters, lr, m = 5, 0.1, 2
    c = ndp_opt.NDPConfig.from_any(Obj())
    assert (c.iters, c.lr, c.m, c.width, c.w_reg) == (5, 0.1, 2, 128, 0.05)
    c = ndp_opt.NDPConfig.from_any({"iters": 3, "break_threshold_ratio": 0.01})
    assert (c.iters, c.break_threshold_ratio, c.max_break_count) == (3, 0.01, 15)


def test_mirror_state_dict_names_match_reference_fixture():
    g = np.load(os.path.join(GOLD, "ndp_opt_golden.npz"))
    P = ndp_opt.DeformationPyramid(3, 128, "cpu", -8, 3, nonrigidity_est=True)
    for lvl, layer in enumerate(P.pyramid):
        want = sorted(k[len(f"init/l{lvl}/"):] for k in g.files if k.startswith(f"init/l{lvl}/"))
        assert sorted(layer.state_dict()) == want
