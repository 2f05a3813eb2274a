"""GPU: f4, the NDP level optimisation (graph-captured iterations with the
early-stop rule and Adam on the device) against the reference's own
Deformation_Pyramid run through registration.py's loop on the CPU
(tests/golden/ndp_opt_golden.npz, make_golden_ndp_opt.py).

Tolerances: the first loss of every level depends only on the inputs and the
initial weights (f32 forward, different summation orders): 2e-6 relative.  Later
iterations follow Adam trajectories whose normalised steps amplify f32 rounding
of near-zero gradients, so losses are compared to 2e-3 relative and the warped
points to 2e-3 absolute (clouds of radius 0.6).
"""
import os

import numpy as np
import pytest
import torch

from pointcloudregistration_amd import ndp_opt

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ndp_opt_golden.npz")
CFG = dict(iters=15, lr=0.01, max_break_count=15, break_threshold_ratio=0.001, w_reg=0.05,
           m=3, k0=-8, depth=3, width=128)


def _pyramid(g):
    dev = torch.device("cuda")
    P = ndp_opt.DeformationPyramid(CFG["depth"], CFG["width"], dev, CFG["k0"], CFG["m"], True)
    for lvl, layer in enumerate(P.pyramid):
        sd = {k: torch.from_numpy(g[f"init/l{lvl}/{k}"]) for k in layer.state_dict()}
        layer.load_state_dict(sd)
    return P


@pytest.mark.parametrize("use_graph", [True, False])
def test_ndp_optimisation_matches_reference_loop(use_graph):
    g = np.load(GOLD)
    P = _pyramid(g)
    warped, hist, _, info = ndp_opt.optimize_deformation_pyramid(
        torch.from_numpy(g["src"]).cuda(), torch.from_numpy(g["tgt"]).cuda(), g["inds"], CFG, NDP=P,
        use_graph=use_graph)
    for lvl in range(3):
        want = g[f"loss/l{lvl}"]
        got = info[lvl]["losses"]
        assert info[lvl]["evaluated"] == len(want), lvl
        assert abs(got[0] - want[0]) <= 2e-6 * abs(want[0]), (lvl, got[0], want[0])
        np.testing.assert_allclose(got, want, rtol=2e-3)
        np.testing.assert_allclose(hist[lvl], g[f"hist/l{lvl}"], atol=2e-3)
    np.testing.assert_allclose(warped.cpu().numpy(), g["warped"], atol=2e-3)


def test_graph_and_eager_agree():
    g = np.load(GOLD)
    a = ndp_opt.optimize_deformation_pyramid(torch.from_numpy(g["src"]).cuda(),
                                             torch.from_numpy(g["tgt"]).cuda(), g["inds"], CFG,
                                             NDP=_pyramid(g), use_graph=True)
    b = ndp_opt.optimize_deformation_pyramid(torch.from_numpy(g["src"]).cuda(),
                                             torch.from_numpy(g["tgt"]).cuda(), g["inds"], CFG,
                                             NDP=_pyramid(g), use_graph=False)
    # same kernels, same order: the replayed graph is the eager loop
    assert torch.equal(a[0], b[0])
    for x, y in zip(a[3], b[3]):
        assert np.array_equal(x["losses"], y["losses"])


def test_early_stop_rule_on_device():
    """pcr_ndp_control == registration.py:246-256 on a scripted loss sequence."""
    from pointcloudregistration_amd import _lib
    seq = [0.5, 0.4999, 0.49985, 0.3, 0.29999, 0.299985, 0.2999849, 0.2, 5e-5, 0.1]
    for ratio, mb in [(0.001, 2), (0.001, 15), (1e-6, 2)]:
        st = torch.tensor([1, 0, 1e6, 0, 0, 0, 0, 0], dtype=torch.float64, device="cuda")
        loss = torch.zeros((), dtype=torch.float32, device="cuda")
        dev_steps = []
        for L in seq:
            loss.fill_(L)
            _lib.call("pcr_ndp_control", _lib.ptr(loss), _lib.ptr(st), ratio, mb, 1e-4,
                      _lib.stream_handle())
            dev_steps.append(int(st[5].item()))
        # host restatement
        host, bc, prev, alive = [], 0, 1e6, True
        for L in seq:
            L = float(np.float32(L))
            if not alive:
                host.append(0)
                continue
            if L < 1e-4:
                alive = False
                host.append(0)
                continue
            if abs(prev - L) < prev * ratio:
                bc += 1
            if bc >= mb:
                alive = False
                host.append(0)
                continue
            prev = L
            host.append(1)
        assert dev_steps == host, (ratio, mb, dev_steps, host)


def test_large_target_takes_nnd_path():
    """a target above pcr_ndp_chamfer_max_points() (32,768: an
    unsampled target, c2p.register_c2p passes tgt whole) runs the level Chamfer
    on the nnd drop-in kernels instead of failing; the same level with the
    target cut to the limit runs the fused pass."""
    from pointcloudregistration_amd import _lib
    lim = int(_lib.load().pcr_ndp_chamfer_max_points())
    rng = np.random.default_rng(5)
    tgt = rng.uniform(-0.5, 0.5, (lim + 7000, 3)).astype(np.float32)
    src = (tgt[:3000] + rng.normal(0, 0.01, (3000, 3))).astype(np.float32)
    cfg = dict(CFG, iters=3, m=1)
    torch.manual_seed(0)
    P = ndp_opt.DeformationPyramid(cfg["depth"], cfg["width"], torch.device("cuda"), cfg["k0"], 1, True)
    sd = {k: v.clone() for k, v in P.pyramid[0].state_dict().items()}
    _, _, _, info = ndp_opt.optimize_deformation_pyramid(torch.from_numpy(src).cuda(),
                                                         torch.from_numpy(tgt).cuda(),
                                                         np.arange(0, 3000, 2), cfg, NDP=P)
    assert info[0]["chamfer"] == "nnd" and info[0]["mlp"] == "fused"
    assert np.isfinite(info[0]["losses"]).all()
    # the same level with the target cut below the limit runs the fused pass
    P2 = ndp_opt.DeformationPyramid(cfg["depth"], cfg["width"], torch.device("cuda"), cfg["k0"], 1, True)
    P2.pyramid[0].load_state_dict(sd)
    _, _, _, info2 = ndp_opt.optimize_deformation_pyramid(torch.from_numpy(src).cuda(),
                                                          torch.from_numpy(tgt[:lim]).cuda(),
                                                          np.arange(0, 3000, 2), cfg, NDP=P2)
    assert info2[0]["chamfer"] == "fused"
