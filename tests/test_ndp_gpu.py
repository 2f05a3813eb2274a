"""a10 parity: the fused NDP warp kernel vs the numpy f64 oracle (which is
pinned to the reference's own Deformation_Pyramid.warp output, see
test_oracle_ndp.py) and vs that golden output directly.  Floating point:
north_star's 1e-5 tolerance, absolute on unit-scale coordinates."""
import os

import numpy as np
import pytest
import torch

from pointcloudregistration_amd import ndp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(__file__)


def _golden_levels():
    z = np.load(os.path.join(HERE, "golden", "ndp_golden.npz"))
    levels = [{k[len(f"ndp/l{i}/"):]: z[k] for k in z.files if k.startswith(f"ndp/l{i}/")}
              for i in range(3)]
    return z, levels


def test_ndp_warp_matches_reference_golden():
    z, levels = _golden_levels()
    y, data = ndp.warp(levels, z["ndp/x"])
    np.testing.assert_allclose(y.cpu().numpy(), z["ndp/y"], rtol=0, atol=1e-5)
    for i in range(3):
        np.testing.assert_allclose(data[i][0].cpu().numpy(), z[f"ndp/level{i}"], rtol=0, atol=1e-5)
    assert data[0][1] is None
    for i in (1, 2):
        np.testing.assert_allclose(data[i][1].cpu().numpy(), z[f"ndp/nonrigid{i}"], rtol=0, atol=1e-6)


@pytest.mark.parametrize("width,depth,m", [(128, 3, 9), (64, 2, 4), (96, 4, 3), (32, 1, 2)])
def test_ndp_warp_vs_oracle_configs(oracle, width, depth, m):
    """C5 shape (width 128, depth 3, 9 levels) and others; weights scaled so
    the warp moves points visibly; N not a multiple of the 128-point block."""
    rng = np.random.default_rng(width + depth)
    levels = []
    for i in range(m):
        sd = {"input.0.weight": rng.normal(0, 0.6, (width, 6)), "input.0.bias": rng.normal(0, 0.1, width)}
        for k in range(depth - 1):
            sd[f"mlp.pts_linears.{k}.weight"] = rng.normal(0, 1.5 / np.sqrt(width), (width, width))
            sd[f"mlp.pts_linears.{k}.bias"] = rng.normal(0, 0.1, width)
        for b, o in (("rot_brach", 3), ("trn_branch", 3)):
            sd[f"{b}.weight"] = rng.normal(0, 3.0, (o, width))
            sd[f"{b}.bias"] = rng.normal(0, 0.5, o)
        if i > 0:
            sd["nr_branch.weight"] = rng.normal(0, 3.0, (1, width))
            sd["nr_branch.bias"] = rng.normal(0, 0.5, 1)
        levels.append({k: v.astype(np.float32) for k, v in sd.items()})
    x = rng.uniform(-1.5, 1.5, (3001, 3)).astype(np.float32)
    y, data = ndp.warp(levels, x)
    ry, rdata = oracle.ndp_warp(levels, x)
    assert np.abs(ry - x).max() > 1e-3          # the warp is not the identity
    np.testing.assert_allclose(y.cpu().numpy(), ry, rtol=0, atol=1e-5)
    for i in range(m):
        np.testing.assert_allclose(data[i][0].cpu().numpy(), rdata[i][0], rtol=0, atol=1e-5)


def test_ndp_warp_level_range_and_torch_modules():
    """max_level/min_level as Deformation_Pyramid.warp; modules accepted."""
    z, levels = _golden_levels()
    y_all, d_all = ndp.warp(levels, z["ndp/x"])
    y01, d01 = ndp.warp(levels, z["ndp/x"], max_level=1)
    np.testing.assert_array_equal(y01.cpu().numpy(), d_all[1][0].cpu().numpy())
    y2, _ = ndp.warp(levels, d_all[1][0], min_level=2)
    np.testing.assert_allclose(y2.cpu().numpy(), y_all.cpu().numpy(), rtol=0, atol=1e-6)
    mods = []
    for i, sd in enumerate(levels):
        m = torch.nn.Module()
        m.state_dict = (lambda sd=sd: {k: torch.from_numpy(v) for k, v in sd.items()})
        m.m, m.k0, m.motion, m.rotation_format = i + 1, -8, "SE3", "axis_angle"
        mods.append(m)
    ym, _ = ndp.warp(mods, z["ndp/x"])
    np.testing.assert_array_equal(ym.cpu().numpy(), y_all.cpu().numpy())
