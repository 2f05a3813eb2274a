"""C3 composed (dip/demo.py:64-178) on the GPU vs the oracle chain at the demo's
size: two mm-scale clouds down-sampled at 1.0 (~8-10k points), 2048 samples
each, LRF patches (kernel 3*sqrt(3), 256 points), the descriptor network
(PointNetFeature's architecture with a seeded random init; the
trained weights are not part of this build), the 5th-percentile filter and feature RANSAC at 1.5.

Bar: voxel means, sample indices and patches bit-exact vs oracle; RANSAC T
bit-exact vs the oracle's RANSAC on the same (filtered) points/descriptors."""
import numpy as np
import pytest
import torch

from pointcloudregistration_amd import dip, synth

pytestmark = pytest.mark.gpu


def _pair(seed):
    rng = np.random.default_rng(seed)
    U = synth.surface_points(rng, 60000) * 40.0
    R = synth.rotation_xyz(*np.deg2rad(rng.uniform(-30, 30, 3)))
    t = rng.uniform(-10, 10, 3)
    src = U[rng.permutation(60000)[:40000]] + rng.normal(0, 0.05, (40000, 3))
    tgt = (U[rng.permutation(60000)[:40000]] + rng.normal(0, 0.05, (40000, 3))) @ R.T + t
    return src, tgt, R, t


def test_c3_demo_flow_vs_oracle_chain(oracle):
    src, tgt, R, t = _pair(31)
    torch.manual_seed(1)
    net = dip.PointNetFeature(64).cuda().eval()
    np.random.seed(5)
    out = dip.demo_register(src, tgt, net, seed=3)
    ker, ps = 3.0 * np.sqrt(3.0), 256

    np.random.seed(5)
    clouds = []
    for raw, pcd, col in ((src, out["pcd1"], dip.GREY), (tgt, out["pcd2"], dip.BLUE)):
        d, _, c = oracle.voxel_down_sample(raw, 1.0, colors=np.tile(col, (len(raw), 1)))
        assert np.asarray(pcd.points).tobytes() == d.tobytes()
        assert np.asarray(pcd.colors).tobytes() == c.tobytes()
        clouds.append(d)
    assert 2048 < len(clouds[0]) < 20000
    i1 = np.random.choice(len(clouds[0]), 2048, replace=False)
    i2 = np.random.choice(len(clouds[1]), 2048, replace=False)
    assert np.array_equal(i1, out["inds1"]) and np.array_equal(i2, out["inds2"])
    qs = (clouds[0][i1], clouds[1][i2])
    got = (out["patches1"].cpu().numpy(), out["patches2"].cpu().numpy())
    for i in range(2048):
        for p in range(2):
            cnt = oracle.lrf_count(clouds[p], qs[p][i], ker)
            inds = np.random.choice(max(cnt, ps), ps, replace=False)
            _, patch, _ = oracle.lrf(clouds[p], qs[p][i], ker, ps, inds)
            assert got[p][i].tobytes() == np.ascontiguousarray(patch.T).tobytes(), (i, p)

    g1, g2 = out["good1"], out["good2"]
    assert np.array_equal(g1, dip.percentile_keep(_mx(net, out["patches1"]), 5))
    assert np.array_equal(g2, dip.percentile_keep(_mx(net, out["patches2"]), 5))
    a = qs[0][g1].astype(np.float32)
    b = qs[1][g2].astype(np.float32)
    fa, fb = out["desc1"][g1].astype(np.float32), out["desc2"][g2].astype(np.float32)
    co = oracle.corres(oracle.featnn(fa, fb), oracle.featnn(fb, fa), True, 3)
    r = oracle.ransac(a, b, co, 1.5, dist_check=1.5, seed=3, pair_id=0)
    res = out["result"]
    assert res.transformation.tobytes() == r["T"].tobytes()
    assert np.array_equal(np.asarray(res.correspondence_set), r["correspondence_set"])


def _mx(net, patches):
    with torch.no_grad():
        return torch.cat([net(patches[s:s + 500].float())[1] for s in range(0, len(patches), 500)]
                         ).double().cpu().numpy()

