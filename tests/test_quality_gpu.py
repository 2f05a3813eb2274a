"""GPU: f3 consumers (QualityCheck Chamfer / Hausdorff, ROPNet overlap labels) and
the preprocess_correspondences producer, against the reference's own formulas
(sklearn / scipy / the ROPNet torch expression, run here on the CPU)."""
import numpy as np
import pytest
import torch

from pointcloudregistration_amd import formats, quality, registration as reg, synth

pytestmark = pytest.mark.gpu


def _pair(seed, n=3000, m=2500):
    rng = np.random.default_rng(seed)
    a = synth.surface_points(rng, n).astype(np.float32)
    b = (synth.surface_points(rng, m) + rng.normal(0, 0.01, (m, 3))).astype(np.float32)
    return a, b


def test_qualitycheck_chamfer_matches_sklearn():
    from sklearn.neighbors import NearestNeighbors
    a, b = _pair(1)
    # QualityCheck.py:25-31 verbatim in behaviour
    x_nn = NearestNeighbors(n_neighbors=1, leaf_size=1, algorithm="kd_tree", metric="l2").fit(a)
    y_nn = NearestNeighbors(n_neighbors=1, leaf_size=1, algorithm="kd_tree", metric="l2").fit(b)
    want = np.mean(y_nn.kneighbors(a)[0]) + np.mean(x_nn.kneighbors(b)[0])
    got = quality.chamfer_distance(reg.PointCloud(a), reg.PointCloud(b))
    # f32 squared distances (nnd contract) vs sklearn's f64: relative 1e-6
    assert abs(got - want) <= 1e-6 * want


def test_qualitycheck_hausdorff_matches_scipy():
    from scipy.spatial.distance import directed_hausdorff
    a, b = _pair(2)
    want = max(directed_hausdorff(a.astype(np.float64), b.astype(np.float64))[0],
               directed_hausdorff(b.astype(np.float64), a.astype(np.float64))[0])
    got = quality.hausdorff_distance(reg.PointCloud(a), reg.PointCloud(b))
    assert abs(got - want) <= 1e-6 * want


def test_ropnet_overlap_masks_match_square_dists():
    rng = np.random.default_rng(3)
    B, N, M = 4, 717, 690
    src = torch.from_numpy(rng.uniform(-1, 1, (B, N, 3)).astype(np.float32))
    tgt = torch.from_numpy(rng.uniform(-1, 1, (B, M, 3)).astype(np.float32))
    # ROPNet/src/utils/process.py:14-27 on the CPU
    dists = (torch.sum(src ** 2, -1).view(B, N, 1) + torch.sum(tgt ** 2, -1).view(B, 1, M)
             - 2 * torch.matmul(src, tgt.permute(0, 2, 1)))
    thr = 0.05 * 0.05
    w1, w2 = torch.min(dists, -1)[0], torch.min(dists, 1)[0]
    g1, g2 = quality.min_square_dists(src.cuda(), tgt.cuda())
    # expanded vs direct form: |diff| within a few f32 ulps of |p|^2 scale
    assert torch.allclose(g1.cpu(), w1, atol=2e-6) and torch.allclose(g2.cpu(), w2, atol=2e-6)
    m1, m2 = quality.overlap_masks(src.cuda(), tgt.cuda(), 0.05)
    border1 = (w1 - thr).abs() < 2e-6
    border2 = (w2 - thr).abs() < 2e-6
    assert torch.equal(m1.cpu()[~border1], (w1 < thr)[~border1])
    assert torch.equal(m2.cpu()[~border2], (w2 < thr)[~border2])
    assert m1.any() and (~m1).any()


def test_preprocess_correspondences_batched_icp(oracle):
    """dip/preprocess_correspondences.py:45-58 for ragged pairs in one launch ==
    the per-pair drop-in call (and the oracle's correspondence count)."""
    rng = np.random.default_rng(4)
    data = {"source": [], "target": [], "transformation": []}
    for p, (n, m) in enumerate([(1200, 1100), (900, 1300), (1500, 1500)]):
        b = synth.make_pair(50 + p, n, m, 4)
        src, tgt, R, t = b[0], b[1], b[4], b[5]
        T = np.eye(4)
        T[:3, :3], T[:3, 3] = R, t
        T[:3, 3] += rng.normal(0, 0.01, 3)          # an imperfect stored transformation
        data["source"].append(src.astype(np.float64))
        data["target"].append(tgt.astype(np.float64))
        data["transformation"].append(T)
    corrs = formats.icp_correspondences(data, 0.03)
    for p in range(3):
        r = reg.registration_icp(data["source"][p], data["target"][p], 0.03, data["transformation"][p],
                                 reg.TransformationEstimationPointToPoint())
        assert np.array_equal(corrs[p], r.correspondence_set), p
        o = oracle.icp(data["source"][p].astype(np.float32), data["target"][p].astype(np.float32),
                       0.03, data["transformation"][p])
        assert len(corrs[p]) == o["n_corr"] > 0
