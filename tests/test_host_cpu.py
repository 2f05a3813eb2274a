"""CPU: host-side logic of the registration façade (no compute calls)."""
import numpy as np
import torch

from pointcloudregistration_amd import registration as reg


def test_feature_rows_only_transposes_feature_objects():
    """Open3D Feature.data is (dim, num) and is transposed; raw (N, D) ndarrays and
    tensors -- which carry a `.data` attribute of their own -- pass through."""
    a = np.arange(100 * 33, dtype=np.float32).reshape(100, 33)
    assert reg._feature_rows(a).shape == (100, 33)
    t = torch.from_numpy(a)
    assert tuple(reg._feature_rows(t).shape) == (100, 33)
    f = reg.Feature(a.T.copy())
    assert np.array_equal(reg._feature_rows(f), a)
    ft = reg.Feature(t.t())
    assert torch.equal(reg._feature_rows(ft), t)
    assert reg._feature_rows([[1.0, 2.0]]).shape == (1, 2)


def test_ransac_params_from_open3d_objects():
    prm = reg._ransac_params_from_o3d(
        0.04, reg.TransformationEstimationPointToPoint(False), 3,
        [reg.CorrespondenceCheckerBasedOnEdgeLength(0.9),
         reg.CorrespondenceCheckerBasedOnDistance(0.04)],
        reg.RANSACConvergenceCriteria(100000, 0.999), True, 7)
    c = prm.to_c()
    assert (c.edge_length_ratio, c.distance_check, c.max_iteration, c.ransac_n) == (0.9, 0.04, 100000, 3)
    assert c.mutual_filter == 1 and c.seed == 7
