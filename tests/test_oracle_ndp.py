"""a10 oracle (numpy f64 restatement of NDPLayer.forward / Deformation_Pyramid.warp)
pinned to the reference's own warp output (tests/golden/make_golden_py.py:
torch.manual_seed(3), depth 3, width 32, m 3, axis_angle, SE3, nonrigidity on
levels > 0, weights x3).  The reference computes in f32: 1e-6 absolute."""
import os

import numpy as np

HERE = os.path.dirname(__file__)


def test_ndp_oracle_matches_reference_golden(oracle):
    z = np.load(os.path.join(HERE, "golden", "ndp_golden.npz"))
    levels = [{k[len(f"ndp/l{i}/"):]: z[k] for k in z.files if k.startswith(f"ndp/l{i}/")}
              for i in range(3)]
    y, data = oracle.ndp_warp(levels, z["ndp/x"])
    np.testing.assert_allclose(y, z["ndp/y"], rtol=0, atol=1e-6)
    for i in range(3):
        np.testing.assert_allclose(data[i][0], z[f"ndp/level{i}"], rtol=0, atol=1e-6)
    for i in (1, 2):
        np.testing.assert_allclose(data[i][1], z[f"ndp/nonrigid{i}"], rtol=0, atol=1e-7)
    assert data[0][1] is None
    assert np.abs(z["ndp/y"] - z["ndp/x"]).max() > 1e-2  # far from identity
