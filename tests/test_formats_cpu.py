"""CPU: the RANSAC dataset dict (DataPreparation/RANSAC.py:102-131) and the
correspondence file layout (dip/preprocess_correspondences.py:48-58)."""
import numpy as np

from pointcloudregistration_amd import formats
from pointcloudregistration_amd.registration import RegistrationResult


def test_ransac_dataset_schema_filter_and_pickle_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    clouds = [rng.uniform(size=(n, 3)) for n in (1500, 1200, 900)]
    normals = [rng.standard_normal((len(c), 3)) for c in clouds]
    res = [RegistrationResult(np.eye(4) * (i + 1), np.stack([np.arange(k), np.arange(k)], 1), 0.9,
                              0.01 * (i + 1))
           for i, k in enumerate((1200, 999, 1000))]
    d = formats.ransac_dataset(clouds, clouds, normals, normals, res)
    assert tuple(d) == formats.RANSAC_KEYS
    assert len(d["source"]) == 2                     # the 999-correspondence pair is dropped
    assert d["inlier_ratio"] == [1200 / 1500, 1000 / 900]
    assert d["inlier_rmse"] == [0.01, 0.03]
    p = tmp_path / "RANSACTrainoriginal.pickle"
    formats.save_pickle(p, d)
    back = formats.load_pickle(p)
    assert back.keys() == d.keys()
    for k in d:
        for x, y in zip(back[k], d[k]):
            assert np.array_equal(np.asarray(x), np.asarray(y))


def test_correspondence_file_npz_fallback(tmp_path):
    corrs = [np.array([[0, 1], [2, 3]], np.int32), np.zeros((0, 2), np.int32),
             np.arange(20, dtype=np.int32).reshape(10, 2)]
    path = formats.save_correspondences(tmp_path / "train.npz", corrs)
    back = formats.load_correspondences(path)
    assert len(back) == 3 and all(np.array_equal(a, b) for a, b in zip(back, corrs))
