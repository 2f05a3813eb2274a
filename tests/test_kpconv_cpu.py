"""f2 (KPConv grid subsampling / radius neighbours), CPU side: the oracle
restatement against the reference's golden vectors and, when it was built here,
against the compiled reference itself; the host replay of the reference's
unordered_map emission order (pcr_voxel_map_order, host-only, no GPU)."""
import os

import numpy as np
import pytest

from kpconv_cases import NB_CASES, SUB_CASES, nb_case, sub_case

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(ROOT, "tests", "golden", "kpconv_golden.npz"))


@pytest.fixture(scope="module")
def map_order():
    from pointcloudregistration_amd import _lib
    _lib.load()

    def order(keys):
        k = np.ascontiguousarray(keys, np.uint64)
        o = np.zeros(len(k), np.int32)
        _lib.call("pcr_voxel_map_order", k.ctypes.data, len(k), o.ctypes.data)
        return o
    return order


def _ref():
    import ref_kpconv
    if not ref_kpconv.available():
        pytest.skip("oracle/_ref/libref_kpconv.so not built (needs /root/reference)")
    return ref_kpconv


@pytest.mark.parametrize("name", SUB_CASES)
def test_oracle_subsample_matches_golden(oracle, golden, map_order, name):
    c = sub_case(name)
    res = oracle.grid_subsample(c["points"], c["batches"], c["dl"], features=c["features"],
                                max_p=c["max_p"], order=map_order)
    assert np.array_equal(res[0], golden[f"{name}/points"])
    assert np.array_equal(res[1], golden[f"{name}/lengths"])
    if c["features"] is not None:
        assert np.array_equal(res[2], golden[f"{name}/features"])


def _tie_groups_equal(a, b, q, s, dist_fn):
    """Rows equal up to the order of exactly equal distances (nanoflann's
    traversal order is not reproducible)."""
    if a.shape != b.shape:
        return False
    if np.array_equal(a, b):
        return True
    ns = s.shape[0]
    for i in np.nonzero((a != b).any(1))[0]:
        ra, rb = a[i][a[i] < ns], b[i][b[i] < ns]
        if len(ra) != len(rb) or set(ra) != set(rb):
            return False
        da, db = dist_fn(q[i], s[ra]), dist_fn(q[i], s[rb])
        if not np.array_equal(da, db):
            return False
    return True


def _d32(qi, S):
    d = (qi - S).astype(np.float32)
    return (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]


@pytest.mark.parametrize("name", NB_CASES)
def test_oracle_neighbors_matches_golden(oracle, golden, name):
    c = nb_case(name)
    out, _ = oracle.radius_neighbors(c["queries"], c["supports"], c["q_batches"], c["s_batches"],
                                     c["radius"])
    ref = golden[f"{name}/neighbors"]
    if name == "nb_dups":
        assert _tie_groups_equal(out, ref, c["queries"], c["supports"], _d32)
    else:
        assert np.array_equal(out, ref)


def test_voxel_map_order_against_reference_random(oracle, map_order):
    R = _ref()
    rng = np.random.default_rng(7)
    for _ in range(12):
        n1, n2 = rng.integers(1, 6000, 2)
        p = (rng.standard_normal((n1 + n2, 3)) * rng.uniform(0.1, 10)).astype(np.float32)
        p += rng.uniform(-100, 100, 3).astype(np.float32)
        f = rng.standard_normal((n1 + n2, 2)).astype(np.float32)
        dl = float(np.float32(rng.uniform(0.02, 2.0)))
        mp = int(rng.choice([0, 0, 37]))
        a = R.subsample_batch(p, [n1, n2], features=f, sampleDl=dl, max_p=mp)
        b = oracle.grid_subsample(p, [n1, n2], dl, features=f, max_p=mp, order=map_order)
        for x, y in zip(a, b):
            assert np.array_equal(x, y)


def test_voxel_map_order_rehash_sizes(map_order):
    """Bucket growth is where the iteration order gets intricate: sweep the
    voxel count across several rehash points against the compiled reference."""
    R = _ref()
    rng = np.random.default_rng(11)
    for v in (1, 2, 11, 12, 13, 23, 24, 47, 48, 97, 98, 199, 200, 409, 823, 1741, 3739):
        cells = rng.choice(200 ** 3, v, replace=False)
        ijk = np.stack(np.unravel_index(cells, (200, 200, 200)), 1).astype(np.float32)
        p = ((ijk + 0.5) * np.float32(0.25)).astype(np.float32)
        p = p[rng.permutation(v)]
        a = R.subsample_batch(p, [v], sampleDl=0.25)
        import oracle as O
        b = O.grid_subsample(p, [v], 0.25, order=map_order)
        assert np.array_equal(a[0], b[0]), v


def test_reference_neighbors_random_against_oracle(oracle):
    R = _ref()
    rng = np.random.default_rng(5)
    for _ in range(4):
        n = int(rng.integers(200, 3000))
        s = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
        q = rng.uniform(-1, 1, (n // 3, 3)).astype(np.float32)
        r = float(rng.uniform(0.05, 0.3))
        a = R.batch_query(q, s, [n // 3], [n], radius=r)
        b, _ = oracle.radius_neighbors(q, s, [n // 3], [n], r)
        assert np.array_equal(a, b)
