"""f2 on the GPU: pcr_grid_subsample / pcr_radius_* through the drop-in
mirrors of cpp_subsampling.subsample_batch / cpp_neighbors.batch_query against
the reference (compiled from its sources into oracle/_ref when present, the
committed golden vectors otherwise) and the oracle restatement.

Bar: subsampled points, lengths and features bit-identical, in the reference's
order; neighbour rows bit-identical, except that exactly equal distances may
appear in another order (nanoflann's traversal order; tie-aware comparison in
the duplicate-point cases, documented in DESIGN.md f2)."""
import os

import numpy as np
import pytest
import torch

from kpconv_cases import NB_CASES, SUB_CASES, nb_case, sub_case

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def K():
    from pointcloudregistration_amd import kpconv
    return kpconv


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(ROOT, "tests", "golden", "kpconv_golden.npz"))


@pytest.fixture(scope="module")
def map_order():
    from pointcloudregistration_amd import _lib

    def order(keys):
        k = np.ascontiguousarray(keys, np.uint64)
        o = np.zeros(len(k), np.int32)
        _lib.call("pcr_voxel_map_order", k.ctypes.data, len(k), o.ctypes.data)
        return o
    return order


def _ref():
    import ref_kpconv
    return ref_kpconv if ref_kpconv.available() else None


def _d32(qi, S):
    d = (qi - S).astype(np.float32)
    return (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]


def _rows_equal_up_to_ties(a, b, q, s):
    assert a.shape == b.shape
    ns = s.shape[0]
    for i in np.nonzero((a != b).any(1))[0]:
        ra, rb = a[i][a[i] < ns], b[i][b[i] < ns]
        assert len(ra) == len(rb) and set(ra.tolist()) == set(rb.tolist()), i
        assert np.array_equal(_d32(q[i], s[ra]), _d32(q[i], s[rb])), i


@pytest.mark.parametrize("name", SUB_CASES)
def test_subsample_golden(K, golden, name):
    c = sub_case(name)
    res = K.subsample_batch(c["points"], c["batches"], features=c["features"], sampleDl=c["dl"],
                            max_p=c["max_p"])
    assert isinstance(res[0], np.ndarray)
    assert np.array_equal(res[0], golden[f"{name}/points"])
    assert np.array_equal(res[1], golden[f"{name}/lengths"])
    if c["features"] is not None:
        assert np.array_equal(res[2], golden[f"{name}/features"])


@pytest.mark.parametrize("name", NB_CASES)
def test_batch_query_golden(K, golden, name):
    c = nb_case(name)
    out = K.batch_query(c["queries"], c["supports"], c["q_batches"], c["s_batches"], radius=c["radius"])
    ref = golden[f"{name}/neighbors"]
    if name == "nb_dups":
        _rows_equal_up_to_ties(out, ref, c["queries"], c["supports"])
    else:
        assert np.array_equal(out, ref)


def test_subsample_random_against_reference(K, oracle, map_order):
    R = _ref()
    rng = np.random.default_rng(21)
    for t in range(16):
        nb = int(rng.integers(1, 5))
        sizes = rng.integers(1, 20000, nb)
        p = np.concatenate([(rng.standard_normal((s, 3)) * rng.uniform(0.05, 20)).astype(np.float32)
                            + rng.uniform(-500, 500, 3).astype(np.float32) for s in sizes])
        f = rng.standard_normal((p.shape[0], int(rng.integers(1, 5)))).astype(np.float32)
        dl = float(np.float32(rng.uniform(0.01, 3.0)))
        mp = int(rng.choice([0, 0, 0, 25, 1000]))
        got = K.subsample_batch(p, sizes, features=f, sampleDl=dl, max_p=mp)
        want = (R.subsample_batch(p, sizes, features=f, sampleDl=dl, max_p=mp) if R else
                oracle.grid_subsample(p, sizes, dl, features=f, max_p=mp, order=map_order))
        for x, y in zip(got, want):
            assert np.array_equal(x, y), t


def test_subsample_large_against_oracle(K, oracle, map_order):
    """BASELINE-scale clouds (the ngenet first layer): 2 x 150k points."""
    rng = np.random.default_rng(3)
    p = np.concatenate([rng.uniform(-1, 1, (150000, 3)), rng.uniform(-1.2, 0.9, (150000, 3))]).astype(np.float32)
    f = rng.standard_normal((300000, 3)).astype(np.float32)
    got = K.subsample_batch(p, [150000, 150000], features=f, sampleDl=0.03)
    want = oracle.grid_subsample(p, [150000, 150000], 0.03, features=f, order=map_order)
    for x, y in zip(got, want):
        assert np.array_equal(x, y)


def test_subsample_device_tensors_and_dataloader_api(K):
    c = sub_case("sub_two_clouds")
    P = torch.from_numpy(c["points"]).cuda()
    F = torch.from_numpy(c["features"]).cuda()
    sp, sl, sf = K.subsample_batch(P, c["batches"], features=F, sampleDl=c["dl"])
    assert sp.is_cuda and sf.is_cuda
    hp, hl, hf = K.subsample_batch(c["points"], c["batches"], features=c["features"], sampleDl=c["dl"])
    assert np.array_equal(sp.cpu().numpy(), hp) and np.array_equal(sf.cpu().numpy(), hf)
    tp, tl, tf = K.batch_grid_subsampling(torch.from_numpy(c["points"]),
                                          torch.tensor(c["batches"], dtype=torch.int32),
                                          features=torch.from_numpy(c["features"]), sampleDl=c["dl"])
    assert isinstance(tp, torch.Tensor) and not tp.is_cuda
    assert np.array_equal(tp.numpy(), hp) and np.array_equal(tl.numpy(), hl)


def test_subsample_edges(K, oracle, map_order):
    from pointcloudregistration_amd import PcrError
    # trailing points beyond the batches are ignored (batch_grid_subsampling :140-145)
    p = np.random.default_rng(0).uniform(0, 1, (500, 3)).astype(np.float32)
    got = K.subsample_batch(p, [300], sampleDl=0.2)
    want = oracle.grid_subsample(p[:300], [300], 0.2, order=map_order)
    assert np.array_equal(got[0], want[0])
    # an empty cloud (the reference divides by zero there) yields no points
    got = K.subsample_batch(p, [0, 300, 0], sampleDl=0.2)
    assert got[1].tolist() == [0, want[1][0], 0] and np.array_equal(got[0], want[0])
    q = p.copy()
    q[7, 1] = np.nan
    with pytest.raises(PcrError):
        K.subsample_batch(q, [500], sampleDl=0.2)
    with pytest.raises(PcrError):
        K.subsample_batch(p, [600], sampleDl=0.2)
    with pytest.raises(RuntimeError, match="Error"):
        K.subsample_batch(p[:0], [0], sampleDl=0.2)
    with pytest.raises(RuntimeError, match="method"):
        K.subsample_batch(p, [500], sampleDl=0.2, method="centroids")


def test_batch_query_random_against_reference(K, oracle):
    R = _ref()
    rng = np.random.default_rng(8)
    for t in range(8):
        nb = int(rng.integers(1, 4))
        ss = rng.integers(1, 8000, nb)
        qs = rng.integers(1, 4000, nb)
        s = np.concatenate([rng.uniform(-1, 1, (k, 3)) for k in ss]).astype(np.float32)
        q = np.concatenate([rng.uniform(-1.1, 1.1, (k, 3)) for k in qs]).astype(np.float32)
        r = float(rng.uniform(0.02, 0.25))
        try:
            want = (R.batch_query(q, s, qs, ss, radius=r) if R else
                    oracle.radius_neighbors(q, s, qs, ss, r)[0])
        except RuntimeError:
            want = np.zeros((0, 0), np.int32)
        if want.size == 0:
            # no query has a neighbour: the reference wrapper raises "Error"
            # (cpp_neighbors/wrapper.cpp:201-205), and so does the drop-in
            with pytest.raises(RuntimeError, match="Error"):
                K.batch_query(q, s, qs, ss, radius=r)
            continue
        got = K.batch_query(q, s, qs, ss, radius=r)
        assert np.array_equal(got, want), t


def test_batch_query_ties_against_reference(K):
    """Quantised clouds: most rows hold equal distances, whose order is the
    reference's nanoflann leaf-visit order through std::sort (replayed on the host)."""
    R = _ref()
    if R is None:
        pytest.skip("oracle/_ref/libref_kpconv.so not available")
    rng = np.random.default_rng(9)
    for t in range(5):
        nb = int(rng.integers(1, 4))
        ss = rng.integers(1, 6000, nb)
        qs = rng.integers(1, 3000, nb)
        s = np.concatenate([np.round(rng.uniform(-1, 1, (k, 3)) * 16) / 16 for k in ss]).astype(np.float32)
        q = np.concatenate([np.round(rng.uniform(-1.1, 1.1, (k, 3)) * 16) / 16 for k in qs]).astype(np.float32)
        r = float(rng.uniform(0.1, 0.3))
        try:
            want = R.batch_query(q, s, qs, ss, radius=r)
        except RuntimeError:
            continue
        got = K.batch_query(q, s, qs, ss, radius=r)
        assert np.array_equal(got, want), t
        got7 = K.batch_neighbors(q, s, qs, ss, r, 7).numpy()
        assert np.array_equal(got7, want[:, :7]), t


def test_batch_neighbors_truncation_and_device(K):
    c = nb_case("nb_self")
    full = K.batch_query(c["queries"], c["supports"], c["q_batches"], c["s_batches"], radius=c["radius"])
    t = K.batch_neighbors(torch.from_numpy(c["queries"]).cuda(), torch.from_numpy(c["supports"]).cuda(),
                          torch.tensor(c["q_batches"]), torch.tensor(c["s_batches"]), c["radius"], 7)
    assert t.is_cuda and t.shape == (full.shape[0], min(7, full.shape[1]))
    assert np.array_equal(t.cpu().numpy(), full[:, :7])
    h = K.batch_neighbors(c["queries"], c["supports"], c["q_batches"], c["s_batches"], c["radius"], 0)
    assert not h.is_cuda and np.array_equal(h.numpy(), full)


def test_batch_query_edges(K):
    from pointcloudregistration_amd import PcrError
    rng = np.random.default_rng(2)
    s = rng.uniform(-1, 1, (1000, 3)).astype(np.float32)
    q = rng.uniform(-1, 1, (50, 3)).astype(np.float32)
    # NaN / inf supports and queries never match (d < r2 is false)
    s2 = s.copy()
    s2[3] = np.nan
    s2[4, 0] = np.inf
    q2 = q.copy()
    q2[0] = np.nan
    got = K.batch_query(q2, s2, [50], [1000], radius=0.3)
    import oracle as O
    want, _ = O.radius_neighbors(q2, s2, [50], [1000], 0.3)
    assert np.array_equal(got, want)
    # points far beyond the integer cell range take the all-supports path
    s3 = s.copy()
    s3[10] = [3e9, 0, 0]
    q3 = q.copy()
    q3[1] = [3e9, 0, 0.1]
    got = K.batch_query(q3, s3, [50], [1000], radius=0.3)
    want, _ = O.radius_neighbors(q3, s3, [50], [1000], 0.3)
    assert np.array_equal(got, want)
    # negative radius: r2 = radius^2 (neighbors.cpp :226)
    assert np.array_equal(K.batch_query(q, s, [50], [1000], radius=-0.2),
                          K.batch_query(q, s, [50], [1000], radius=0.2))
    # no neighbour anywhere -> the wrappers' RuntimeError("Error")
    with pytest.raises(RuntimeError, match="Error"):
        K.batch_query(q + 100, s, [50], [1000], radius=0.01)
    with pytest.raises(RuntimeError, match="Wrong number"):
        K.batch_query(q, s, [50], [500, 500], radius=0.1)
    # the reference's batch walk misassigns queries after a middle empty batch
    with pytest.raises(PcrError):
        K.batch_query(q, s, [25, 0, 25], [300, 300, 400], radius=0.1)
    with pytest.raises(PcrError):
        K.batch_query(q, s, [40], [1000], radius=0.1)


def test_collate_pyramid_against_reference(K):
    """The collate_fn layer loop (dataloader.py:116-167), threedmatch blocks."""
    R = _ref()
    if R is None:
        pytest.skip("oracle/_ref/libref_kpconv.so not available")
    sys_path = os.path.join(ROOT, "tools")
    import sys
    sys.path.insert(0, sys_path)
    from kpconv_bench import ARCH, fragment
    rng = np.random.default_rng(4)
    src, tgt = fragment(rng, 6000), fragment(rng, 5000)
    pts = np.concatenate([src, tgt])
    nrm = rng.standard_normal(pts.shape).astype(np.float32)
    lens = np.array([6000, 5000], np.int32)
    got = K.pyramid(torch.from_numpy(pts).cuda(), lens, torch.from_numpy(nrm).cuda(), ARCH, 0.025,
                    2.5, [30, 30, 30, 30])
    want = R.pyramid(pts, lens, nrm, ARCH, 0.025, 2.5, [30, 30, 30, 30])
    for k in ("points", "normals", "pools", "neighbors", "upsamples", "stacked_lengths"):
        assert len(got[k]) == len(want[k]), k
        for x, y in zip(got[k], want[k]):
            x = x.cpu().numpy() if isinstance(x, torch.Tensor) else x
            assert np.array_equal(x, y), k
    # the dict-level mirror
    items = [dict(src_points=src, tgt_points=tgt, src_points_raw=src, tgt_points_raw=tgt,
                  src_feats=np.ones((6000, 1), np.float32), tgt_feats=np.ones((5000, 1), np.float32),
                  src_normals=nrm[:6000], tgt_normals=nrm[6000:], transf=np.eye(4), coors=np.zeros((3, 2)))]

    class Cfg:
        architecture, first_subsampling_dl, conv_radius = ARCH, 0.025, 2.5
    d = K.collate_fn(items, Cfg, [30, 30, 30, 30])
    assert np.array_equal(d["neighbors"][2].numpy(), want["neighbors"][2])
    assert d["feats"].shape == (11000, 1) and d["transf"].shape == (1, 4, 4)
