"""GPU parity of the registration path (a5-a9) against the CPU oracle.

Bar: bit-exact -- feature NN indices, correspondence sets, RANSAC/ICP 4x4
transforms (raw f64 bits), fitness / inlier_rmse (raw bits), iteration and
validation counts, inlier masks.  Known-answer RRE/RTE checks pin the restated
Open3D semantics to ground truth (Open3D itself is absent: parity vs the
reference's RANSAC/ICP is unpinned)."""
import numpy as np
import pytest
import torch

from pointcloudregistration_amd import registration as reg
from pointcloudregistration_amd import synth

pytestmark = pytest.mark.gpu


def _np(t):
    return t.detach().cpu().numpy()


def _bits_equal(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()


@pytest.mark.parametrize("n,m,d,noise", [(1000, 1100, 32, 1.0), (777, 640, 33, 0.8),
                                         (2048, 2048, 64, 1.2), (300, 5000, 8, 0.5)])
def test_feature_match_bitexact_vs_oracle(oracle, n, m, d, noise):
    rng = np.random.default_rng(n + m)
    code = rng.standard_normal((max(n, m) * 2, d)).astype(np.float32)
    fs = (code[rng.permutation(len(code))[:n]] + rng.normal(0, noise, (n, d))).astype(np.float32)
    ft = (code[rng.permutation(len(code))[:m]] + rng.normal(0, noise, (m, d))).astype(np.float32)
    nn12, nn21 = reg.feature_match(fs[None], ft[None])
    assert np.array_equal(_np(nn12)[0], oracle.featnn(fs, ft))
    assert np.array_equal(_np(nn21)[0], oracle.featnn(ft, fs))


def test_feature_match_ties_and_duplicates(oracle):
    """Exact duplicate descriptors force the ambiguous-row exact rescan path;
    the lowest index must win (the oracle's rule)."""
    rng = np.random.default_rng(5)
    base = rng.standard_normal((200, 32)).astype(np.float32)
    ft = base[rng.integers(0, 200, 1500)]            # many exact duplicates
    fs = base[rng.integers(0, 200, 900)] + np.float32(1e-7)
    nn12, nn21 = reg.feature_match(fs[None], ft[None])
    assert np.array_equal(_np(nn12)[0], oracle.featnn(fs, ft))
    assert np.array_equal(_np(nn21)[0], oracle.featnn(ft, fs))


def test_feature_match_vs_reference_vote_semantics():
    """vote.get_coor_points (c2p-net/ngenet/models/vote.py:6-9) = argmin of
    torch.cdist; on untied float64 distances it must agree."""
    rng = np.random.default_rng(9)
    fs = rng.standard_normal((1500, 32)).astype(np.float32)
    ft = rng.standard_normal((1300, 32)).astype(np.float32)
    ref = torch.cdist(torch.from_numpy(fs).double(), torch.from_numpy(ft).double()).min(-1)[1]
    nn12, _ = reg.feature_match(fs[None], ft[None])
    assert np.array_equal(_np(nn12)[0], ref.numpy())


def test_feature_match_ragged_batch(oracle):
    P, N, M, D = 3, 700, 650, 32
    rng = np.random.default_rng(3)
    fs = rng.standard_normal((P, N, D)).astype(np.float32)
    ft = rng.standard_normal((P, M, D)).astype(np.float32)
    ns = np.array([700, 1, 333], np.int32)
    nt = np.array([650, 400, 17], np.int32)
    nn12, nn21 = reg.feature_match(fs, ft, ns, nt)
    for p in range(P):
        assert np.array_equal(_np(nn12)[p, :ns[p]], oracle.featnn(fs[p, :ns[p]], ft[p, :nt[p]]))
        assert np.array_equal(_np(nn21)[p, :nt[p]], oracle.featnn(ft[p, :nt[p]], fs[p, :ns[p]]))


@pytest.mark.parametrize("mutual", [True, False])
def test_correspondences_vs_oracle(oracle, mutual):
    rng = np.random.default_rng(1)
    P, N, M = 2, 900, 800
    nn12 = rng.integers(0, M, (P, N)).astype(np.int32)
    nn21 = rng.integers(0, N, (P, M)).astype(np.int32)
    for p in range(P):  # plant mutual pairs
        js = rng.permutation(M)[:300]
        nn21[p, js] = np.arange(300)
        nn12[p, :300] = js
    co, nc = reg.correspondences(nn12, nn21, mutual_filter=mutual)
    for p in range(P):
        exp = oracle.corres(nn12[p], nn21[p], mutual, 3)
        assert _np(nc)[p] == len(exp)
        assert np.array_equal(_np(co)[p, :len(exp)], exp)


def _synthetic_batch(P, n, noise=1.0, seed0=1000):
    return synth.make_batch(P, n=n, m=n, d=32, base_seed=seed0, feat_noise=noise)


@pytest.mark.parametrize("noise,n", [(1.0, 2048), (0.8, 4096), (1.2, 1500)])
def test_ransac_bitexact_vs_oracle(oracle, noise, n):
    P = 3
    B = _synthetic_batch(P, n, noise)
    prm = reg.RansacParams(max_correspondence_distance=0.04, seed=123)
    res = reg.register_feature_ransac_batch(B.src, B.tgt, B.src_feat, B.tgt_feat, prm,
                                            pair_ids=np.arange(P, dtype=np.int32) + 50)
    T, fit, rmse = _np(res.transformation), _np(res.fitness), _np(res.inlier_rmse)
    st, ct, mk = _np(res.stats), _np(res.corr_tgt), _np(res.inlier_mask)
    for p in range(P):
        nn12 = oracle.featnn(B.src_feat[p], B.tgt_feat[p])
        nn21 = oracle.featnn(B.tgt_feat[p], B.src_feat[p])
        co = oracle.corres(nn12, nn21, True, 3)
        r = oracle.ransac(B.src[p], B.tgt[p], co, 0.04, seed=123, pair_id=50 + p)
        assert st[p, 3] == 1 and r["found"] == 1
        assert _bits_equal(T[p], r["T"]), f"pair {p}: T differs\n{T[p]}\n{r['T']}"
        assert _bits_equal(fit[p], r["fitness"]) and _bits_equal(rmse[p], r["inlier_rmse"])
        assert (st[p, 0], st[p, 1], st[p, 2]) == (r["iters"], r["validated"], r["best_itr"])
        cs = r["correspondence_set"]
        assert st[p, 4] == len(cs)
        got = np.nonzero(ct[p] >= 0)[0]
        assert np.array_equal(got, cs[:, 0]) and np.array_equal(ct[p, got], cs[:, 1])
        bits = np.unpackbits(mk[p].view(np.uint8), bitorder="little")[:n].astype(bool)
        assert np.array_equal(np.nonzero(bits)[0], cs[:, 0])
        rre, rte = synth.rre_rte(T[p, :3, :3], T[p, :3, 3], B.R[p], B.t[p])
        assert rre < 5.0 and rte < 0.05


def test_ransac_no_checkers_and_small_inputs(oracle):
    B = _synthetic_batch(2, 600, 0.9, seed0=77)
    prm = reg.RansacParams(max_correspondence_distance=0.05, edge_length_ratio=-1,
                           distance_check=-1, ransac_n=4, max_iteration=500, seed=9,
                           mutual_filter=False)
    res = reg.register_feature_ransac_batch(B.src, B.tgt, B.src_feat, B.tgt_feat, prm)
    for p in range(2):
        nn12 = oracle.featnn(B.src_feat[p], B.tgt_feat[p])
        co = np.stack([np.arange(600), nn12], 1).astype(np.int32)
        r = oracle.ransac(B.src[p], B.tgt[p], co, 0.05, ransac_n=4, edge_ratio=-1, dist_check=-1,
                          max_iteration=500, seed=9, pair_id=p)
        assert _bits_equal(_np(res.transformation)[p], r["T"])
        assert _np(res.stats)[p, 0] == r["iters"]


def test_ransac_invalid_inputs_return_identity():
    src = np.random.default_rng(0).random((1, 10, 3)).astype(np.float32)
    corres = np.zeros((1, 10, 2), np.int32)
    prm = reg.RansacParams(max_correspondence_distance=0.05)
    res = reg.ransac_batch(src, src, corres, np.array([2], np.int32), prm)  # K < ransac_n
    assert np.array_equal(_np(res.transformation)[0], np.eye(4))
    assert _np(res.stats)[0, 3] == -1 and _np(res.fitness)[0] == 0.0


@pytest.mark.parametrize("r,noise_init", [(0.02, 0.01), (0.05, 0.03)])
def test_icp_bitexact_vs_oracle(oracle, r, noise_init):
    P, n = 3, 3000
    B = _synthetic_batch(P, n, 1.0, seed0=500)
    init = np.zeros((P, 4, 4))
    rng = np.random.default_rng(4)
    for p in range(P):
        Rp = synth.rotation_xyz(*rng.normal(0, noise_init, 3)) @ B.R[p]
        init[p, :3, :3] = Rp
        init[p, :3, 3] = B.t[p] + rng.normal(0, noise_init, 3)
        init[p, 3, 3] = 1
    res = reg.icp_batch(B.src, B.tgt, init, reg.IcpParams(r))
    for p in range(P):
        o = oracle.icp(B.src[p], B.tgt[p], r, init=init[p])
        assert _bits_equal(_np(res.transformation)[p], o["T"])
        assert _bits_equal(_np(res.fitness)[p], o["fitness"])
        assert _bits_equal(_np(res.inlier_rmse)[p], o["inlier_rmse"])
        assert tuple(_np(res.stats)[p]) == (o["iters"], o["n_corr"])
        assert int((_np(res.corr_tgt)[p] >= 0).sum()) == o["n_corr"]


@pytest.mark.parametrize("P", [2, 300])
def test_icp_correspondence_reuse_stress(oracle, P):
    """The sweep reuses a point's last correspondence while its clearance bound
    certifies it (icp.hip CorrState).  Adversarial inputs for that certificate: a
    lattice target with exact duplicate points (ties broken by the lowest index),
    sources on the lattice's mid-planes (near-equidistant targets), and 30 full
    iterations of ever smaller motion (relative criteria 0).  P = 2: G > 1
    workgroups per pair; P = 300: one workgroup per pair plus the tail launch."""
    rng = np.random.default_rng(11)
    g = np.stack(np.meshgrid(*[np.arange(12)] * 3, indexing="ij"), -1).reshape(-1, 3) * 0.01
    n = 1500
    S = np.zeros((P, n, 3), np.float32)
    T = np.zeros((P, g.shape[0] + 64, 3), np.float32)
    init = np.zeros((P, 4, 4))
    for p in range(P):
        t = g + rng.normal(0, 0.0005 if p % 2 else 0.0, g.shape)
        t = np.concatenate([t, t[rng.choice(len(t), 64, replace=False)]])  # exact duplicates
        T[p] = t
        s = t[rng.choice(len(t), n)] + 0.005 * (rng.random((n, 3)) < 0.3)  # some on mid-planes
        S[p] = s + rng.normal(0, 0.002, s.shape)
        init[p, :3, :3] = synth.rotation_xyz(*rng.normal(0, 0.01, 3))
        init[p, :3, 3] = rng.normal(0, 0.004, 3)
        init[p, 3, 3] = 1
    prm = reg.IcpParams(0.012, relative_fitness=0.0, relative_rmse=0.0, max_iteration=30)
    res = reg.icp_batch(S, T, init, prm)
    for p in list(range(min(P, 4))) + [P - 1]:
        o = oracle.icp(S[p], T[p], 0.012, init=init[p], relative_fitness=0.0, relative_rmse=0.0)
        assert _bits_equal(_np(res.transformation)[p], o["T"]), p
        assert _bits_equal(_np(res.fitness)[p], o["fitness"]), p
        assert _bits_equal(_np(res.inlier_rmse)[p], o["inlier_rmse"]), p
        assert tuple(_np(res.stats)[p]) == (o["iters"], o["n_corr"]), p


@pytest.mark.parametrize("P", [2, 260])
def test_icp_hbm_grid_vs_oracle(oracle, P):
    """Targets too large for the LDS grid copy (M = 12,000: the walks read the
    HBM grid, GridView) through the correspondence-reuse sweep, at G > 1 (P = 2)
    and one workgroup per pair with the tail launch (P = 260): bit-exact."""
    n, m = 2500, 12000
    B = synth.make_batch(P, n=n, m=m, d=4, base_seed=900, feat_noise=1.0)
    init = np.zeros((P, 4, 4))
    rng = np.random.default_rng(8)
    for p in range(P):
        init[p, :3, :3] = synth.rotation_xyz(*rng.normal(0, 0.01, 3)) @ B.R[p]
        init[p, :3, 3] = B.t[p] + rng.normal(0, 0.005, 3)
        init[p, 3, 3] = 1
    res = reg.icp_batch(B.src, B.tgt, init, reg.IcpParams(0.02))
    for p in list(range(min(P, 3))) + [P - 1]:
        o = oracle.icp(B.src[p], B.tgt[p], 0.02, init=init[p])
        assert _bits_equal(_np(res.transformation)[p], o["T"]), p
        assert _bits_equal(_np(res.fitness)[p], o["fitness"]), p
        assert _bits_equal(_np(res.inlier_rmse)[p], o["inlier_rmse"]), p
        assert tuple(_np(res.stats)[p]) == (o["iters"], o["n_corr"]), p


def test_radius_nn_vs_oracle_bruteforce(oracle):
    rng = np.random.default_rng(2)
    tgt = (rng.random((2, 3000, 3)) * 2 - 1).astype(np.float32)
    tgt[1, 100:110] = tgt[1, 5]          # exact duplicates -> lowest index
    q = rng.random((2, 4000, 3)) * 2 - 1
    q[1, :50] = tgt[1, 5].astype(np.float64)
    idx, d2 = reg.radius_nn(tgt, q, 0.07)
    for p in range(2):
        ei, ed = oracle.radius_nn(tgt[p], q[p], 0.07, use_grid=False)
        assert np.array_equal(_np(idx)[p], ei)
        hit = ei >= 0
        assert _bits_equal(_np(d2)[p][hit], ed[hit])


def test_open3d_facade_known_answer():
    B = _synthetic_batch(1, 4096, 1.0, seed0=31)
    src, tgt = reg.PointCloud(B.src[0]), reg.PointCloud(B.tgt[0])
    fs, ft = reg.Feature(B.src_feat[0].T), reg.Feature(B.tgt_feat[0].T)
    d = 0.04
    res = reg.registration_ransac_based_on_feature_matching(
        src, tgt, fs, ft, True, d, reg.TransformationEstimationPointToPoint(False), 3,
        [reg.CorrespondenceCheckerBasedOnEdgeLength(0.9), reg.CorrespondenceCheckerBasedOnDistance(d)],
        reg.RANSACConvergenceCriteria(100000, 0.999))
    icp = reg.registration_icp(src, tgt, 0.02, res.transformation,
                               reg.TransformationEstimationPointToPoint())
    rre, rte = synth.rre_rte(icp.transformation[:3, :3], icp.transformation[:3, 3], B.R[0], B.t[0])
    assert rre < 0.5 and rte < 0.01
    assert len(icp.correspondence_set) > 1000 and 0 < icp.inlier_rmse < 0.02
    R, t = reg.register(B.src[0], B.tgt[0], B.src_feat[0], B.tgt_feat[0], d)
    assert np.array_equal(R, res.transformation[:3, :3])


def test_procrustes_bitexact_vs_oracle(oracle):
    from pointcloudregistration_amd import procrustes as pr
    rng = np.random.default_rng(0)
    B, N = 5, 1000
    src = rng.standard_normal((B, N, 3)).astype(np.float32)
    tgt = rng.standard_normal((B, N, 3)).astype(np.float32)
    w = rng.random((B, N)).astype(np.float32)
    for absw, eps in ((0, 1e-8), (1, 1e-4)):
        T = pr.procrustes_batch(src, tgt, w, absw, eps)
        assert _bits_equal(_np(T), oracle.procrustes_batch(src, tgt, w, absw, eps))


def _stress_cases():
    rng = np.random.default_rng(77)
    cases = {}
    # per-dimension magnitudes over 9 decades
    sc = (10.0 ** rng.uniform(-6, 3, 32)).astype(np.float32)
    cases["dynamic_range"] = ((rng.standard_normal((900, 32)) * sc).astype(np.float32),
                              (rng.standard_normal((1000, 32)) * sc).astype(np.float32))
    # far from the origin, tiny spread: nearly every row is ambiguous -> rescan
    base = rng.standard_normal(32).astype(np.float32) * 1000
    cases["offset"] = ((base + rng.standard_normal((600, 32)) * 1e-3).astype(np.float32),
                       (base + rng.standard_normal((700, 32)) * 1e-3).astype(np.float32))
    # zero rows and repeated rows
    a = rng.standard_normal((500, 32)).astype(np.float32)
    a[::7] = 0
    b = rng.standard_normal((450, 32)).astype(np.float32)
    b[::5] = 0
    b[1::9] = a[3]
    cases["zeros_repeats"] = (a, b)
    cases["d1"] = (rng.standard_normal((513, 1)).astype(np.float32),
                   rng.standard_normal((300, 1)).astype(np.float32))
    cases["d100_fallback"] = (rng.standard_normal((400, 100)).astype(np.float32),
                              rng.standard_normal((333, 100)).astype(np.float32))
    cases["subnormal"] = ((rng.standard_normal((300, 16)) * 1e-39).astype(np.float32),
                          (rng.standard_normal((280, 16)) * 1e-39).astype(np.float32))
    a = rng.standard_normal((400, 32)).astype(np.float32)
    b = rng.standard_normal((380, 32)).astype(np.float32)
    a[5, 3] = np.nan                  # NaN query row: every distance NaN -> index 0
    b[[7, 100], 0] = np.nan           # NaN candidates never win (strict <)
    cases["nan_rows"] = (a, b)
    return cases


@pytest.mark.parametrize("name", list(_stress_cases()))
def test_feature_match_stress_vs_oracle(oracle, name):
    """Screen + certification + rescan stay exact on adversarial descriptors:
    the f16x3 split screen (D <= 64) and the f32 fallback (d100_fallback)."""
    fs, ft = _stress_cases()[name]
    nn12, nn21 = reg.feature_match(fs[None], ft[None])
    assert np.array_equal(_np(nn12)[0], oracle.featnn(fs, ft))
    assert np.array_equal(_np(nn21)[0], oracle.featnn(ft, fs))


def test_feature_match_many_pairs_xcd_mapping(oracle):
    """P not a multiple of 8 exercises the XCD-aware block->pair map's idle blocks."""
    P, N, M, D = 11, 300, 260, 32
    rng = np.random.default_rng(11)
    fs = rng.standard_normal((P, N, D)).astype(np.float32)
    ft = rng.standard_normal((P, M, D)).astype(np.float32)
    nn12, nn21 = reg.feature_match(fs, ft)
    for p in range(P):
        assert np.array_equal(_np(nn12)[p], oracle.featnn(fs[p], ft[p]))
        assert np.array_equal(_np(nn21)[p], oracle.featnn(ft[p], fs[p]))


def test_ragged_batches_equal_per_pair_runs(oracle):
    """Pairs with n_src != n_tgt padded into one batch give each pair's own result
    (regression: per-call count tensors must stay alive across the launch)."""
    sizes = [(1200, 1100), (900, 1300), (1500, 1500), (700, 1000)]
    S = np.zeros((4, 1500, 3), np.float32)
    G = np.zeros((4, 1500, 3), np.float32)
    FS = np.zeros((4, 1500, 16), np.float32)
    FG = np.zeros((4, 1500, 16), np.float32)
    T0 = np.tile(np.eye(4), (4, 1, 1))
    for p, (n, m) in enumerate(sizes):
        b = synth.make_pair(70 + p, n, m, 16, feat_noise=0.3)
        S[p, :n], G[p, :m], FS[p, :n], FG[p, :m] = b[0], b[1], b[2], b[3]
        T0[p, :3, :3], T0[p, :3, 3] = b[4], b[5] + 0.005
    ns = np.array([s[0] for s in sizes], np.int32)
    nt = np.array([s[1] for s in sizes], np.int32)
    prm = reg.RansacParams(max_correspondence_distance=0.04, seed=3)
    rb = reg.register_feature_ransac_batch(S, G, FS, FG, prm, n_src=ns, n_tgt=nt,
                                           pair_ids=np.arange(4, dtype=np.int32))
    ib = reg.icp_batch(S, G, T0, reg.IcpParams(max_correspondence_distance=0.02), n_src=ns, n_tgt=nt)
    for p, (n, m) in enumerate(sizes):
        r1 = reg.register_feature_ransac_batch(S[p:p + 1, :n], G[p:p + 1, :m], FS[p:p + 1, :n],
                                               FG[p:p + 1, :m], prm,
                                               pair_ids=np.array([p], np.int32))
        assert torch.equal(rb.transformation[p], r1.transformation[0]), p
        assert rb.fitness[p].item() == r1.fitness[0].item(), p
        i1 = reg.icp_batch(S[p:p + 1, :n], G[p:p + 1, :m], T0[p:p + 1],
                           reg.IcpParams(max_correspondence_distance=0.02))
        assert torch.equal(ib.transformation[p], i1.transformation[0]), p
        assert np.array_equal(ib.correspondence_set(p), i1.correspondence_set(0)), p
        o = oracle.icp(S[p, :n], G[p, :m], 0.02, T0[p])
        assert np.array_equal(o["T"], _np(ib.transformation[p]))
