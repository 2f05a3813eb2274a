"""GPU: pcr_feature_correspondences, the mutual feature matching without nn21
for every target (csrc/featnn.hip featnn_row7: the rows screened with their
argmin, the targets some source picked screened for top-2 values only, each
candidate decided from certified values or the exact column rescan).

Bar: bit-exact -- nn12, n_corres and the correspondence set equal the oracle's
corres(featnn(F, G), featnn(G, F)) (Open3D 0.13's mutual filter with the exact
f64 1-NN, DataPreparation/RANSAC.py:43-52) and the two-call path
correspondences(*feature_match(...)), on the adversarial cases of the feature
screen (ties, duplicates, NaN rows, 9-decade ranges, offsets, subnormals)."""
import numpy as np
import pytest

from pointcloudregistration_amd import registration as reg
from pointcloudregistration_amd import synth

pytestmark = pytest.mark.gpu


def _np(t):
    return t.detach().cpu().numpy()


def _cases():
    rng = np.random.default_rng(123)
    c = {}
    B = synth.make_batch(1, n=4096, m=4096, d=32, base_seed=77, feat_noise=1.0)
    c["synthetic_4096"] = (B.src_feat[0], B.tgt_feat[0])
    B = synth.make_batch(1, n=3000, m=2500, d=32, base_seed=78, feat_noise=0.3)
    c["clean_3000x2500"] = (B.src_feat[0], B.tgt_feat[0])
    base = rng.standard_normal((300, 32)).astype(np.float32)
    # exact duplicate SOURCE rows: a column's winner is tied between them -> the
    # lowest index is mutual, the others not (undecidable from values: rescan)
    c["dup_rows"] = (base[rng.integers(0, 300, 1400)], base[rng.integers(0, 300, 1100)]
                     + np.float32(1e-6))
    c["dup_both"] = (base[rng.integers(0, 300, 900)], base[rng.integers(0, 300, 1500)])
    sc = (10.0 ** rng.uniform(-6, 3, 32)).astype(np.float32)
    c["dynamic_range"] = ((rng.standard_normal((900, 32)) * sc).astype(np.float32),
                          (rng.standard_normal((1000, 32)) * sc).astype(np.float32))
    off = rng.standard_normal(32).astype(np.float32) * 1000
    c["offset"] = ((off + rng.standard_normal((600, 32)) * 1e-3).astype(np.float32),
                   (off + rng.standard_normal((700, 32)) * 1e-3).astype(np.float32))
    a = rng.standard_normal((500, 32)).astype(np.float32)
    a[::7] = 0
    b = rng.standard_normal((450, 32)).astype(np.float32)
    b[::5] = 0
    b[1::9] = a[3]
    c["zeros_repeats"] = (a, b)
    a = rng.standard_normal((400, 32)).astype(np.float32)
    b = rng.standard_normal((380, 32)).astype(np.float32)
    a[5, 3] = np.nan
    a[0, :] = np.nan
    b[[0, 7, 100], 0] = np.nan
    c["nan_rows"] = (a, b)
    # twin targets a few ulps from each source row: the screen cannot order a
    # twin pair, so its argmin (J is built from it, beside the exact row rescan)
    # is often the exact loser, and the exact winner is in no other row's J
    a = rng.standard_normal((600, 32)).astype(np.float32)
    tw = np.repeat(a, 2, axis=0) + (rng.standard_normal((1200, 32)) * 1e-6).astype(np.float32)
    c["near_twins"] = (a, np.concatenate([tw, rng.standard_normal((100, 32)).astype(np.float32)]))
    c["subnormal"] = ((rng.standard_normal((300, 16)) * 1e-39).astype(np.float32),
                      (rng.standard_normal((280, 16)) * 1e-39).astype(np.float32))
    # the packs' speculative scale (feat_sample: the first 64 rows' max with one
    # binade of headroom): a tail far above the sample takes the repair path,
    # one far below it only loses precision; NaN / inf past the sample
    a = rng.standard_normal((700, 32)).astype(np.float32)
    b = rng.standard_normal((650, 32)).astype(np.float32)
    a[:80] *= np.float32(1e-3)
    b[:65] *= np.float32(1e-3)
    c["tail_above_sample"] = (a, b)
    a = rng.standard_normal((700, 32)).astype(np.float32)
    b = rng.standard_normal((650, 32)).astype(np.float32)
    a[:32] *= np.float32(1e4)
    c["tail_below_sample"] = (a, b)
    a = rng.standard_normal((600, 32)).astype(np.float32)
    b = rng.standard_normal((500, 32)).astype(np.float32)
    a[400, 7] = np.nan
    b[300, 1] = np.inf
    c["nonfinite_past_sample"] = (a, b)
    c["d1"] = (rng.standard_normal((513, 1)).astype(np.float32),
               rng.standard_normal((300, 1)).astype(np.float32))
    c["d33_small"] = (rng.standard_normal((40, 33)).astype(np.float32),
                      rng.standard_normal((7, 33)).astype(np.float32))
    c["d64"] = (rng.standard_normal((1200, 64)).astype(np.float32),
                rng.standard_normal((1100, 64)).astype(np.float32))
    c["d100_f32"] = (rng.standard_normal((400, 100)).astype(np.float32),
                     rng.standard_normal((333, 100)).astype(np.float32))
    return c


CASES = _cases()


@pytest.mark.parametrize("mutual", [True, False])
@pytest.mark.parametrize("name", list(CASES))
def test_feature_correspondences_vs_oracle(oracle, name, mutual):
    fs, ft = CASES[name]
    co, nc, nn12 = reg.feature_correspondences(fs[None], ft[None], mutual_filter=mutual)
    e12 = oracle.featnn(fs, ft)
    exp = oracle.corres(e12, oracle.featnn(ft, fs), mutual, 3)
    assert np.array_equal(_np(nn12)[0], e12)
    assert int(_np(nc)[0]) == len(exp)
    assert np.array_equal(_np(co)[0, :len(exp)], exp)
    # == the two-call path
    a12, a21 = reg.feature_match(fs[None], ft[None])
    co2, nc2 = reg.correspondences(a12, a21, mutual_filter=mutual)
    assert int(_np(nc2)[0]) == len(exp) and np.array_equal(_np(co2)[0, :len(exp)], exp)


def test_feature_correspondences_ragged_many_pairs(oracle):
    """11 pairs (not a multiple of 8: idle blocks of the XCD map), ragged counts
    incl. a 1-row source and a 17-row target, both passes' row lists."""
    P, N, M, D = 11, 700, 650, 32
    rng = np.random.default_rng(3)
    code = rng.standard_normal((P, 900, D)).astype(np.float32)
    fs = np.stack([code[p, rng.permutation(900)[:N]] for p in range(P)]) + \
        rng.normal(0, 0.7, (P, N, D)).astype(np.float32)
    ft = np.stack([code[p, rng.permutation(900)[:M]] for p in range(P)]) + \
        rng.normal(0, 0.7, (P, M, D)).astype(np.float32)
    fs, ft = fs.astype(np.float32), ft.astype(np.float32)
    ns = np.array([700, 1, 333, 700, 650, 20, 699, 512, 513, 64, 300], np.int32)
    nt = np.array([650, 400, 17, 650, 1, 650, 640, 511, 512, 65, 299], np.int32)
    co, nc, nn12 = reg.feature_correspondences(fs, ft, ns, nt)
    for p in range(P):
        f, g = fs[p, :ns[p]], ft[p, :nt[p]]
        e12 = oracle.featnn(f, g)
        exp = oracle.corres(e12, oracle.featnn(g, f), True, 3)
        assert np.array_equal(_np(nn12)[p, :ns[p]], e12), p
        assert int(_np(nc)[p]) == len(exp), p
        assert np.array_equal(_np(co)[p, :len(exp)], exp), p


@pytest.mark.parametrize("d", [32, 24])
def test_feature_correspondences_repair_mixed_batch(oracle, d):
    """20 pairs, 11 of them with rows far above their sample's range (the packs'
    repair path: flagged pairs by rank over kRepairR blocks, ranks past 8
    included), D = 32 (register pack) and 24 (LDS pack): every pair equals the
    oracle."""
    P, N, M = 20, 400, 380
    rng = np.random.default_rng(9)
    fs = rng.standard_normal((P, N, d)).astype(np.float32)
    ft = rng.standard_normal((P, M, d)).astype(np.float32)
    flagged = [0, 2, 3, 5, 8, 9, 11, 13, 16, 18, 19]
    for p in flagged:
        fs[p, 64 + p:] *= np.float32(200.0) if p % 2 else np.float32(1.0)
        ft[p, 100:] *= np.float32(300.0)
    co, nc, nn12 = reg.feature_correspondences(fs, ft)
    for p in range(P):
        e12 = oracle.featnn(fs[p], ft[p])
        exp = oracle.corres(e12, oracle.featnn(ft[p], fs[p]), True, 3)
        assert np.array_equal(_np(nn12)[p], e12), p
        assert int(_np(nc)[p]) == len(exp), p
        assert np.array_equal(_np(co)[p, :len(exp)], exp), p


def _twins(rng, n, d, sep, twin_src):
    """Near-tie descriptors for the 1-term screen: every target has a twin
    `sep` away (relative ~1e-3 of a distance: inside the 1-term f16 screen's
    error bound, far outside the 3-term split's), so the row screen cannot
    order the twins and leaves nearly every row to the 3-term screen; with
    twin_src the sources are twinned too, which does the same to the columns
    of pass 2."""
    a = rng.standard_normal((n, d)).astype(np.float32)
    b = (a + 0.5 * rng.standard_normal((n, d))).astype(np.float32)
    tw = (b + sep * rng.standard_normal((n, d))).astype(np.float32)
    ft = np.concatenate([b, tw])[rng.permutation(2 * n)]
    if twin_src:
        a = np.concatenate([a, (a + sep * rng.standard_normal((n, d))).astype(np.float32)])
    return a, ft


@pytest.mark.parametrize("twin_src", [False, True])
def test_one_term_fallback_near_ties(oracle, monkeypatch, twin_src):
    """The 1-term screens' fallback (featnn_row8<.., kOne = false> over the rows
    and J columns the 1-term screens could not certify) on near-tie descriptors:
    the fallback runs (pcr_featnn_fallback_rows), and nn12 / the mutual set are
    bit-exact vs the oracle and equal the 3-term-only path (PCR_FEAT_ONE=0)."""
    from pointcloudregistration_amd import _lib
    rng = np.random.default_rng(61)
    fs, ft = _twins(rng, 700, 32, 1e-2, twin_src)
    _lib.featnn_fallback_rows(reset=True)
    co, nc, nn12 = reg.feature_correspondences(fs[None], ft[None])
    r12, c21 = _lib.featnn_fallback_rows(reset=True)
    assert r12 > len(fs) // 2, r12
    if twin_src:
        assert c21 > 0, c21
    e12 = oracle.featnn(fs, ft)
    exp = oracle.corres(e12, oracle.featnn(ft, fs), True, 3)
    assert np.array_equal(_np(nn12)[0], e12)
    assert int(_np(nc)[0]) == len(exp)
    assert np.array_equal(_np(co)[0, :len(exp)], exp)
    monkeypatch.setenv("PCR_FEAT_ONE", "0")
    co3, nc3, nn3 = reg.feature_correspondences(fs[None], ft[None])
    assert _lib.featnn_fallback_rows(reset=True) == (0, 0)
    assert np.array_equal(_np(nn3), _np(nn12)) and int(_np(nc3)[0]) == len(exp)
    assert np.array_equal(_np(co3)[0, :len(exp)], exp)


@pytest.mark.parametrize("name", ["synthetic_4096", "dup_rows", "dynamic_range", "offset", "nan_rows",
                                  "near_twins", "subnormal", "tail_above_sample", "d1"])
def test_feature_correspondences_three_term_only(oracle, monkeypatch, name):
    """The round-5 path (the 3-term split screens alone, PCR_FEAT_ONE=0) stays
    bit-exact: it is what the 1-term screens fall back to."""
    monkeypatch.setenv("PCR_FEAT_ONE", "0")
    fs, ft = CASES[name]
    co, nc, nn12 = reg.feature_correspondences(fs[None], ft[None])
    e12 = oracle.featnn(fs, ft)
    exp = oracle.corres(e12, oracle.featnn(ft, fs), True, 3)
    assert np.array_equal(_np(nn12)[0], e12)
    assert int(_np(nc)[0]) == len(exp)
    assert np.array_equal(_np(co)[0, :len(exp)], exp)


def _used_flags(P, Nmax, Mmax):
    """featmut_jbuild / featmut_resolve's per-column flags of the last
    pcr_feature_correspondences call (its scratch, pcr_featmut_debug_copy):
    [P][Mmax + 1] ints after v12 (f64) | e12 (f32) | wq (float4, 16-aligned)."""
    import torch
    from pointcloudregistration_amd import _lib
    off = ((12 * P * Nmax + 15) // 16) * 16 + 16 * P * Mmax
    n = P * (Mmax + 1)
    buf = torch.empty(off + 4 * n, dtype=torch.uint8, device="cuda")
    _lib.call("pcr_featmut_debug_copy", buf.data_ptr(), buf.numel(), _lib.stream_handle())
    torch.cuda.synchronize()
    return _np(buf[off:].view(torch.int32)).reshape(P, Mmax + 1)


@pytest.mark.parametrize("P", [1, 192])
def test_resolve_outside_j(oracle, P):
    """featmut_resolve's branch for a rescanned row whose exact argmin is outside
    J (J is built from the screened argmins, beside the exact row rescan, which
    runs on a side stream at P >= 192): near-twin targets make the screened
    argmin the exact loser for about half the rows.  The branch runs (columns
    flagged 3 in the resolve's scratch) at P = 1 and at P = 192, and every pair
    is bit-exact vs the oracle."""
    rng = np.random.default_rng(500 + P)
    N, K, D = 160, 20, 32
    M = 2 * N + K
    fs = rng.standard_normal((P, N, D)).astype(np.float32)
    ft = np.empty((P, M, D), np.float32)
    for p in range(P):
        tw = np.repeat(fs[p], 2, axis=0) + (rng.standard_normal((2 * N, D)) * 1e-6).astype(np.float32)
        ft[p] = np.concatenate([tw, rng.standard_normal((K, D)).astype(np.float32)])[rng.permutation(M)]
    co, nc, nn12 = reg.feature_correspondences(fs, ft)
    used = _used_flags(P, N, M)
    outside = (used[:, :M] == 3).sum(axis=1)
    assert outside.min() > 0, outside
    nn12, nc, co = _np(nn12), _np(nc), _np(co)
    for p in range(P):
        e12 = oracle.featnn(fs[p], ft[p])
        exp = oracle.corres(e12, oracle.featnn(ft[p], fs[p]), True, 3)
        assert np.array_equal(nn12[p], e12), p
        assert int(nc[p]) == len(exp), p
        assert np.array_equal(co[p, :len(exp)], exp), p


def test_mutual_mmax_16383(oracle):
    """Mmax = 16383: J's build no longer fits its LDS form beside the block
    scan's static LDS (4 (Mmax + 1) + 64 > 64 KB) and takes the HBM form."""
    rng = np.random.default_rng(16383)
    fs = rng.standard_normal((300, 32)).astype(np.float32)
    ft = rng.standard_normal((16383, 32)).astype(np.float32)
    ft[:300] = fs + (0.1 * rng.standard_normal((300, 32))).astype(np.float32)
    co, nc, nn12 = reg.feature_correspondences(fs[None], ft[None])
    e12 = oracle.featnn(fs, ft)
    exp = oracle.corres(e12, oracle.featnn(ft, fs), True, 3)
    assert np.array_equal(_np(nn12)[0], e12)
    assert int(_np(nc)[0]) == len(exp)
    assert np.array_equal(_np(co)[0, :len(exp)], exp)


def test_row9_path_runs_and_row8_path_equal(oracle, monkeypatch):
    """The shipped 1-term passes are featnn_row9 + featnn_regroup9 (the regroup's
    profile slot counts its two launches, one per pass); PCR_FEAT_ROW9=0 selects
    the round-6 featnn_row8 1-term passes, which give the same nn12 and set."""
    from pointcloudregistration_amd import _lib
    fs, ft = CASES["synthetic_4096"]
    _lib.profile_enable(True)
    _lib.profile_read(_lib.PROF_FEAT_REGROUP, reset=True)
    co, nc, nn12 = reg.feature_correspondences(fs[None], ft[None])
    _, launches = _lib.profile_read(_lib.PROF_FEAT_REGROUP, reset=True)
    _lib.profile_enable(False)
    assert launches == 2, launches
    monkeypatch.setenv("PCR_FEAT_ROW9", "0")
    co8, nc8, nn8 = reg.feature_correspondences(fs[None], ft[None])
    e12 = oracle.featnn(fs, ft)
    exp = oracle.corres(e12, oracle.featnn(ft, fs), True, 3)
    for c, n, nn in ((co, nc, nn12), (co8, nc8, nn8)):
        assert np.array_equal(_np(nn)[0], e12)
        assert int(_np(n)[0]) == len(exp)
        assert np.array_equal(_np(c)[0, :len(exp)], exp)


@pytest.mark.parametrize("name", ["dup_rows", "dynamic_range", "near_twins", "nan_rows", "d1"])
def test_feature_correspondences_row8_one_term(oracle, monkeypatch, name):
    """The featnn_row8 1-term passes (PCR_FEAT_ROW9=0) stay bit-exact."""
    monkeypatch.setenv("PCR_FEAT_ROW9", "0")
    fs, ft = CASES[name]
    co, nc, nn12 = reg.feature_correspondences(fs[None], ft[None])
    e12 = oracle.featnn(fs, ft)
    exp = oracle.corres(e12, oracle.featnn(ft, fs), True, 3)
    assert np.array_equal(_np(nn12)[0], e12)
    assert int(_np(nc)[0]) == len(exp)
    assert np.array_equal(_np(co)[0, :len(exp)], exp)


def test_colterm_bias_per_pair(oracle):
    """featnn_row9's column terms ct = f32(|y|^2 + B) with B the pair's power of
    two above BOTH clouds' max |x|^2 (feat_colterms, csrc/featnn.hip): pairs whose
    clouds differ by decades in norm (B set by the rows in pass 1, by the columns
    in pass 2), a single huge-norm row, an all-zero target cloud but one row (B
    near 1), tiny descriptors (the pair scale lifts them) -- in one batch, every
    pair equal to the oracle."""
    P, N, M, D = 6, 600, 550, 32
    rng = np.random.default_rng(21)
    code = rng.standard_normal((P, 800, D)).astype(np.float32)
    fs = np.stack([code[p, rng.permutation(800)[:N]] for p in range(P)]) + \
        rng.normal(0, 0.6, (P, N, D)).astype(np.float32)
    ft = np.stack([code[p, rng.permutation(800)[:M]] for p in range(P)]) + \
        rng.normal(0, 0.6, (P, M, D)).astype(np.float32)
    fs, ft = fs.astype(np.float32), ft.astype(np.float32)
    fs[1] *= np.float32(1000.0)
    ft[2] *= np.float32(1000.0)
    fs[3, 17] *= np.float32(1e4)
    ft[4] = 0.0
    ft[4, 5] = fs[4, 9]
    fs[5] *= np.float32(1e-20)
    ft[5] *= np.float32(1e-20)
    co, nc, nn12 = reg.feature_correspondences(fs, ft)
    for p in range(P):
        e12 = oracle.featnn(fs[p], ft[p])
        exp = oracle.corres(e12, oracle.featnn(ft[p], fs[p]), True, 3)
        assert np.array_equal(_np(nn12)[p], e12), p
        assert int(_np(nc)[p]) == len(exp), p
        assert np.array_equal(_np(co)[p, :len(exp)], exp), p
