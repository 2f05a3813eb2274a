"""GPU parity of the nndistance drop-in (a1/a2) against the oracle and the
reference's golden vectors.  Bar: bit-exact (distances compared as raw f32
bits, indices exactly, gradients as raw bits)."""
import hashlib

import numpy as np
import pytest
import torch

from nnd_cases import CASES, make_inputs

pytestmark = pytest.mark.gpu


def _gpu(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _run_fwd_bwd(x1, x2, gd1, gd2):
    from pointcloudregistration_amd import nndistance as nd
    t1, t2 = _gpu(x1), _gpu(x2)
    d1, d2, i1, i2 = nd.nnd_with_index(t1, t2)
    g1 = torch.empty_like(t1)
    g2 = torch.empty_like(t2)
    nd.nnd_backward_cuda(t1, t2, g1, g2, _gpu(gd1), _gpu(gd2), i1, i2)
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in (d1, d2, i1, i2, g1, g2)]


def assert_bitexact(got, exp, what):
    """Bit-exact for every non-NaN float, exact NaN positions (NaN sign/payload
    bits are platform NaN-propagation detail and are not compared), exact ints."""
    assert got.shape == exp.shape, what
    if got.dtype == np.float32:
        gn, en = np.isnan(got), np.isnan(exp)
        assert np.array_equal(gn, en), f"{what}: NaN positions differ ({(gn != en).sum()})"
        bad = (got.view(np.uint32) != exp.view(np.uint32)) & ~gn
        assert not bad.any(), f"{what}: {bad.sum()} of {bad.size} values differ"
    else:
        bad = got != exp
        assert not bad.any(), f"{what}: {bad.sum()} of {bad.size} entries differ"


ALGOS = ["auto", "brute", "grid"]  # PCR_NND_ALGO: size rule / forced brute force / forced grid


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("name", sorted(CASES))
def test_nnd_bitexact_vs_reference_golden(golden_nnd, monkeypatch, name, algo):
    monkeypatch.setenv("PCR_NND_ALGO", algo)
    x1, x2, gd1, gd2 = make_inputs(CASES[name])
    got = _run_fwd_bwd(x1, x2, gd1, gd2)
    keys = ("d1", "d2", "i1", "i2", "g1", "g2")
    if f"{name}/d1" in golden_nnd:  # full reference outputs stored
        for k, g in zip(keys, got):
            assert_bitexact(g, golden_nnd[f"{name}/{k}"], f"{name}/{k}")
        return
    d1, d2, i1, i2, g1, g2 = got
    h = hashlib.sha256()
    for a in (d1, d2, i1, i2):
        h.update(a.tobytes())
    assert h.digest() == bytes(golden_nnd[f"{name}/sha_fwd"]), name
    h = hashlib.sha256()
    h.update(g1.tobytes())
    h.update(g2.tobytes())
    assert h.digest() == bytes(golden_nnd[f"{name}/sha_bwd"]), name


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("b,n,m", [(1, 333, 4097), (3, 8192, 100), (64, 700, 900), (2, 3000, 5000)])
def test_nnd_bitexact_vs_oracle(oracle, monkeypatch, b, n, m, algo):
    monkeypatch.setenv("PCR_NND_ALGO", algo)
    rng = np.random.default_rng(b * 7 + n)
    x1 = (rng.random((b, n, 3), dtype=np.float32) * 2 - 1).astype(np.float32)
    x2 = (rng.random((b, m, 3), dtype=np.float32) * 2 - 1).astype(np.float32)
    gd1 = rng.standard_normal((b, n)).astype(np.float32)
    gd2 = rng.standard_normal((b, m)).astype(np.float32)
    got = _run_fwd_bwd(x1, x2, gd1, gd2)
    e1, e2, j1, j2 = oracle.nnd_forward(x1, x2)
    eg1, eg2 = oracle.nnd_backward(x1, x2, gd1, gd2, j1, j2)
    for k, g, e in zip(("d1", "d2", "i1", "i2", "g1", "g2"), got, (e1, e2, j1, j2, eg1, eg2)):
        assert_bitexact(g, e, k)


def test_nnd_autograd_function_matches_reference_semantics():
    """NNDFunction: returns (dist1, dist2) only; backward of sum(dist1) as in test.py."""
    from pointcloudregistration_amd.nndistance import nnd
    import oracle
    rng = np.random.default_rng(11)
    p1 = rng.random((16, 2048, 3), dtype=np.float32)
    p2 = rng.random((16, 1024, 3), dtype=np.float32)
    t1 = _gpu(p1).requires_grad_(True)
    t2 = _gpu(p2).requires_grad_(True)
    d1, d2 = nnd(t1, t2)
    loss = torch.sum(d1)
    loss.backward()
    e1, e2, j1, j2 = oracle.nnd_forward(p1, p2)
    eg1, eg2 = oracle.nnd_backward(p1, p2, np.ones_like(e1), np.zeros_like(e2), j1, j2)
    assert np.array_equal(d1.detach().cpu().numpy().view(np.uint32), e1.view(np.uint32))
    assert np.array_equal(t1.grad.cpu().numpy().view(np.uint32), eg1.view(np.uint32))
    assert np.array_equal(t2.grad.cpu().numpy().view(np.uint32), eg2.view(np.uint32))


def test_nnd_full_size_properties():
    """BASELINE C4 size (256 pairs x 8192): properties the domain guarantees.
    Sampled queries are re-checked by brute force in float64 on the host
    (the f32 result must be the f32-rounded argmin), plus d==0 self-match."""
    from pointcloudregistration_amd import nndistance as nd
    g = torch.Generator(device="cuda").manual_seed(0)
    x1 = torch.rand(256, 8192, 3, device="cuda", generator=g)
    d1, d2, i1, i2 = nd.nnd_with_index(x1, x1.clone())
    torch.cuda.synchronize()
    assert torch.all(d1 == 0) and torch.all(d2 == 0)
    # identical clouds: every point's first exact match is itself unless an
    # earlier duplicate exists (none for random floats)
    ar = torch.arange(8192, device="cuda", dtype=torch.int32)
    assert torch.all(i1 == ar) and torch.all(i2 == ar)
    x2 = torch.rand(256, 8192, 3, device="cuda", generator=g)
    d1, d2, i1, i2 = nd.nnd_with_index(x1, x2)
    rows = torch.randint(0, 8192, (64,), device="cuda", generator=g)
    for bat in (0, 101, 255):
        q = x1[bat, rows].double()
        dd = ((q[:, None, :] - x2[bat].double()[None]) ** 2).sum(-1)
        best = dd.min(dim=1).values
        picked = dd.gather(1, i1[bat, rows].long()[:, None])[:, 0]
        assert torch.all(picked <= best * (1 + 1e-6) + 1e-12)


def _adversarial(kind, rng):
    if kind == "outliers":       # far queries: rings never certify -> per-query full scan
        x1 = rng.random((2, 1500, 3), dtype=np.float32)
        x1[:, ::50] += np.float32(100.0)
        x2 = rng.random((2, 1400, 3), dtype=np.float32)
    elif kind == "planar":       # zero-thickness box
        x1 = rng.random((1, 2000, 3), dtype=np.float32)
        x1[..., 2] = 0.5
        x2 = rng.random((1, 2100, 3), dtype=np.float32)
        x2[..., 2] = 0.5
    elif kind == "identical":    # every point the same: all distances tie
        x1 = np.full((1, 1200, 3), 0.25, np.float32)
        x2 = np.full((1, 1300, 3), 0.25, np.float32)
    elif kind == "quantised":    # many exact ties
        x1 = (rng.integers(0, 8, (2, 2048, 3)) / 8).astype(np.float32)
        x2 = (rng.integers(0, 8, (2, 2048, 3)) / 8).astype(np.float32)
    elif kind == "huge_offset":
        x1 = (rng.random((1, 1500, 3)) * 10 + 3e6).astype(np.float32)
        x2 = (rng.random((1, 1600, 3)) * 10 + 3e6).astype(np.float32)
    elif kind == "inf":          # non-finite: the reference loop (seed rule) answers
        x1 = rng.random((2, 1100, 3), dtype=np.float32)
        x2 = rng.random((2, 1200, 3), dtype=np.float32)
        x2[1, 0, 1] = np.inf
        x1[0, 5, 0] = -np.inf
    else:                        # "nan"
        x1 = rng.random((1, 1100, 3), dtype=np.float32)
        x2 = rng.random((1, 1200, 3), dtype=np.float32)
        x2[0, 0, 2] = np.nan
        x1[0, 9, 1] = np.nan
    return x1, x2


@pytest.mark.parametrize("kind", ["outliers", "planar", "identical", "quantised",
                                  "huge_offset", "inf", "nan"])
def test_nnd_grid_adversarial_vs_oracle(oracle, monkeypatch, kind):
    """The certified grid search stays exact where certification is hard."""
    monkeypatch.setenv("PCR_NND_ALGO", "grid")
    rng = np.random.default_rng(len(kind))
    x1, x2 = _adversarial(kind, rng)
    gd1 = rng.standard_normal(x1.shape[:2]).astype(np.float32)
    gd2 = rng.standard_normal(x2.shape[:2]).astype(np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        got = _run_fwd_bwd(x1, x2, gd1, gd2)
        e1, e2, j1, j2 = oracle.nnd_forward(x1, x2)
        eg1, eg2 = oracle.nnd_backward(x1, x2, gd1, gd2, j1, j2)
    for k, g, e in zip(("d1", "d2", "i1", "i2", "g1", "g2"), got, (e1, e2, j1, j2, eg1, eg2)):
        assert_bitexact(g, e, f"{kind}/{k}")


@pytest.mark.parametrize("lpq", ["1", "2", "4", "8", "16"])
@pytest.mark.parametrize("kind", ["outliers", "quantised", "identical", "nan", "random"])
def test_nnd_grid_lanes_per_query_vs_oracle(oracle, monkeypatch, kind, lpq):
    """Splitting each query's ring columns and fallback scan over LPQ lanes
    (PCR_NND_LPQ; the size rule picks 8 for one pair, 1 for C4 batches) keeps
    the exact (d, j) answer, ties and the non-finite reference loop included."""
    monkeypatch.setenv("PCR_NND_ALGO", "grid")
    monkeypatch.setenv("PCR_NND_LPQ", lpq)
    rng = np.random.default_rng(len(kind) + 100)
    if kind == "random":  # the NDP Chamfer shape: a 5000-point subset vs 20000 targets
        x1 = (rng.random((1, 5000, 3), dtype=np.float32) * 2 - 1).astype(np.float32)
        x2 = (rng.random((1, 20000, 3), dtype=np.float32) * 2 - 1).astype(np.float32)
    else:
        x1, x2 = _adversarial(kind, rng)
    gd1 = rng.standard_normal(x1.shape[:2]).astype(np.float32)
    gd2 = rng.standard_normal(x2.shape[:2]).astype(np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        got = _run_fwd_bwd(x1, x2, gd1, gd2)
        e1, e2, j1, j2 = oracle.nnd_forward(x1, x2)
        eg1, eg2 = oracle.nnd_backward(x1, x2, gd1, gd2, j1, j2)
    for k, g, e in zip(("d1", "d2", "i1", "i2", "g1", "g2"), got, (e1, e2, j1, j2, eg1, eg2)):
        assert_bitexact(g, e, f"{kind}/lpq{lpq}/{k}")



def test_nnd_grid_mixed_batch_vs_oracle(oracle, monkeypatch):
    """A 70-cloud batch holding every hard kind at once -- outliers (full-scan
    fallback), planar, identical, quantised ties, a NaN and an Inf cloud (the
    reference loop) -- next to ordinary clouds, with the queries walked in their
    own grid's slot order: bit for bit against the oracle, backward included."""
    monkeypatch.setenv("PCR_NND_ALGO", "grid")
    rng = np.random.default_rng(64)
    B, n, m = 70, 1100, 1200
    x1 = rng.random((B, n, 3), dtype=np.float32)
    x2 = rng.random((B, m, 3), dtype=np.float32)
    x1[0, ::50] += np.float32(100.0)                        # outliers
    x1[1, :, 2] = 0.5
    x2[1, :, 2] = 0.5                                       # planar
    x1[2] = 0.25
    x2[2] = 0.25                                            # identical
    x1[3] = (rng.integers(0, 8, (n, 3)) / 8).astype(np.float32)
    x2[3] = (rng.integers(0, 8, (m, 3)) / 8).astype(np.float32)   # quantised ties
    x2[4, 0, 2] = np.nan
    x1[5, 7, 0] = np.inf                                    # the reference loop
    gd1 = rng.standard_normal((B, n)).astype(np.float32)
    gd2 = rng.standard_normal((B, m)).astype(np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        got = _run_fwd_bwd(x1, x2, gd1, gd2)
        e1, e2, j1, j2 = oracle.nnd_forward(x1, x2)
        eg1, eg2 = oracle.nnd_backward(x1, x2, gd1, gd2, j1, j2)
    for k, g, e in zip(("d1", "d2", "i1", "i2", "g1", "g2"), got, (e1, e2, j1, j2, eg1, eg2)):
        assert_bitexact(g, e, f"mixed/{k}")
