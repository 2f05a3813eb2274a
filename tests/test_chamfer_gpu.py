"""a3 on the GPU: the Chamfer reductions of chamfer.py against a numpy
restatement of c2p-net/deformationpyramid/model/loss.py:104-200 applied to the
oracle's (bit-exact, reference-pinned) nnd distances.

compute_truncated_chamfer_distance: squared 1-NN distances both ways, entries
>= trunc zeroed, the point mean over the FULL length (loss.py:151-154,187-195),
optional per-cloud weights, batch mean/sum.  chamfer_distance = pytorch3d's
default mean/mean (dip/train.py:84,113); pytorch3d itself is absent, so parity
vs pytorch3d is unpinned beyond these shared semantics.  Tolerance: the
distances are bit-exact, the f32 sums may be ordered differently -> 1e-6 rel.
"""
import numpy as np
import pytest
import torch

from pointcloudregistration_amd.chamfer import chamfer_distance, compute_truncated_chamfer_distance

pytestmark = pytest.mark.gpu


def np_truncated_chamfer(oracle, x, y, trunc, batch_reduction="mean", point_reduction="mean",
                         weights=None):
    """loss.py:140-200 in numpy (f64 sums of the oracle's f32 squared distances)."""
    d1, d2, _, _ = oracle.nnd_forward(x, y)
    N, P1, P2 = x.shape[0], x.shape[1], y.shape[1]
    cx = np.where(d1 >= trunc, 0.0, d1.astype(np.float64))
    cy = np.where(d2 >= trunc, 0.0, d2.astype(np.float64))
    if weights is not None:
        cx = cx * weights[:, None]
        cy = cy * weights[:, None]
    cx, cy = cx.sum(1), cy.sum(1)
    if point_reduction == "mean":
        cx, cy = cx / P1, cy / P2
    if batch_reduction is not None:
        cx, cy = cx.sum(), cy.sum()
        if batch_reduction == "mean":
            div = weights.sum() if weights is not None else N
            cx, cy = cx / div, cy / div
    return cx + cy


def _clouds(seed, b, n, m):
    rng = np.random.default_rng(seed)
    return (rng.random((b, n, 3), dtype=np.float32),
            (rng.random((b, m, 3), dtype=np.float32) * 1.3 - 0.15).astype(np.float32))


@pytest.mark.parametrize("b,n,m", [(1, 700, 900), (3, 2048, 1500), (2, 5000, 4096)])
@pytest.mark.parametrize("br,pr", [("mean", "mean"), ("sum", "mean"), (None, "sum"), ("mean", "sum")])
def test_truncated_chamfer_masks_vs_numpy(oracle, b, n, m, br, pr):
    x, y = _clouds(b * n + m, b, n, m)
    d1, _, _, _ = oracle.nnd_forward(x, y)
    trunc = float(np.quantile(d1, 0.7))   # a finite trunc that masks ~30 % of x's terms
    got = compute_truncated_chamfer_distance(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(),
                                             trunc=trunc, batch_reduction=br, point_reduction=pr)
    ref = np_truncated_chamfer(oracle, x, y, trunc, br, pr)
    assert (d1 >= trunc).mean() > 0.2
    np.testing.assert_allclose(got.detach().cpu().numpy(), ref, rtol=1e-6, atol=0)


def test_truncated_chamfer_weights(oracle):
    x, y = _clouds(3, 4, 1000, 1200)
    w = np.array([0.5, 2.0, 0.0, 1.0], np.float32)
    for br in ("mean", "sum", None):
        got = compute_truncated_chamfer_distance(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(),
                                                 trunc=0.01, batch_reduction=br,
                                                 weights=torch.from_numpy(w).cuda())
        ref = np_truncated_chamfer(oracle, x, y, 0.01, br, "mean", w.astype(np.float64))
        np.testing.assert_allclose(got.detach().cpu().numpy(), ref, rtol=1e-6)
    # all-zero weights: the reference returns a (zero, zero) pair (loss.py:133-139)
    z = compute_truncated_chamfer_distance(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(),
                                           weights=torch.zeros(4, device="cuda"))
    assert isinstance(z, tuple) and float(z[0]) == 0.0 and float(z[1]) == 0.0
    with pytest.raises(ValueError):
        compute_truncated_chamfer_distance(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(),
                                           weights=-torch.ones(4, device="cuda"))


def test_truncated_chamfer_gradient_masked_terms(oracle):
    """Backward through the mask: masked x terms get no gradient from dist1; the
    gradient equals the oracle's nnd_backward of the reduction's dL/dd."""
    x, y = _clouds(11, 2, 1500, 1300)
    d1, d2, i1, i2 = oracle.nnd_forward(x, y)
    trunc = float(np.quantile(d1, 0.5))
    X = torch.from_numpy(x).cuda().requires_grad_(True)
    Y = torch.from_numpy(y).cuda().requires_grad_(True)
    compute_truncated_chamfer_distance(X, Y, trunc=trunc).backward()
    B, P1, P2 = 2, 1500, 1300
    g1 = np.where(d1 >= trunc, 0.0, 1.0 / (P1 * B)).astype(np.float32)
    g2 = np.where(d2 >= trunc, 0.0, 1.0 / (P2 * B)).astype(np.float32)
    e1, e2 = oracle.nnd_backward(x, y, g1, g2, i1, i2)
    np.testing.assert_allclose(X.grad.cpu().numpy(), e1, rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(Y.grad.cpu().numpy(), e2, rtol=1e-5, atol=1e-9)


def test_chamfer_distance_pytorch3d_default(oracle, golden_nnd):
    """dip/train.py:84 chamfer_distance(x, y) -> (loss, None), on the C2 golden
    shape (the nnd fixture's inputs: reference-compiled distances)."""
    x, y = _clouds(0, 1, 4096, 4096)
    loss, nrm = chamfer_distance(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda())
    assert nrm is None
    ref = np_truncated_chamfer(oracle, x, y, np.inf)
    np.testing.assert_allclose(float(loss), ref, rtol=1e-6)


# --------------------------------------------------------------------------
# the reference's full interface (loss.py:60-71): lengths, normals, f64
# --------------------------------------------------------------------------
def np_chamfer_full(oracle, x, y, xl, yl, trunc, br="mean", pr="mean", weights=None):
    """loss.py:104-218 in numpy on ragged clouds: per cloud the oracle's nnd of
    x[k,:xl[k]] vs y[k,:yl[k]] (f32) or an f64 brute force (f64 inputs)."""
    N = x.shape[0]
    cx_s, cy_s = np.zeros(N), np.zeros(N)
    for k in range(N):
        a, b = x[k, :xl[k]], y[k, :yl[k]]
        if x.dtype == np.float32:
            d1, d2, _, _ = oracle.nnd_forward(a[None], b[None])
            d1, d2 = d1[0].astype(np.float64), d2[0].astype(np.float64)
        else:
            d1, d2 = np_nn_f64(a, b)[0], np_nn_f64(b, a)[0]
        cx = np.where(d1 >= trunc, 0.0, d1)
        cy = np.where(d2 >= trunc, 0.0, d2)
        if weights is not None:
            cx, cy = cx * weights[k], cy * weights[k]
        cx_s[k], cy_s[k] = cx.sum(), cy.sum()
    if pr == "mean":
        cx_s, cy_s = cx_s / xl, cy_s / yl
    if br is not None:
        cx_s, cy_s = cx_s.sum(), cy_s.sum()
        if br == "mean":
            div = weights.sum() if weights is not None else N
            cx_s, cy_s = cx_s / div, cy_s / div
    return cx_s + cy_s


def np_nn_f64(q, c):
    """f64 1-NN: d = (dx*dx + dy*dy) + dz*dz, dx = c - q, first index of the min."""
    if len(c) == 0:
        return np.zeros(len(q)), np.zeros(len(q), np.int64)
    d = c[None, :, :] - q[:, None, :]
    D = (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]
    j = np.argmin(D, axis=1)
    return D[np.arange(len(q)), j], j


def _ragged(seed, N, P1, P2, dtype=np.float32):
    rng = np.random.default_rng(seed)
    x = rng.random((N, P1, 3)).astype(dtype)
    y = (rng.random((N, P2, 3)) * 1.2 - 0.1).astype(dtype)
    xl = rng.integers(P1 // 3, P1 + 1, N)
    yl = rng.integers(P2 // 3, P2 + 1, N)
    xl[0], yl[-1] = P1, P2
    return x, y, xl, yl


def test_chamfer_reference_signature_and_defaults(oracle):
    """Positional binding and defaults of loss.py:60-71 (trunc=0.2, mean/mean)."""
    x, y = _clouds(5, 2, 900, 1100)
    X, Y = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    got = compute_truncated_chamfer_distance(X, Y)
    ref = np_truncated_chamfer(oracle, x, y, 0.2)
    np.testing.assert_allclose(float(got), ref, rtol=1e-6)
    w = np.array([0.7, 1.5], np.float32)
    xl, yl = np.array([900, 600]), np.array([800, 1100])
    got = compute_truncated_chamfer_distance(
        X, Y, torch.from_numpy(xl).cuda(), torch.from_numpy(yl).cuda(), None, None,
        torch.from_numpy(w).cuda(), 0.01, "sum", "mean")
    ref = np_chamfer_full(oracle, x, y, xl, yl, 0.01, "sum", "mean", w.astype(np.float64))
    np.testing.assert_allclose(float(got), ref, rtol=1e-6)
    with pytest.raises(TypeError):
        compute_truncated_chamfer_distance(X.half(), Y.half())
    with pytest.raises(ValueError):
        compute_truncated_chamfer_distance(X, Y, point_reduction="max")


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("br,pr", [("mean", "mean"), ("sum", "sum"), (None, "mean")])
def test_chamfer_ragged_lengths_vs_numpy(oracle, dtype, br, pr):
    x, y, xl, yl = _ragged(17, 4, 1500, 1200, dtype)
    # padding rows hold far-away junk that must not be found or counted
    for k in range(4):
        x[k, xl[k]:] = 50.0
        y[k, yl[k]:] = -50.0
    got = compute_truncated_chamfer_distance(
        torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(), torch.from_numpy(xl).cuda(),
        torch.from_numpy(yl).cuda(), trunc=0.004, batch_reduction=br, point_reduction=pr)
    assert got.dtype == (torch.float64 if dtype == np.float64 else torch.float32)
    ref = np_chamfer_full(oracle, x, y, xl, yl, 0.004, br, pr)
    np.testing.assert_allclose(got.detach().cpu().numpy(), ref, rtol=1e-12 if dtype == np.float64 else 1e-6)


def test_nnd_ragged_kernel_bitexact_vs_oracle(oracle):
    """pcr_nnd_forward_ragged: per cloud == the reference-pinned oracle on the
    cloud's own points (ties, duplicates, NaN rows, an empty cloud); rows past
    a length and rows whose other cloud is empty are (0, 0)."""
    from pointcloudregistration_amd import _lib
    rng = np.random.default_rng(3)
    N, P1, P2 = 5, 1300, 700
    x = (np.round(rng.random((N, P1, 3)) * 8) / 8).astype(np.float32)   # many ties
    y = (np.round(rng.random((N, P2, 3)) * 8) / 8).astype(np.float32)
    x[1, 5] = np.nan
    y[2, 0] = np.nan                                 # candidate-0 NaN seed rule
    xl = np.array([P1, 1000, 1, 77, 1300], np.int32)
    yl = np.array([P2, 650, 700, 0, 1], np.int32)    # cloud 3 has an empty y
    X, Y = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    out = [torch.full((N, P), 7, dtype=t, device="cuda") for P, t in
           ((P1, torch.float32), (P2, torch.float32), (P1, torch.int32), (P2, torch.int32))]
    n1, n2 = torch.from_numpy(xl).cuda(), torch.from_numpy(yl).cuda()
    _lib.call("pcr_nnd_forward_ragged", _lib.ptr(X), _lib.ptr(Y), N, P1, P2, _lib.ptr(n1),
              _lib.ptr(n2), *[_lib.ptr(o) for o in out], _lib.stream_handle(X.device))
    d1, d2, i1, i2 = (o.cpu().numpy() for o in out)
    for k in range(N):
        a, b = x[k, :xl[k]], y[k, :yl[k]]
        if len(b):
            e1, _, j1, _ = oracle.nnd_forward(a[None], b[None])
            assert np.array_equal(d1[k, :xl[k]].view(np.int32) & 0x7fffffff,
                                  e1[0].view(np.int32) & 0x7fffffff), k
            assert np.array_equal(i1[k, :xl[k]], j1[0]), k
        else:
            assert not d1[k, :xl[k]].any() and not i1[k, :xl[k]].any()
        if len(a) and len(b):
            _, e2, _, j2 = oracle.nnd_forward(a[None], b[None])
            assert np.array_equal(d2[k, :yl[k]].view(np.int32) & 0x7fffffff,
                                  e2[0].view(np.int32) & 0x7fffffff), k
            assert np.array_equal(i2[k, :yl[k]], j2[0]), k
        assert not d1[k, xl[k]:].any() and not i1[k, xl[k]:].any()
        assert not d2[k, yl[k]:].any() and not i2[k, yl[k]:].any()


def test_nnd_f64_kernel_vs_numpy():
    from pointcloudregistration_amd import _lib
    rng = np.random.default_rng(8)
    N, P1, P2 = 3, 2000, 900
    x = rng.standard_normal((N, P1, 3)) * 1e3          # mm-scale, f64 resolution matters
    y = x[:, :P2] + rng.standard_normal((N, P2, 3)) * 1e-9
    X, Y = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    d1 = torch.empty(N, P1, dtype=torch.float64, device="cuda")
    d2 = torch.empty(N, P2, dtype=torch.float64, device="cuda")
    i1 = torch.empty(N, P1, dtype=torch.int32, device="cuda")
    i2 = torch.empty(N, P2, dtype=torch.int32, device="cuda")
    _lib.call("pcr_nnd_forward_f64", _lib.ptr(X), _lib.ptr(Y), N, P1, P2, None, None, _lib.ptr(d1),
              _lib.ptr(d2), _lib.ptr(i1), _lib.ptr(i2), _lib.stream_handle(X.device))
    for k in range(N):
        e1, j1 = np_nn_f64(x[k], y[k])
        e2, j2 = np_nn_f64(y[k], x[k])
        assert np.array_equal(d1[k].cpu().numpy(), e1) and np.array_equal(i1[k].cpu().numpy(), j1)
        assert np.array_equal(d2[k].cpu().numpy(), e2) and np.array_equal(i2[k].cpu().numpy(), j2)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_chamfer_ragged_gradient(oracle, dtype):
    """d loss / d x for ragged clouds: 2 (x - y_nn) / (N len_x) on kept rows plus
    the scatter of the y-side terms, zero on padding rows."""
    x, y, xl, yl = _ragged(23, 3, 800, 600, dtype)
    X = torch.from_numpy(x).cuda().requires_grad_(True)
    Y = torch.from_numpy(y).cuda().requires_grad_(True)
    compute_truncated_chamfer_distance(X, Y, torch.from_numpy(xl).cuda(), torch.from_numpy(yl).cuda(),
                                       trunc=1e9).backward()
    gx = np.zeros(x.shape)
    gy = np.zeros(y.shape)
    N = 3
    for k in range(N):
        a, b = x[k, :xl[k]].astype(np.float64), y[k, :yl[k]].astype(np.float64)
        if dtype == np.float32:   # the f32 argmin (reference-pinned oracle)
            _, _, j1, j2 = oracle.nnd_forward(x[k:k + 1, :xl[k]], y[k:k + 1, :yl[k]])
            j1, j2 = j1[0], j2[0]
        else:
            _, j1 = np_nn_f64(a, b)
            _, j2 = np_nn_f64(b, a)
        t1 = 2 * (a - b[j1]) / (N * xl[k])
        t2 = 2 * (b - a[j2]) / (N * yl[k])
        gx[k, :xl[k]] += t1
        np.add.at(gy[k], j1, -t1)
        gy[k, :yl[k]] += t2
        np.add.at(gx[k], j2, -t2)
    tol = 1e-12 if dtype == np.float64 else 2e-6
    np.testing.assert_allclose(X.grad.cpu().numpy(), gx, atol=tol * np.abs(gx).max())
    np.testing.assert_allclose(Y.grad.cpu().numpy(), gy, atol=tol * np.abs(gy).max())
