"""GPU: the NDP level Chamfer pass (csrc/ndp_chamfer.hip) against the nnd drop-in
kernels it specialises (a1 / a2, themselves bit-exact vs the reference's
my_lib.cpp: test_nnd_gpu.py).

* distances and indices: bit-exact vs pcr_nnd_forward, for every ring cap
  (PCR_NDP_CHAMFER_RINGS 0..3: more or fewer queries go to the tiled exact
  scan) of the grid path and on the box path (default) from any starting
  answers, on a partially overlapping pair (a third of the target far from the
  subset), quantised ties, and with a NaN (the reference loop);
* the gradient (exact two-word fixed-point sums of the f32 terms, the exponent
  taken from the iteration's extents): per entry within 1e-12 relative of the
  exact sum of the same f32 terms (numpy, f64) -- on unit-scale, near-converged
  (1e-9 offsets) and millimetre / 1e7-scale pairs, where the round-3 2^-44
  quantum lost small entries and |terms| >= 4096 turned the gradient into NaN;
  and vs pcr_nnd_backward (f32 sums in the reference's index order) within
  2e-6 of the largest entry;
* repeated steps (the per-iteration resets) give the same bits; a closed gate
  skips the step.
"""
import ctypes
import math
import os

import numpy as np
import pytest
import torch

from pointcloudregistration_amd import _lib
from pointcloudregistration_amd.ndp_opt import GACC_REPLICAS, _ChamferC
from pointcloudregistration_amd.nndistance import nnd_backward_cuda, nnd_forward_cuda

pytestmark = pytest.mark.gpu


class _Nc:
    def __init__(self, xs, tgt, trunc=1e9, xs0=None):
        self.xs, self.tgt = xs.contiguous(), tgt.contiguous()
        K, M = xs.shape[0], tgt.shape[0]
        self.K, self.M, self.trunc = K, M, trunc
        f = dict(device="cuda")
        self.d1, self.d2 = torch.zeros(K, **f), torch.zeros(M, **f)
        self.i1 = torch.zeros(K, dtype=torch.int32, **f)
        self.i2 = torch.zeros(M, dtype=torch.int32, **f)
        self.gacc = torch.zeros(int(_lib.load().pcr_ndp_chamfer_gacc_words(K)), dtype=torch.int64, **f)
        nb = int(_lib.load().pcr_ndp_chamfer_scratch_bytes(K, M))
        self.raw = torch.empty(nb + 256, dtype=torch.uint8, **f)
        c = _ChamferC()
        c.xs, c.tgt, c.K, c.M, c.trunc = self.xs.data_ptr(), self.tgt.data_ptr(), K, M, trunc
        c.d1, c.d2, c.i1, c.i2 = (self.d1.data_ptr(), self.d2.data_ptr(), self.i1.data_ptr(),
                                  self.i2.data_ptr())
        c.gacc = self.gacc.data_ptr()
        c.scratch = self.raw.data_ptr() + (-self.raw.data_ptr()) % 256
        self.c = c
        x0 = self.xs if xs0 is None else xs0.contiguous()
        _lib.call("pcr_ndp_chamfer_prepare", ctypes.byref(c), _lib.ptr(x0), _lib.stream_handle())

    def step(self):
        _lib.call("pcr_ndp_chamfer_step", ctypes.byref(self.c), _lib.stream_handle())
        torch.cuda.synchronize()

    def grad64(self):
        """(dL/dxs (K, 3) f64 decoded from the two words, non-finite flag, s)."""
        a = self.gacc.cpu().numpy()
        hw = int(a[0])
        sh = (hw >> 8) - 2048
        n = 3 * self.K * GACC_REPLICAS
        hi = a[1:1 + n].reshape(GACC_REPLICAS, self.K, 3).sum(0)
        lo = a[1 + n:1 + 2 * n].reshape(GACC_REPLICAS, self.K, 3).sum(0)
        g = np.ldexp(hi.astype(np.float64), -sh) + np.ldexp(lo.astype(np.float64), -sh - 40)
        return g, hw & 1, sh

    def grad(self):
        g, bad, _ = self.grad64()
        return torch.from_numpy(g).float().cuda(), bad


def _reference(xs, tgt, trunc):
    K, M = xs.shape[0], tgt.shape[0]
    d1, d2 = torch.zeros(1, K, device="cuda"), torch.zeros(1, M, device="cuda")
    i1 = torch.zeros(1, K, dtype=torch.int32, device="cuda")
    i2 = torch.zeros(1, M, dtype=torch.int32, device="cuda")
    nnd_forward_cuda(xs[None].contiguous(), tgt[None].contiguous(), d1, d2, i1, i2)
    gd1 = torch.where(d1 >= trunc, 0.0, torch.full_like(d1, np.float32(1.0 / K)))
    gd2 = torch.where(d2 >= trunc, 0.0, torch.full_like(d2, np.float32(1.0 / M)))
    g1, g2 = torch.zeros(1, K, 3, device="cuda"), torch.zeros(1, M, 3, device="cuda")
    nnd_backward_cuda(xs[None].contiguous(), tgt[None].contiguous(), g1, g2, gd1, gd2, i1, i2)
    torch.cuda.synchronize()
    return d1[0], d2[0], i1[0], i2[0], g1[0]


def _exact_grad(xs, tgt, d1, d2, i1, i2, trunc):
    """The kernel's f32 terms (emit: g = f32(1/K) * 2 where d < trunc, term =
    g * (x - y) in f32; the target side -(g2 * (y - x))) summed in f64."""
    xs, tgt = xs.cpu().numpy(), tgt.cpu().numpy()
    d1, d2, i1, i2 = (t.cpu().numpy() for t in (d1, d2, i1, i2))
    K, M = len(xs), len(tgt)
    g1 = np.where(d1 >= trunc, np.float32(0), np.float32(1.0 / K)) * np.float32(2)
    g2 = np.where(d2 >= trunc, np.float32(0), np.float32(1.0 / M)) * np.float32(2)
    t0 = (g1[:, None] * (xs - tgt[i1])).astype(np.float64)
    t1 = (-(g2[:, None] * (tgt - xs[i2]))).astype(np.float64)
    # correctly rounded sums per entry (math.fsum): the fixed point is exact, so
    # the comparison must not carry f64 summation error of its own
    order = np.argsort(i2, kind="stable")
    starts = np.searchsorted(i2[order], np.arange(K + 1))
    out = np.empty((K, 3))
    for k in range(K):
        rows = order[starts[k]:starts[k + 1]]
        for c in range(3):
            out[k, c] = math.fsum([t0[k, c], *t1[rows, c]])
    return out


def _partial_pair(seed, K=6000, M=12000):
    """A warped subset of a surface against a target of which a third lies far
    from it (the C5 regime that sends queries past the ring cap)."""
    rng = np.random.default_rng(seed)
    u = rng.uniform(0, 1, (M, 2))
    t = np.stack([u[:, 0], u[:, 1], 0.1 * np.sin(6 * u[:, 0]) * np.cos(4 * u[:, 1])], 1)
    s = t[u[:, 0] < 0.66][:K] + rng.normal(0, 0.004, (min(K, int((u[:, 0] < 0.66).sum())), 3))
    return (torch.from_numpy(s.astype(np.float32)).cuda(), torch.from_numpy(t.astype(np.float32)).cuda())


class _env:
    """Set environment variables for the duration of a block (None: unset)."""

    def __init__(self, **kv):
        self.kv, self.old = kv, {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = os.environ.get(k)
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = str(v)

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _check(xs, tgt, trunc=1e9, rings=None, seeds=None):
    """rings given: the grid path (PCR_NC_BOX=0) with that ring cap; else the
    box path, its searches started from `seeds` (i1, i2) when given."""
    with _env(PCR_NDP_CHAMFER_RINGS=rings, PCR_NC_BOX=None if rings is None else 0):
        nc = _Nc(xs, tgt, trunc)
        if seeds is not None:
            nc.i1.copy_(seeds[0])
            nc.i2.copy_(seeds[1])
        nc.step()
    d1, d2, i1, i2, g1 = _reference(xs, tgt, trunc)
    assert torch.equal(nc.d1, d1) and torch.equal(nc.i1, i1)
    assert torch.equal(nc.d2, d2) and torch.equal(nc.i2, i2)
    g, bad = nc.grad()
    assert bad == 0
    tol = 2e-6 * float(g1.abs().max()) + 1e-12
    assert torch.allclose(g, g1, atol=tol, rtol=0), float((g - g1).abs().max())
    _check_exact(nc, trunc)
    return nc


def _check_exact(nc, trunc):
    """Per entry: the two-word sums == the exact sum of the f32 terms."""
    g, bad, sh = nc.grad64()
    assert bad == 0
    want = _exact_grad(nc.xs, nc.tgt, nc.d1, nc.d2, nc.i1, nc.i2, trunc)
    err = np.abs(g - want)
    assert np.all(err <= 1e-12 * np.abs(want) + 2.0 ** (-sh - 30)), (float(err.max()), sh)
    return g, want


@pytest.mark.parametrize("rings", [None, 0, 1, 2, 3])
def test_partial_overlap_bitexact_every_ring_cap(rings):
    xs, tgt = _partial_pair(1)
    _check(xs, tgt, rings=rings)


def test_box_path_any_seed():
    """The box path's searches start from the previous answers (i1 / i2): exact
    from any start -- out-of-range and negative indices, the worst point, the
    exact answers themselves."""
    xs, tgt = _partial_pair(6, K=3000, M=7000)
    K, M = xs.shape[0], tgt.shape[0]
    _, _, i1, i2, _ = _reference(xs, tgt, 1e9)
    far1 = torch.argmax(torch.cdist(xs, tgt), dim=1).int()
    far2 = torch.argmax(torch.cdist(tgt, xs), dim=1).int()
    i32 = dict(dtype=torch.int32, device="cuda")
    for seeds in [(torch.full((K,), -7, **i32), torch.full((M,), 10 ** 9, **i32)),
                  (far1, far2), (i1, i2),
                  (torch.randint(0, M, (K,), **i32), torch.randint(0, K, (M,), **i32))]:
        _check(xs, tgt, seeds=seeds)


@pytest.mark.parametrize("K,M", [(1, 1), (1, 37), (33, 1), (31, 1025), (1025, 33), (2049, 4097)])
def test_small_and_ragged_sizes(K, M):
    """Partial leaves and groups (n not a multiple of 32 / 1024), single points,
    both paths."""
    rng = np.random.default_rng(K * 7919 + M)
    xs = torch.from_numpy(rng.normal(0, 1, (K, 3)).astype(np.float32)).cuda()
    tgt = torch.from_numpy(rng.normal(0, 1, (M, 3)).astype(np.float32)).cuda()
    _check(xs, tgt)
    _check(xs, tgt, rings=1)


def test_quantised_ties_and_truncation():
    rng = np.random.default_rng(2)
    xs = torch.from_numpy((rng.integers(0, 20, (3000, 3)) * 0.05).astype(np.float32)).cuda()
    tgt = torch.from_numpy((rng.integers(0, 20, (5000, 3)) * 0.05).astype(np.float32)).cuda()
    for rings in (None, 1):  # the box path, the grid path
        _check(xs, tgt, rings=rings)
        _check(xs, tgt, trunc=0.0025, rings=rings)  # d >= trunc: no gradient, as the glue's mask


@pytest.mark.parametrize("rings", [None, 0, 1])
def test_far_clusters_and_duplicates(rings):
    """Two target clusters far apart (one 50 cells from every subset point: the
    coarse-box search walks many empty and colliding slots), duplicated points
    (index ties), a subset straddling both."""
    rng = np.random.default_rng(11)
    a = rng.normal(0, 0.05, (4000, 3))
    b = rng.normal(0, 0.05, (3000, 3)) + np.array([3.0, -2.0, 1.0])
    tgt = np.concatenate([a, b, a[:500]]).astype(np.float32)
    xs = np.concatenate([a[::3] + rng.normal(0, 0.01, (1334, 3)), b[:40]]).astype(np.float32)
    _check(torch.from_numpy(xs).cuda(), torch.from_numpy(tgt).cuda(), rings=rings)


@pytest.mark.parametrize("box", [1, 0])
def test_nan_switches_to_reference_loop(box):
    xs, tgt = _partial_pair(3, K=2000, M=3000)
    xs[17, 1] = float("nan")
    with _env(PCR_NC_BOX=box):
        nc = _Nc(xs, tgt)
        nc.step()
    d1, d2, i1, i2, _ = _reference(xs, tgt, 1e9)
    assert torch.equal(nc.i1, i1) and torch.equal(nc.i2, i2)
    assert torch.equal(torch.nan_to_num(nc.d1, nan=-1.0), torch.nan_to_num(d1, nan=-1.0))
    assert torch.equal(torch.nan_to_num(nc.d2, nan=-1.0), torch.nan_to_num(d2, nan=-1.0))
    assert nc.grad64()[1] != 0  # the NaN term is flagged (the backward returns NaN)


@pytest.mark.parametrize("box", [1, 0])
def test_repeated_steps_and_moving_subset(box):
    """Per-iteration resets: a second step on the same input gives the same bits,
    then a moved subset (the cell / the spatial order fixed at prepare) is still
    exact."""
    xs, tgt = _partial_pair(4)
    with _env(PCR_NC_BOX=box):
        nc = _Nc(xs, tgt)
        nc.step()
        first = [t.clone() for t in (nc.d1, nc.d2, nc.i1, nc.i2, nc.gacc)]
        nc.step()
        for a, b in zip(first, (nc.d1, nc.d2, nc.i1, nc.i2, nc.gacc)):
            assert torch.equal(a, b)
        nc.xs.mul_(1.3).add_(0.05)  # the level's warp moves the subset
        nc.step()
    d1, d2, i1, i2, g1 = _reference(nc.xs, tgt, 1e9)
    assert torch.equal(nc.d1, d1) and torch.equal(nc.i1, i1)
    assert torch.equal(nc.d2, d2) and torch.equal(nc.i2, i2)
    g, _ = nc.grad()
    assert torch.allclose(g, g1, atol=2e-6 * float(g1.abs().max()) + 1e-12, rtol=0)
    _check_exact(nc, 1e9)   # the exponent follows the moved (larger) subset


@pytest.mark.parametrize("scale,offset", [(1.0, 0.0), (1000.0, 500.0), (1e7, 0.0)])
def test_gradient_relative_precision_any_scale(scale, offset):
    """Near-converged pair (every subset point 1e-9 x scale from a target
    point) at unit, millimetre (x1000, +500) and 1e7 scale: the small terms keep
    their relative precision; at 1e7 the terms reach 2e6 x 2/K >= 4096, where
    round 3 flagged the whole gradient NaN -- now finite and exact."""
    rng = np.random.default_rng(31)
    t = rng.uniform(-1, 1, (4000, 3))
    s = t[:1500] + rng.normal(0, 1e-9, (1500, 3))
    tgt = torch.from_numpy((t * scale + offset).astype(np.float32)).cuda()
    xs = torch.from_numpy((s * scale + offset).astype(np.float32)).cuda()
    nc = _Nc(xs, tgt)
    nc.step()
    d1, d2, i1, i2, g1 = _reference(xs, tgt, 1e9)
    assert torch.equal(nc.d1, d1) and torch.equal(nc.i1, i1)
    assert torch.equal(nc.d2, d2) and torch.equal(nc.i2, i2)
    g, want = _check_exact(nc, 1e9)
    assert np.isfinite(g).all()
    small = np.abs(want) > 0
    rel = np.abs(g[small] - want[small]) / np.abs(want[small])
    assert rel.max() <= 1e-12, rel.max()


def test_gate_closed_skips_step():
    xs, tgt = _partial_pair(5, K=1500, M=2500)
    nc = _Nc(xs, tgt)
    gate = torch.zeros(8, dtype=torch.float64, device="cuda")
    _lib.call("pcr_set_gate", _lib.ptr(gate))
    try:
        nc.step()
    finally:
        _lib.call("pcr_set_gate", None)
    assert int(nc.i1.abs().sum()) == 0 and int(nc.gacc.abs().sum()) == 0
