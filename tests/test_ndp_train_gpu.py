"""GPU: the fused NDP level step (csrc/ndp_train.hip) against torch autograd of
the same layer (the reference's NDPLayer restated in ndp_opt.NDPLayer, whose
warp matches the reference's own to 1e-6: test_ndp_opt_cpu.py).

Tolerance: forward x' to 2e-6 absolute (f32, different summation order of the
MFMA chains vs hipBLASLt); gradients to 2e-4 of each tensor's largest entry (f32
sums over 3000 points in different orders)."""
import ctypes

import numpy as np
import pytest
import torch

from pointcloudregistration_amd import _lib, ndp_opt

pytestmark = pytest.mark.gpu


def _layer(level, seed, scale=3.0):
    torch.manual_seed(seed)
    L = ndp_opt.NDPLayer(3, 128, -8, level + 1, nonrigidity_est=level > 0).cuda()
    with torch.no_grad():
        for p in L.parameters():
            if p.dim() > 1:
                p.mul_(scale)  # far from the identity warp of a fresh init
            else:
                p.uniform_(-0.2, 0.2)
    return L


@pytest.mark.parametrize("level", [0, 1, 5])
def test_fused_forward_and_gradients_match_autograd(level):
    rng = np.random.default_rng(level)
    N = 3000
    x = torch.from_numpy(rng.uniform(-0.8, 0.8, (N, 3)).astype(np.float32)).cuda()
    t = torch.from_numpy(rng.uniform(-0.8, 0.8, (500, 3)).astype(np.float32)).cuda()
    inds = torch.arange(0, N, 3, device="cuda")
    L = _layer(level, 10 + level)
    cfg = ndp_opt.NDPConfig(w_reg=0.05)
    lv = ndp_opt._LevelFused(L, x, t, inds, level, cfg)
    st = _lib.stream_handle()
    _lib.call("pcr_ndp_train_forward", ctypes.byref(lv.desc), st)
    xo, nr = L(x)
    assert torch.allclose(lv.xo, xo.detach(), atol=2e-6, rtol=0)
    if nr is not None:
        assert torch.allclose(lv.aux[6], nr.detach(), atol=2e-6, rtol=0)
    g = torch.from_numpy(rng.standard_normal((N, 3)).astype(np.float32)).cuda()
    lv.desc.inv = lv.desc.xs = lv.desc.gsub = None  # dL/dx' from gx (subset path: below)
    lv.gx.copy_(g)
    _lib.call("pcr_ndp_train_backward", ctypes.byref(lv.desc), _lib.ptr(lv.part), lv.CHUNK,
              ctypes.cast(lv.grad_ptrs, ctypes.c_void_p), st)
    loss = (xo * g).sum()
    if lv.bce_on:
        loss = loss + cfg.w_reg * torch.mean(-torch.log(1 - nr))
    want = torch.autograd.grad(loss, lv.params)
    torch.cuda.synchronize()
    for (name, _), got, w in zip(L.named_parameters(), lv.grads, want):
        tol = 2e-4 * float(w.abs().max()) + 1e-12
        assert torch.allclose(got, w, atol=tol, rtol=0), (name, float((got - w).abs().max()), tol)


def test_subset_path_matches_explicit_gather_scatter():
    """inv/xs/gsub (the forward writes x'[inds], the backward reads dL/dx' of the
    subset) == index_select + index_add_ into a full gradient, bit for bit."""
    rng = np.random.default_rng(7)
    N, K = 3000, 1000
    x = torch.from_numpy(rng.uniform(-0.8, 0.8, (N, 3)).astype(np.float32)).cuda()
    t = torch.from_numpy(rng.uniform(-0.8, 0.8, (500, 3)).astype(np.float32)).cuda()
    inds = torch.from_numpy(np.sort(rng.choice(N, K, replace=False))).cuda()
    L = _layer(2, 17)
    lv = ndp_opt._LevelFused(L, x, t, inds, 2, ndp_opt.NDPConfig(w_reg=0.05))
    assert lv.use_inv
    lv.desc.gacc = None  # the gsub form of the subset gradient (gacc: test_ndp_chamfer_gpu.py)
    st = _lib.stream_handle()
    _lib.call("pcr_ndp_train_forward", ctypes.byref(lv.desc), st)
    assert torch.equal(lv.xs[0], lv.xo[inds])
    gs = torch.from_numpy(rng.standard_normal((K, 3)).astype(np.float32)).cuda()
    lv.gsub[0].copy_(gs)
    args = (_lib.ptr(lv.part), lv.CHUNK, ctypes.cast(lv.grad_ptrs, ctypes.c_void_p), st)
    _lib.call("pcr_ndp_train_backward", ctypes.byref(lv.desc), *args)
    got = [g.clone() for g in lv.grads]
    lv.desc.inv = lv.desc.xs = lv.desc.gsub = None
    lv.gx.zero_()
    lv.gx.index_add_(0, inds, gs)
    _lib.call("pcr_ndp_train_backward", ctypes.byref(lv.desc), *args)
    torch.cuda.synchronize()
    for a, b in zip(got, lv.grads):
        assert torch.equal(a, b)


def test_chamfer_glue_matches_torch_loss():
    """pcr_ndp_chamfer_glue == the loss of registration.py:231-244 as torch
    computes it (sum order differs: 1e-6 relative), gradients and log exact."""
    rng = np.random.default_rng(5)
    K, M, N = 1100, 1300, 2000
    d1 = torch.from_numpy(rng.random((1, K)).astype(np.float32) * 0.1).cuda()
    d2 = torch.from_numpy(rng.random((1, M)).astype(np.float32) * 0.1).cuda()
    d1[0, 7] = 2e9  # truncated
    s = torch.from_numpy(rng.random(N).astype(np.float32) * 0.9).cuda()
    s[3] = 1.0  # log(0) -> clamped to -100
    gd1, gd2 = torch.empty_like(d1), torch.empty_like(d2)
    loss = torch.zeros((), device="cuda")
    log = torch.zeros(4, device="cuda")
    ctr = torch.tensor([5], dtype=torch.long, device="cuda")
    _lib.call("pcr_ndp_chamfer_glue", _lib.ptr(d1), K, _lib.ptr(d2), M, _lib.ptr(s), N, 0.05, 1e9,
              _lib.ptr(gd1), _lib.ptr(gd2), _lib.ptr(loss), _lib.ptr(log), _lib.ptr(ctr), 3,
              _lib.stream_handle())
    c1 = torch.where(d1 >= 1e9, torch.zeros_like(d1), d1)
    want = c1.sum() / K + d2.sum() / M + 0.05 * torch.mean(-torch.clamp(torch.log(1 - s), min=-100.0))
    torch.cuda.synchronize()
    assert abs(float(loss) - float(want)) <= 1e-6 * abs(float(want))
    assert torch.equal(gd1, torch.where(d1 >= 1e9, torch.zeros_like(d1), torch.full_like(d1, 1.0 / K)))
    assert torch.equal(gd2, torch.full_like(d2, 1.0 / M))
    assert float(log[3]) == float(loss) and int(ctr) == 6


def test_fused_optimisation_close_to_autograd_path():
    """The whole level loop: fused kernels vs the autograd path (same graph-captured
    control + Adam): losses to 1e-4 relative, warped points to 1e-4."""
    rng = np.random.default_rng(3)
    n = 2500
    u = rng.standard_normal((n, 3))
    src = (u / np.linalg.norm(u, axis=1, keepdims=True) * 0.6).astype(np.float32)
    w = rng.standard_normal((2000, 3))
    tgt = (w / np.linalg.norm(w, axis=1, keepdims=True) * 0.6 + 0.05).astype(np.float32)
    inds = np.sort(rng.choice(n, 2000, replace=False))
    cfg = dict(iters=10, m=3)

    def run(fused):
        torch.manual_seed(0)
        P = ndp_opt.DeformationPyramid(3, 128, torch.device("cuda"), -8, 3, True)
        return ndp_opt.optimize_deformation_pyramid(torch.from_numpy(src).cuda(),
                                                    torch.from_numpy(tgt).cuda(), inds, cfg,
                                                    NDP=P, fused=fused)
    a, b = run(True), run(False)
    for x, y in zip(a[3], b[3]):
        np.testing.assert_allclose(x["losses"], y["losses"], rtol=1e-4)
    assert torch.allclose(a[0], b[0], atol=1e-4)


def test_fused_loss_and_control_match_glue_then_control():
    """pcr_ndp_chamfer_loss (32-block loss + the early-stop rule in one launch) ==
    pcr_ndp_chamfer_glue followed by pcr_ndp_control: the loss to 1e-6 relative
    (another f32 summation order), the log / counter, and the rule's state over
    a sequence of losses that counts breaks and stops."""
    rng = np.random.default_rng(9)
    K, M, N = 5000, 20000, 20000
    s = torch.from_numpy(rng.random(N).astype(np.float32) * 0.9).cuda()
    st = _lib.stream_handle()
    scratch = torch.zeros(int(_lib.load().pcr_ndp_loss_scratch_bytes()), dtype=torch.uint8, device="cuda")
    state = [torch.tensor([1.0, 0, 1e6, 0, 0, 0, 0, 0], dtype=torch.float64, device="cuda") for _ in range(2)]
    loss = [torch.zeros((), device="cuda") for _ in range(2)]
    log = [torch.zeros(41, device="cuda") for _ in range(2)]
    ctr = [torch.zeros(1, dtype=torch.long, device="cuda") for _ in range(2)]
    base1 = rng.random(K).astype(np.float32) * 0.01
    base2 = rng.random(M).astype(np.float32) * 0.01
    for it in range(12):
        f = 1.0 if it < 4 else 1.0 + 1e-5 * it  # flat losses: the break counter runs
        d1 = torch.from_numpy(base1 * f).cuda()
        d2 = torch.from_numpy(base2 * f).cuda()
        _lib.call("pcr_ndp_chamfer_glue", _lib.ptr(d1), K, _lib.ptr(d2), M, _lib.ptr(s), N, 0.05, 1e9,
                  None, None, _lib.ptr(loss[0]), _lib.ptr(log[0]), _lib.ptr(ctr[0]), 40, st)
        _lib.call("pcr_ndp_control", _lib.ptr(loss[0]), _lib.ptr(state[0]), 0.001, 3, 1e-4, st)
        _lib.call("pcr_ndp_chamfer_loss", _lib.ptr(d1), K, _lib.ptr(d2), M, _lib.ptr(s), N, 0.05, 1e9,
                  _lib.ptr(loss[1]), _lib.ptr(log[1]), _lib.ptr(ctr[1]), 40, _lib.ptr(state[1]), 0.001, 3, 1e-4,
                  _lib.ptr(scratch), st)
        torch.cuda.synchronize()
        assert abs(float(loss[1]) - float(loss[0])) <= 1e-6 * abs(float(loss[0]))
        assert torch.equal(state[0][[0, 1, 3, 5, 6]], state[1][[0, 1, 3, 5, 6]]), it
    assert int(ctr[0]) == int(ctr[1]) == 12 and float(state[1][0]) == 0.0
    assert int(scratch.view(torch.int32)[96]) == 0  # the completion counter is left at zero
