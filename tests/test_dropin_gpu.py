"""The `torch_nndistance` drop-in PACKAGE on sys.path, driven through the
reference's own test sequence (dip/torch-nndistance/test.py:3-24): import
torch_nndistance as NND; (16, 2048, 3) / (16, 1024, 3) clouds; NND.nnd twice --
once with a non-leaf `points1` (Variable(p1, requires_grad=True).cuda(): its
.grad stays None, as in the reference) and once with a leaf on the device.
Distances and gradients are checked bit for bit against the oracle (pinned to the
reference's compiled my_lib.cpp by tests/golden/nnd_golden.npz)."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "pointcloudregistration_amd", "dropin")


@pytest.fixture()
def NND():
    sys.path.insert(0, DROPIN)
    try:
        import torch_nndistance
        yield torch_nndistance
    finally:
        sys.path.remove(DROPIN)


def test_reference_test_sequence(NND, oracle):
    from torch.autograd import Variable
    torch.manual_seed(0)
    p1 = torch.rand(16, 2048, 3)
    p2 = torch.rand(16, 1024, 3)
    x1, x2 = p1.numpy(), p2.numpy()
    e1, e2, j1, j2 = oracle.nnd_forward(x1, x2)
    g1, g2 = oracle.nnd_backward(x1, x2, np.ones_like(e1), np.zeros_like(e2), j1, j2)

    # first half of test.py: Variable(...).cuda() is a non-leaf
    points1 = Variable(p1, requires_grad=True)
    points2 = Variable(p2)
    points1 = points1.cuda()
    points2 = points2.cuda()
    dist1, dist2 = NND.nnd(points1, points2)
    assert np.array_equal(dist1.detach().cpu().numpy(), e1)
    assert np.array_equal(dist2.detach().cpu().numpy(), e2)
    loss = torch.sum(dist1)
    loss.backward()
    assert points2.grad is None

    # second half: a leaf on the device gets the gradient
    points1 = Variable(p1.cuda(), requires_grad=True)
    points2 = Variable(p2.cuda())
    dist1, dist2 = NND.nnd(points1, points2)
    loss = torch.sum(dist1)
    loss.backward()
    assert np.array_equal(points1.grad.cpu().numpy(), g1)
    assert points2.grad is None
    assert np.isclose(float(loss), float(e1.astype(np.float64).sum()), rtol=1e-5)


def test_package_exports_reference_names(NND):
    import torch_nndistance_aten as aten
    assert NND.my_lib is aten
    for name in ("nnd_forward_cuda", "nnd_backward_cuda", "nnd_forward", "nnd_backward"):
        assert callable(getattr(aten, name))
    assert hasattr(NND, "NNDFunction") and callable(NND.nnd)


def test_aten_inplace_contract(NND, oracle):
    """nnd_forward_cuda / nnd_backward_cuda write caller-allocated outputs and return 1
    (my_lib_cuda.cpp:25-72), the way the reference's NNDFunction calls them."""
    import torch_nndistance_aten as aten
    rng = np.random.default_rng(3)
    x1 = rng.random((2, 777, 3), dtype=np.float32)
    x2 = rng.random((2, 1500, 3), dtype=np.float32)
    t1, t2 = torch.from_numpy(x1).cuda(), torch.from_numpy(x2).cuda()
    d1, d2 = torch.zeros(2, 777, device="cuda"), torch.zeros(2, 1500, device="cuda")
    i1 = torch.zeros(2, 777, dtype=torch.int32, device="cuda")
    i2 = torch.zeros(2, 1500, dtype=torch.int32, device="cuda")
    assert aten.nnd_forward_cuda(t1, t2, d1, d2, i1, i2) == 1
    e1, e2, j1, j2 = oracle.nnd_forward(x1, x2)
    assert np.array_equal(d1.cpu().numpy(), e1) and np.array_equal(i1.cpu().numpy(), j1)
    assert np.array_equal(d2.cpu().numpy(), e2) and np.array_equal(i2.cpu().numpy(), j2)
    gd1 = rng.standard_normal((2, 777)).astype(np.float32)
    gd2 = rng.standard_normal((2, 1500)).astype(np.float32)
    gx1, gx2 = torch.zeros_like(t1), torch.zeros_like(t2)
    assert aten.nnd_backward_cuda(t1, t2, gx1, gx2, torch.from_numpy(gd1).cuda(),
                                  torch.from_numpy(gd2).cuda(), i1, i2) == 1
    f1, f2 = oracle.nnd_backward(x1, x2, gd1, gd2, j1, j2)
    assert np.array_equal(gx1.cpu().numpy(), f1) and np.array_equal(gx2.cpu().numpy(), f2)
