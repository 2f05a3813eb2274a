"""Host mirror of the reference's ``torch_nndistance`` operator (a1/a2).

Reference surface (dip/torch-nndistance):
  * extension module ``torch_nndistance_aten`` with
    ``nnd_forward_cuda(xyz1, xyz2, dist1, dist2, idx1, idx2) -> int`` and
    ``nnd_backward_cuda(xyz1, xyz2, gradxyz1, gradxyz2, graddist1, graddist2, idx1, idx2) -> int``
    (src/my_lib_cuda.cpp:25-77): caller-allocated outputs written in place,
    returns 1 on success;
  * ``NNDFunction`` autograd function and ``nnd(xyz1, xyz2) -> (dist1, dist2)``
    (torch_nndistance/__init__.py:10-61); idx tensors are saved for backward but
    not returned.

Here every call goes through libpcr.so (HIP, gfx950) via its C ABI, on torch's
current stream.  The reference only checks device + contiguity
(my_lib_cuda.cpp:4-6); we additionally check dtype and shapes and raise
``ValueError`` instead of reading out of bounds.  CPU tensors raise: the
reference's CPU branch is not built by its own build.py (it references a
``my_lib.nnd_forward`` that does not exist), and this library has no CPU path.
"""
from __future__ import annotations

import torch

from . import _lib


def _check(name, t, dtype, shape=None):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA (ROCm/HIP) tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")


def _dims(xyz1, xyz2):
    if xyz1.dim() != 3 or xyz1.shape[2] != 3 or xyz2.dim() != 3 or xyz2.shape[2] != 3:
        raise ValueError("xyz1/xyz2 must be (B, N, 3) / (B, M, 3)")
    if xyz1.shape[0] != xyz2.shape[0]:
        raise ValueError("xyz1 and xyz2 must have the same batch size")
    if xyz1.device != xyz2.device:
        raise ValueError("xyz1 and xyz2 must be on the same device")
    return xyz1.shape[0], xyz1.shape[1], xyz2.shape[1]


def nnd_forward_cuda(xyz1, xyz2, dist1, dist2, idx1, idx2):
    """In-place forward; mirrors my_lib_cuda.cpp:25-41. Returns 1 on success."""
    _check("xyz1", xyz1, torch.float32)
    _check("xyz2", xyz2, torch.float32)
    b, n, m = _dims(xyz1, xyz2)
    _check("dist1", dist1, torch.float32, (b, n))
    _check("dist2", dist2, torch.float32, (b, m))
    _check("idx1", idx1, torch.int32, (b, n))
    _check("idx2", idx2, torch.int32, (b, m))
    with torch.cuda.device(xyz1.device):
        _lib.call("pcr_nnd_forward", _lib.ptr(xyz1), _lib.ptr(xyz2), b, n, m,
                  _lib.ptr(dist1), _lib.ptr(dist2), _lib.ptr(idx1), _lib.ptr(idx2),
                  _lib.stream_handle(xyz1.device))
    return 1


def nnd_backward_cuda(xyz1, xyz2, gradxyz1, gradxyz2, graddist1, graddist2, idx1, idx2):
    """In-place backward; mirrors my_lib_cuda.cpp:44-72. Returns 1 on success.

    gradxyz1/gradxyz2 are fully overwritten (the reference requires them zeroed)."""
    _check("xyz1", xyz1, torch.float32)
    _check("xyz2", xyz2, torch.float32)
    b, n, m = _dims(xyz1, xyz2)
    _check("gradxyz1", gradxyz1, torch.float32, (b, n, 3))
    _check("gradxyz2", gradxyz2, torch.float32, (b, m, 3))
    _check("graddist1", graddist1, torch.float32, (b, n))
    _check("graddist2", graddist2, torch.float32, (b, m))
    _check("idx1", idx1, torch.int32, (b, n))
    _check("idx2", idx2, torch.int32, (b, m))
    with torch.cuda.device(xyz1.device):
        _lib.call("pcr_nnd_backward", _lib.ptr(xyz1), _lib.ptr(xyz2), _lib.ptr(graddist1),
                  _lib.ptr(graddist2), _lib.ptr(idx1), _lib.ptr(idx2), b, n, m,
                  _lib.ptr(gradxyz1), _lib.ptr(gradxyz2), _lib.stream_handle(xyz1.device))
    return 1


def _no_cpu(*_args, **_kw):
    raise _lib.PcrError(
        "torch_nndistance CPU path: libpcr is a GPU (gfx950) library; move tensors to "
        "the GPU (the reference's own CPU branch is not built by its build.py)")


nnd_forward = _no_cpu
nnd_backward = _no_cpu


class NNDFunction(torch.autograd.Function):
    """Mirror of torch_nndistance.NNDFunction (__init__.py:10-57)."""

    @staticmethod
    def forward(ctx, xyz1, xyz2):
        batchsize, n, _ = xyz1.size()
        _, m, _ = xyz2.size()
        if not xyz1.is_cuda:
            _no_cpu()
        xyz1 = xyz1.contiguous()
        xyz2 = xyz2.contiguous()
        dev = xyz1.device
        dist1 = torch.zeros(batchsize, n, device=dev)
        dist2 = torch.zeros(batchsize, m, device=dev)
        idx1 = torch.zeros(batchsize, n, dtype=torch.int32, device=dev)
        idx2 = torch.zeros(batchsize, m, dtype=torch.int32, device=dev)
        nnd_forward_cuda(xyz1, xyz2, dist1, dist2, idx1, idx2)
        ctx.save_for_backward(xyz1, xyz2, dist1, dist2, idx1, idx2)
        ctx.mark_non_differentiable(idx1, idx2)
        return dist1, dist2

    @staticmethod
    def backward(ctx, graddist1, graddist2):
        xyz1, xyz2, _dist1, _dist2, idx1, idx2 = ctx.saved_tensors
        dev = xyz1.device
        graddist1 = (graddist1 if graddist1 is not None
                     else torch.zeros(idx1.shape, device=dev)).contiguous().float()
        graddist2 = (graddist2 if graddist2 is not None
                     else torch.zeros(idx2.shape, device=dev)).contiguous().float()
        gradxyz1 = torch.empty(xyz1.size(), device=dev)
        gradxyz2 = torch.empty(xyz2.size(), device=dev)
        nnd_backward_cuda(xyz1, xyz2, gradxyz1, gradxyz2, graddist1, graddist2, idx1, idx2)
        return gradxyz1, gradxyz2


def nnd(xyz1, xyz2):
    """(dist1, dist2) = squared 1-NN distances both ways (torch_nndistance.nnd)."""
    return NNDFunction.apply(xyz1, xyz2)


def nnd_with_index(xyz1, xyz2):
    """Forward only, also returning the int32 indices (dist1, dist2, idx1, idx2)."""
    b, n, m = _dims(xyz1, xyz2)
    dev = xyz1.device
    dist1 = torch.empty(b, n, device=dev)
    dist2 = torch.empty(b, m, device=dev)
    idx1 = torch.empty(b, n, dtype=torch.int32, device=dev)
    idx2 = torch.empty(b, m, dtype=torch.int32, device=dev)
    nnd_forward_cuda(xyz1.contiguous(), xyz2.contiguous(), dist1, dist2, idx1, idx2)
    return dist1, dist2, idx1, idx2
