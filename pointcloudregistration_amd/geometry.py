"""f2: Open3D voxel down-sampling on the GPU (the C3 input stage).

Reference call: ``pcd.voxel_down_sample(voxel_size)`` at dip/demo.py:73-74
(Open3D 0.13 ``PointCloud::VoxelDownSample``; Open3D itself is absent here, the
semantics are those restated in oracle/voxel_oracle.cpp -- parity vs Open3D
unpinned beyond its published algorithm).  Every call runs on libpcr
(``pcr_voxel_down_sample``, csrc/voxel.hip): keys, sort, per-voxel sums on the
GPU, the unordered_map emission order replayed on the host.

* ``voxel_down_sample(pcd, voxel_size) -> PointCloud`` (also the
  ``PointCloud.voxel_down_sample`` method of registration.PointCloud);
* ``voxel_down_sample_batch(clouds, voxel_size, normals=None, colors=None)`` for
  many clouds in one call.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .registration import PointCloud, _device, _stream


def _f64_dev(x, dev):
    t = x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(x))
    return t.to(device=dev, dtype=torch.float64).reshape(-1, 3).contiguous()


def voxel_down_sample_batch(clouds, voxel_size, normals=None, colors=None):
    """clouds: list of (n_i, 3) arrays / tensors.  Returns a list of
    (points (k_i, 3), normals or None, colors or None) f64 device tensors."""
    dev = None
    for c in clouds:
        if isinstance(c, torch.Tensor) and c.is_cuda:
            dev = c.device
            break
    dev = dev or _device()
    pts = [_f64_dev(c, dev) for c in clouds]
    lens = np.array([p.shape[0] for p in pts], np.int32)
    n = int(lens.sum())
    P = torch.cat(pts, 0) if n else torch.zeros((0, 3), dtype=torch.float64, device=dev)
    Nr = None if normals is None else torch.cat([_f64_dev(x, dev) for x in normals], 0)
    Cl = None if colors is None else torch.cat([_f64_dev(x, dev) for x in colors], 0)
    for name, extra in (("normals", Nr), ("colors", Cl)):
        if extra is not None and extra.shape[0] != n:
            raise ValueError(f"{name} must have one row per point")
    cap = max(n, 1)
    op = torch.empty((cap, 3), dtype=torch.float64, device=dev)
    on = torch.empty((cap, 3), dtype=torch.float64, device=dev) if Nr is not None else None
    oc = torch.empty((cap, 3), dtype=torch.float64, device=dev) if Cl is not None else None
    out_len = np.zeros(len(pts), np.int32)
    total = np.zeros(1, np.int32)
    with torch.cuda.device(dev):
        _lib.call("pcr_voxel_down_sample", _lib.ptr(P), n, lens.ctypes.data_as(_lib._p), len(pts),
                  float(voxel_size), _lib.ptr(Nr), _lib.ptr(Cl), _lib.ptr(op), _lib.ptr(on),
                  _lib.ptr(oc), out_len.ctypes.data_as(_lib._p), total.ctypes.data_as(_lib._p),
                  _stream(dev))
    out, pos = [], 0
    for k in out_len:
        k = int(k)
        out.append((op[pos:pos + k], on[pos:pos + k] if on is not None else None,
                    oc[pos:pos + k] if oc is not None else None))
        pos += k
    return out


def voxel_down_sample(pcd, voxel_size):
    """Drop-in for ``o3d.geometry.PointCloud.voxel_down_sample(voxel_size)``:
    a new PointCloud with the voxel means (numpy f64, Open3D's order), normals
    and colors averaged too when the input has them."""
    pts = pcd.points if hasattr(pcd, "points") else pcd
    nrm = getattr(pcd, "normals", None)
    col = getattr(pcd, "colors", None)
    has_n = nrm is not None and len(nrm) > 0
    has_c = col is not None and len(col) > 0
    (p, n, c), = voxel_down_sample_batch([pts], voxel_size, [nrm] if has_n else None,
                                         [col] if has_c else None)
    out = PointCloud(p.cpu().numpy())
    if n is not None:
        out.normals = n.cpu().numpy()
    if c is not None:
        out.colors = c.cpu().numpy()
    return out
