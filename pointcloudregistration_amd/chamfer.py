"""a3: Chamfer reductions on the nnd kernels (libpcr), with autograd.

* ``compute_truncated_chamfer_distance(x, y, trunc=1e9, ...)`` mirrors
  c2p-net/deformationpyramid/model/loss.py:60-218 as called by the NDP loop
  (registration.py:236): squared 1-NN distances both ways, entries >= trunc
  zeroed, point mean over the FULL length (the divisor keeps masked entries,
  loss.py:151-154,187-195), batch mean, cham_x + cham_y.  pytorch3d.knn_points
  is replaced by torch_nndistance's kernel (same squared-distance definition:
  (dx*dx+dy*dy)+dz*dz in f32, first index on ties).
* ``chamfer_distance(x, y)`` = pytorch3d.loss.chamfer_distance's default
  (mean/mean) as used by dip/train.py:84,113 (returns (loss, None)).

Homogeneous batches only (x (N,P1,3), y (N,P2,3)); the reference's
heterogeneous-length path (x_lengths) is not used by its callers.
"""
from __future__ import annotations

import torch

from .nndistance import nnd


def _check(x, y):
    if x.dim() != 3 or y.dim() != 3 or x.shape[2] != 3 or y.shape[2] != 3:
        raise ValueError("x, y must be (N, P, 3)")
    if x.shape[0] != y.shape[0]:
        raise ValueError("y does not have the correct shape.")


def compute_truncated_chamfer_distance(x, y, trunc=1e9, batch_reduction="mean",
                                       point_reduction="mean", weights=None):
    _check(x, y)
    if point_reduction not in ("mean", "sum"):
        raise ValueError('point_reduction must be one of ["mean", "sum"]')
    if batch_reduction not in (None, "mean", "sum"):
        raise ValueError('batch_reduction must be one of ["mean", "sum"] or None')
    N, P1, P2 = x.shape[0], x.shape[1], y.shape[1]
    if weights is not None:  # loss.py:127-139
        if weights.size(0) != N:
            raise ValueError("weights must be of shape (N,).")
        if not (weights >= 0).all():
            raise ValueError("weights cannot be negative.")
        if weights.sum() == 0.0:
            w = weights.view(N, 1)
            if batch_reduction in ("mean", "sum"):
                return ((x.sum((1, 2)) * w).sum() * 0.0, (x.sum((1, 2)) * w).sum() * 0.0)
            return ((x.sum((1, 2)) * w) * 0.0, (x.sum((1, 2)) * w) * 0.0)
    dist1, dist2 = nnd(x.float().contiguous(), y.float().contiguous())
    cham_x = torch.where(dist1 >= trunc, torch.zeros_like(dist1), dist1)
    cham_y = torch.where(dist2 >= trunc, torch.zeros_like(dist2), dist2)
    if weights is not None:
        cham_x = cham_x * weights.view(N, 1)
        cham_y = cham_y * weights.view(N, 1)
    cham_x = cham_x.sum(1)
    cham_y = cham_y.sum(1)
    if point_reduction == "mean":
        cham_x = cham_x / P1
        cham_y = cham_y / P2
    if batch_reduction is not None:
        cham_x = cham_x.sum()
        cham_y = cham_y.sum()
        if batch_reduction == "mean":
            div = weights.sum() if weights is not None else N
            cham_x = cham_x / div
            cham_y = cham_y / div
    return cham_x + cham_y


def chamfer_distance(x, y, batch_reduction="mean", point_reduction="mean"):
    """pytorch3d.loss.chamfer_distance(x, y) (no normals) -> (loss, None)."""
    return compute_truncated_chamfer_distance(x, y, float("inf"), batch_reduction,
                                              point_reduction), None
