"""f3: the Chamfer / nearest-distance consumers either side of the path, on the
nnd kernels (libpcr a1).

* ``chamfer_distance(p1, p2)``  -- DataPreparation/QualityCheck.py:25-31: mean
  Euclidean (not squared) 1-NN distance both ways, float32 inputs (the reference
  uses two sklearn KD-trees).
* ``hausdorff_distance(p1, p2)`` -- QualityCheck.py:13-23 (scipy
  directed_hausdorff both ways, max).
* ``overlap_masks(src, tgt, dist_thresh)`` -- ROPNet's overlap ground truth
  (ROPNet/src/eval.py:59-65, loss/loss.py:54-55 Ol_loss): ``min_j d2 < thresh^2``
  per source point and ``min_i d2 < thresh^2`` per target point, where the
  reference forms the full (B, N, M) matrix with utils/process.py:14-27
  square_dists and reduces it.
* ``min_square_dists(points1, points2)`` -- those two reductions themselves.

The squared distances are the nnd contract, ``(dx*dx + dy*dy) + dz*dz`` in f32
(direct form).  The references compute them differently (sklearn / scipy in f64,
ROPNet in the expanded ``|a|^2 + |b|^2 - 2 a.b`` f32 form), so values agree to
rounding (tests/test_quality_gpu.py states the tolerances) and a threshold test
can only differ for a distance within that rounding of the threshold.
"""
from __future__ import annotations

import numpy as np
import torch

from .nndistance import nnd_forward_cuda
from .registration import _cuda


def _cloud(p):
    pts = p.points if hasattr(p, "points") else p
    t = _cuda(np.asarray(pts, dtype=np.float32) if not isinstance(pts, torch.Tensor) else pts,
              torch.float32)
    if t.dim() == 2:
        t = t.unsqueeze(0)
    if t.dim() != 3 or t.shape[2] != 3:
        raise ValueError("points must be (N, 3) or (B, N, 3)")
    return t


def _nn2(a, b):
    B, N, M = a.shape[0], a.shape[1], b.shape[1]
    d1 = torch.empty(B, N, device=a.device)
    d2 = torch.empty(B, M, device=a.device)
    i1 = torch.empty(B, N, dtype=torch.int32, device=a.device)
    i2 = torch.empty(B, M, dtype=torch.int32, device=a.device)
    nnd_forward_cuda(a, b, d1, d2, i1, i2)
    return d1, d2


def min_square_dists(points1, points2):
    """(torch.min(square_dists(p1, p2), -1)[0], torch.min(..., 1)[0]): (B,N), (B,M) f32."""
    return _nn2(_cloud(points1), _cloud(points2))


def overlap_masks(src, tgt, dist_thresh=0.05):
    """ROPNet overlap labels: (src (B,N) bool, tgt (B,M) bool)."""
    d1, d2 = min_square_dists(src, tgt)
    thr = dist_thresh * dist_thresh
    return d1 < thr, d2 < thr


def chamfer_distance(p1, p2):
    """QualityCheck.chamfer_distance: mean 1-NN Euclidean distance p1->p2 plus p2->p1
    (a Python float, like the reference's numpy scalar)."""
    d1, d2 = _nn2(_cloud(p1), _cloud(p2))
    return float(torch.sqrt(d1.double()).mean() + torch.sqrt(d2.double()).mean())


def hausdorff_distance(original_cloud, aug_cloud):
    """QualityCheck.hausdorffDistance: max of the two directed Hausdorff distances."""
    d1, d2 = _nn2(_cloud(original_cloud), _cloud(aug_cloud))
    return float(torch.sqrt(torch.maximum(d1.max(), d2.max()).double()))
