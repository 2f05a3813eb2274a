"""f1: normal estimation + FPFH on the GPU.

Mirrors the two Open3D calls of DataPreparation/RANSAC.py:12-22
(``preprocess_point_cloud``)::

    pcd.estimate_normals(o3d.geometry.KDTreeSearchParamHybrid(radius=4*voxel, max_nn=30))
    fpfh = o3d.pipelines.registration.compute_fpfh_feature(
        pcd, o3d.geometry.KDTreeSearchParamHybrid(radius=7*voxel, max_nn=100))

with the same names, argument meaning and result layout (``Feature.data`` is
(33, N) f64), plus batched forms over P clouds for the pair-sharded pipeline.
Every call runs on libpcr (``pcr_hybrid_search`` / ``pcr_estimate_normals`` /
``pcr_compute_fpfh``, csrc/fpfh.hip); there is no CPU path.  Open3D is absent
in this image, so the semantics are those of the restatement in
oracle/fpfh_oracle.c (parity vs Open3D unpinned; GPU == restatement bit for bit).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .registration import Feature, PointCloud, _batch3, _counts, _cuda, _stream

MAX_NN_LIMIT = 448


class KDTreeSearchParamHybrid:
    """o3d.geometry.KDTreeSearchParamHybrid(radius, max_nn)."""

    def __init__(self, radius, max_nn):
        self.radius = float(radius)
        self.max_nn = int(max_nn)

    def __repr__(self):
        return f"KDTreeSearchParamHybrid with radius = {self.radius:f} and max_nn = {self.max_nn:d}"


def _param(p):
    if not isinstance(p, KDTreeSearchParamHybrid) and not (hasattr(p, "radius") and
                                                           hasattr(p, "max_nn")):
        raise TypeError("search_param must be a KDTreeSearchParamHybrid(radius, max_nn)")
    r, k = float(p.radius), int(p.max_nn)
    if not (r > 0.0 and np.isfinite(r)):
        raise ValueError("radius must be finite and > 0")
    if not 1 <= k <= MAX_NN_LIMIT:
        raise ValueError(f"max_nn must be in [1, {MAX_NN_LIMIT}]")
    return r, k


# --------------------------------------------------------------------------
# batched API: (P, N, 3) f32 device clouds, optional per-cloud counts
# --------------------------------------------------------------------------


def hybrid_search_batch(xyz, radius, max_nn, n_pts=None):
    """KDTreeFlann.search_hybrid_vector_3d for every point of every cloud:
    (idx (P,N,K) int32, d2 (P,N,K) f64, counts (P,N) int32) on the GPU."""
    x = _batch3(xyz, "xyz")
    P, N = x.shape[0], x.shape[1]
    dev = x.device
    n = _counts(n_pts, P, dev)
    idx = torch.empty((P, N, max_nn), dtype=torch.int32, device=dev)
    d2 = torch.empty((P, N, max_nn), dtype=torch.float64, device=dev)
    cnt = torch.zeros((P, N), dtype=torch.int32, device=dev)
    _lib.call("pcr_hybrid_search", _lib.ptr(x), P, N, _lib.ptr(n), float(radius), int(max_nn),
              _lib.ptr(idx), _lib.ptr(d2), _lib.ptr(cnt), _stream(dev))
    return idx, d2, cnt


def estimate_normals_batch(xyz, radius, max_nn, n_pts=None, prior_normals=None):
    """Normals (P, N, 3) f64 of P clouds (EstimateNormals, fast_normal_computation)."""
    x = _batch3(xyz, "xyz")
    P, N = x.shape[0], x.shape[1]
    dev = x.device
    n = _counts(n_pts, P, dev)
    prior = None
    if prior_normals is not None:
        prior = _cuda(prior_normals, torch.float64, dev).reshape(P, N, 3)
    out = torch.zeros((P, N, 3), dtype=torch.float64, device=dev)
    _lib.call("pcr_estimate_normals", _lib.ptr(x), P, N, _lib.ptr(n), float(radius), int(max_nn),
              _lib.ptr(prior), _lib.ptr(out), _stream(dev))
    return out


def compute_fpfh_batch(xyz, normals, radius, max_nn, n_pts=None, want_spfh=False):
    """FPFH (P, N, 33) f64 and its f32 rounding (the feature-matching input);
    with want_spfh also the SPFH histograms."""
    x = _batch3(xyz, "xyz")
    P, N = x.shape[0], x.shape[1]
    dev = x.device
    n = _counts(n_pts, P, dev)
    nm = _cuda(normals, torch.float64, dev).reshape(P, N, 3)
    f64 = torch.zeros((P, N, 33), dtype=torch.float64, device=dev)
    f32 = torch.zeros((P, N, 33), dtype=torch.float32, device=dev)
    sp = torch.zeros((P, N, 33), dtype=torch.float64, device=dev) if want_spfh else None
    _lib.call("pcr_compute_fpfh", _lib.ptr(x), _lib.ptr(nm), P, N, _lib.ptr(n), float(radius),
              int(max_nn), _lib.ptr(f64), _lib.ptr(f32), _lib.ptr(sp), _stream(dev))
    return (f64, f32, sp) if want_spfh else (f64, f32)


# --------------------------------------------------------------------------
# Open3D-shaped drop-ins (RANSAC.py:12-22)
# --------------------------------------------------------------------------


def _cloud_xyz(pcd):
    pts = pcd.points if hasattr(pcd, "points") else pcd
    if isinstance(pts, torch.Tensor):
        return pts.reshape(-1, 3), True
    return np.asarray(pts, dtype=np.float64).reshape(-1, 3), False


def estimate_normals(pcd, search_param, fast_normal_computation=True):
    """pcd.estimate_normals(search_param): sets ``pcd.normals`` (N, 3) f64 (numpy for a
    numpy cloud, a CUDA tensor for a tensor cloud) and returns it.  Normals the cloud
    already holds orient the result, as Open3D's has_normal branch does."""
    if not fast_normal_computation:
        raise NotImplementedError("fast_normal_computation=False (Eigen solver) is not built")
    r, k = _param(search_param)
    xyz, is_t = _cloud_xyz(pcd)
    prior = getattr(pcd, "normals", None)
    if prior is not None and len(prior) != len(xyz):
        prior = None
    out = estimate_normals_batch(_cuda(xyz, torch.float32), r, k,
                                 prior_normals=prior if prior is not None else None)[0]
    res = out if is_t else out.cpu().numpy()
    if hasattr(pcd, "points"):
        pcd.normals = res
    return res


def compute_fpfh_feature(pcd, search_param):
    """o3d.pipelines.registration.compute_fpfh_feature(input, search_param) -> Feature
    with ``.data`` (33, N) f64; ``.data32`` keeps the f32 (N, 33) rows on the GPU for
    registration_ransac_based_on_feature_matching."""
    r, k = _param(search_param)
    xyz, is_t = _cloud_xyz(pcd)
    nm = getattr(pcd, "normals", None)
    if nm is None or len(nm) != len(xyz):
        raise ValueError("compute_fpfh_feature: the point cloud has no normals "
                         "(Open3D errors out here as well); call estimate_normals first")
    f64, f32 = compute_fpfh_batch(_cuda(xyz, torch.float32), nm, r, k)
    data = f64[0].t() if is_t else f64[0].cpu().numpy().T
    feat = Feature(data)
    feat.data32 = f32[0]
    return feat


def preprocess_point_cloud(pcd, voxel_size):
    """RANSAC.py:12-22 in one call: normals (4 voxel, 30) then FPFH (7 voxel, 100)."""
    estimate_normals(pcd, KDTreeSearchParamHybrid(radius=voxel_size * 4, max_nn=30))
    fpfh = compute_fpfh_feature(pcd, KDTreeSearchParamHybrid(radius=voxel_size * 7, max_nn=100))
    return pcd, fpfh


__all__ = ["KDTreeSearchParamHybrid", "PointCloud", "Feature", "hybrid_search_batch",
           "estimate_normals_batch", "compute_fpfh_batch", "estimate_normals",
           "compute_fpfh_feature", "preprocess_point_cloud"]
