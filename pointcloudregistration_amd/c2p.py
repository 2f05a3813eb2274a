"""C2P-Net's registration flow on libpcr: level voting, feature
RANSAC and the NDP non-rigid refinement, with the reference's names.

  get_coor_points              c2p-net/ngenet/models/vote.py:6-9
  vote                         c2p-net/ngenet/models/vote.py:12-37
  execute_global_registration  c2p-net/ngenet/utils/o3d.py:164-184
  register_c2p                 c2p-net/testScript.py:161-196 (vote -> global
                               registration -> NDP on the unique inlier sources)

The three nearest-target searches of vote run as one batched feature screen
(pcr_feature_match, P = 3 levels when they share a shape) and the distance tests
plus the row replacement as one kernel (pcr_vote_apply); the indices are the
exact f64 argmin (the reference's torch.cdist + min in f32 agrees wherever the
two nearest distances are not within f32 rounding of each other).

numpy inputs are updated in place and returned as numpy, like the reference;
device tensors stay on the device (and are likewise updated in place).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .registration import (CorrespondenceCheckerBasedOnDistance,
                           CorrespondenceCheckerBasedOnEdgeLength, Feature, PointCloud,
                           RANSACConvergenceCriteria, RansacParams,
                           TransformationEstimationPointToPoint, _cuda, _device,
                           feature_match, register_feature_ransac_batch,
                           registration_ransac_based_on_feature_matching, transform_batch)


def _rows(x, dev):
    t = _cuda(x, torch.float32, dev)
    if t.dim() != 2:
        raise ValueError("features must be (N, D)")
    return t


def _nn_levels(S, T):
    """nearest target per source row at each level, (3, n) int32 on the device"""
    if all(s.shape == S[0].shape for s in S) and all(t.shape == T[0].shape for t in T):
        nn12, _ = feature_match(torch.stack(S), torch.stack(T))
        return nn12
    return torch.stack([feature_match(s, t)[0][0] for s, t in zip(S, T)])


def get_coor_points(source_feats_npy, target_feats_npy, target_npy, use_cuda=True):
    """vote.py:6-9: (target[inds], inds) with inds = nearest target row in feature
    space of every source row."""
    dev = _device()
    nn12, _ = feature_match(_rows(source_feats_npy, dev), _rows(target_feats_npy, dev))
    inds = nn12[0]
    if isinstance(target_npy, torch.Tensor):
        return target_npy[inds.to(target_npy.device).long()], inds
    inds = inds.cpu().numpy().astype(np.int64)
    return np.asarray(target_npy)[inds], inds


def vote(source_npy, target_npy, source_feats, target_feats, voxel_size, use_cuda=True,
         return_mask=False):
    """vote.py:12-37: where the m and l levels agree on a target (within 2 voxel)
    and h agrees with neither, the source's h row and its m-target's h row are
    replaced by the m rows.  Returns [source, target, source_feats_h,
    target_feats_h] (+ the replaced mask (n,) bool when return_mask)."""
    dev = _device()
    fs_in, ft_in = list(source_feats), list(target_feats)
    if len(fs_in) != 3 or len(ft_in) != 3:
        raise ValueError("vote takes (h, m, l) feature levels for source and target")
    S = [_rows(f, dev) for f in fs_in]
    T = [_rows(f, dev) for f in ft_in]
    n, D = S[0].shape
    m = T[0].shape[0]
    if S[1].shape != (n, D) or T[1].shape != (m, D):
        raise ValueError("the h and m levels must share their shape (rows are copied m -> h)")
    if S[2].shape[0] != n or T[2].shape[0] != m:
        raise ValueError("every level must have the same rows as the clouds")
    tgt = _cuda(target_npy, torch.float32, dev).reshape(-1, 3)
    if tgt.shape[0] != m:
        raise ValueError("target_npy and target_feats disagree on the number of points")
    nn = _nn_levels(S, T)
    rep = torch.empty(n, dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        _lib.call("pcr_vote_apply", _lib.ptr(tgt), m, _lib.ptr(nn[0]), _lib.ptr(nn[1]),
                  _lib.ptr(nn[2]), n, float(voxel_size), _lib.ptr(S[0]), _lib.ptr(S[1]),
                  _lib.ptr(T[0]), _lib.ptr(T[1]), D, _lib.ptr(rep), _lib.stream_handle(dev))
    fs_h, ft_h = S[0], T[0]
    if isinstance(fs_in[0], np.ndarray):
        fs_in[0][...] = fs_h.cpu().numpy()
        fs_h = fs_in[0]
    elif fs_h.data_ptr() != fs_in[0].data_ptr():
        fs_in[0].copy_(fs_h)
        fs_h = fs_in[0]
    if isinstance(ft_in[0], np.ndarray):
        ft_in[0][...] = ft_h.cpu().numpy()
        ft_h = ft_in[0]
    elif ft_h.data_ptr() != ft_in[0].data_ptr():
        ft_in[0].copy_(ft_h)
        ft_h = ft_in[0]
    out = [source_npy, target_npy, fs_h, ft_h]
    if return_mask:
        return out, rep.bool()
    return out


def execute_global_registration(source, target, source_feats, target_feats, voxel_size, seed=0):
    """o3d.py:164-184: mutual feature RANSAC at distance voxel_size (EdgeLength
    0.9, Distance(voxel_size), 100000 / 0.999) -> (T, estimate, result), estimate =
    a transformed copy of source."""
    result = registration_ransac_based_on_feature_matching(
        source, target, source_feats, target_feats, True, voxel_size,
        TransformationEstimationPointToPoint(False), 3,
        [CorrespondenceCheckerBasedOnEdgeLength(0.9),
         CorrespondenceCheckerBasedOnDistance(voxel_size)],
        RANSACConvergenceCriteria(100000, 0.999), seed=seed)
    T = result.transformation
    pts = source.points if hasattr(source, "points") else source
    estimate = PointCloud(np.array(pts, dtype=np.float64).reshape(-1, 3))
    estimate.transform(T)
    return T, estimate, result


def register_c2p(source, target, source_feats, target_feats, voxel_size, dist_thresh=None,
                 ndp_config=None, NDP=None, seed=0, pair_id=0, use_graph=True):
    """testScript.py:161-196 on the device: vote -> RANSAC (distance dist_thresh,
    default voxel_size: dist_thresh_maps['10000'] = first_subsampling_dl) ->
    estimate = T source (f64, then f32 as the reference's .float()) -> NDP
    optimisation on the unique inlier source indices.  Returns a dict with
    T (4,4) f64, warped (n,3) f32 cuda, corrs (K,) int64, the RANSAC result
    fields and the NDP per-level info."""
    from .ndp_opt import optimize_deformation_pyramid
    dev = _device()
    src = _cuda(source, torch.float32, dev).reshape(-1, 3)
    tgt = _cuda(target, torch.float32, dev).reshape(-1, 3)
    S = [_rows(f, dev).clone() for f in source_feats]
    T = [_rows(f, dev).clone() for f in target_feats]
    _, _, fs_h, ft_h = vote(src, tgt, S, T, voxel_size)
    d = float(voxel_size if dist_thresh is None else dist_thresh)
    prm = RansacParams(max_correspondence_distance=d, distance_check=d, seed=seed)
    br = register_feature_ransac_batch(src, tgt, fs_h, ft_h, prm,
                                       pair_ids=torch.tensor([pair_id], dtype=torch.int32),
                                       want_mask=False)
    est = transform_batch(src.unsqueeze(0), br.transformation)[0]
    ct = br.corr_tgt[0]
    corrs = torch.nonzero(ct >= 0).flatten()  # ascending = np.unique of the set's sources
    warped, hist, _, info = optimize_deformation_pyramid(est, tgt, corrs.cpu().numpy(),
                                                         ndp_config, NDP, use_graph=use_graph)
    return {"T": br.transformation[0], "fitness": br.fitness[0], "inlier_rmse": br.inlier_rmse[0],
            "estimate": est, "corrs": corrs, "warped": warped, "hist": hist, "info": info,
            "source_feats_h": fs_h, "target_feats_h": ft_h}


__all__ = ["get_coor_points", "vote", "execute_global_registration", "register_c2p", "Feature",
           "PointCloud"]
