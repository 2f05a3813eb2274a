"""DIP's registration demo (dip/demo.py:64-188) on libpcr.

  demo_register   one source/target pair through demo.py's sequence:
                  voxel_down_sample(1.0) (:73-74) -> np.random.choice of 2048
                  points per cloud (:80-87) -> LRF patches of every sampled point,
                  draws interleaved frag1 i / frag2 i (:109-114) -> descriptor
                  network in batches of 500 (:128-147; stays PyTorch, passed in)
                  -> 5th-percentile filter on |mx| (:149-156) -> feature RANSAC at
                  1.5 voxel (:37-53, :178)
  percentile_keep the filter of :149-153

The voxel step, the LRF frames and patches, the feature matching and RANSAC run
on libpcr; the draws use the caller's numpy RNG in the demo's order, so a seeded
caller gets the demo's samples and patches.  `estimate_normals()` (:76-77) is
skipped: nothing downstream reads the normals (only the demo's visualisation).
The sampled voxel means stay f64 through the LRF (Open3D stores double); RANSAC
takes them as f32 (libpcr's registration kernels are f32-coordinate, like the
C1/C4/C5 inputs), a deviation below 1e-5 mm at the demo's mm scale.
"""
from __future__ import annotations

import numpy as np
import torch

from . import lrf as _lrf
from .registration import (CorrespondenceCheckerBasedOnDistance,
                           CorrespondenceCheckerBasedOnEdgeLength, Feature, PointCloud,
                           RANSACConvergenceCriteria, TransformationEstimationPointToPoint,
                           registration_ransac_based_on_feature_matching)

GREY = [128 / 255, 128 / 255, 128 / 255]
BLUE = [0 / 255, 76 / 255, 153 / 255]


def percentile_keep(mx, perc=5):
    """demo.py:149-153: rows whose |mx| (f64 norm) exceeds the perc-th percentile"""
    mx = np.asarray(mx, np.float64)
    mag = np.linalg.norm(mx.reshape(mx.shape[0], -1), axis=1)  # (B, 256) or (B, 256, 1)
    return mag > np.percentile(mag, perc)


def execute_global_registration(source_down, target_down, source_fpfh, target_fpfh, voxel_size,
                                seed=0):
    """demo.py:37-53: mutual feature RANSAC at 1.5 voxel, EdgeLength(0.9),
    Distance(1.5 voxel), (100000, 0.999)."""
    d = voxel_size * 1.5
    return registration_ransac_based_on_feature_matching(
        source_down, target_down, source_fpfh, target_fpfh, True, d,
        TransformationEstimationPointToPoint(False), 3,
        [CorrespondenceCheckerBasedOnEdgeLength(0.9), CorrespondenceCheckerBasedOnDistance(d)],
        RANSACConvergenceCriteria(100000, 0.999), seed=seed)


def _describe(net, patches, batch_size):
    """demo.py:128-147: f, mx for (Q, 3, ps) patches in batches (f32 on the device,
    like torch.Tensor(patches).cuda()); returned as f64 numpy like the demo's
    np.empty buffers."""
    f_out, mx_out = [], []
    for s in range(0, patches.shape[0], batch_size):
        b = patches[s:s + batch_size].to(torch.float32)
        with torch.no_grad():
            out = net(b)
        f, mx = out[0], out[1]
        f_out.append(f.detach().to(torch.float64).cpu().numpy())
        mx_out.append(mx.detach().to(torch.float64).cpu().numpy().reshape(b.shape[0], -1))
    return np.concatenate(f_out), np.concatenate(mx_out)


def demo_register(source, target, net, voxel_size=1.0, lrf_kernel=3.0 * np.sqrt(3),
                  patch_size=256, pts_to_sample=2048, perc=5, batch_size=500, seed=0):
    """One pair through dip/demo.py:64-178.  `net(patches (B,3,ps) f32 cuda) ->
    (f (B,dim), mx (B,256), ...)` is the descriptor network (PointNetFeature in the
    reference).  Returns a dict with the RANSAC result and the intermediates
    (down-sampled clouds, sample indices, patches, descriptors, keep masks)."""
    pcd1, pcd2 = PointCloud(np.asarray(source)), PointCloud(np.asarray(target))
    pcd1.paint_uniform_color(GREY)
    pcd2.paint_uniform_color(BLUE)
    pcd1 = pcd1.voxel_down_sample(voxel_size)
    pcd2 = pcd2.voxel_down_sample(voxel_size)
    p1, p2 = np.asarray(pcd1.points), np.asarray(pcd2.points)
    inds1 = np.random.choice(p1.shape[0], pts_to_sample, replace=False)
    inds2 = np.random.choice(p2.shape[0], pts_to_sample, replace=False)
    pts1, pts2 = p1[inds1], p2[inds2]
    patches1, patches2 = _lrf.demo_patches(p1, p2, pts1, pts2, lrf_kernel, patch_size)
    desc1, mx1 = _describe(net, patches1, batch_size)
    desc2, mx2 = _describe(net, patches2, batch_size)
    good1, good2 = percentile_keep(mx1, perc), percentile_keep(mx2, perc)
    f1, f2 = Feature(desc1[good1].T), Feature(desc2[good2].T)
    result = execute_global_registration(PointCloud(pts1[good1]), PointCloud(pts2[good2]), f1, f2,
                                         voxel_size, seed=seed)
    return {"result": result, "pcd1": pcd1, "pcd2": pcd2, "inds1": inds1, "inds2": inds2,
            "patches1": patches1, "patches2": patches2, "desc1": desc1, "desc2": desc2,
            "good1": good1, "good2": good2}


def _block(layer, n):
    return torch.nn.Sequential(layer, torch.nn.Dropout(p=0.5), torch.nn.BatchNorm1d(n), torch.nn.ReLU())


class _STN3d(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = _block(torch.nn.Conv1d(3, 128, 1), 128)
        self.conv2 = _block(torch.nn.Conv1d(128, 256, 1), 256)
        self.fc1 = _block(torch.nn.Linear(256, 128), 128)
        self.fc2 = torch.nn.Sequential(torch.nn.Linear(128, 9))

    def forward(self, x):
        x = self.conv2(self.conv1(x)).max(dim=2)[0]
        x = self.fc2(self.fc1(x)) + torch.eye(3, device=x.device, dtype=x.dtype).reshape(1, 9)
        return x.view(-1, 3, 3)


class PointNetFeature(torch.nn.Module):
    """The architecture of DIP's descriptor network (dip/network.py:50-122:
    T-net, Conv1d 3->128->256 with BatchNorm, max-pool, Linear 256->128->dim,
    l2-normalised), with the same parameter names so the reference's state dict
    loads into it.  It stays PyTorch (not on the hot path); with a seeded random
    init it is SURVEY 8(d)'s C3 descriptor for tests and the bench.  forward(x)
    -> (f (B, dim), mx (B, 256, 1), amx) as the demo calls it (:137)."""

    def __init__(self, dim=64, l2norm=True, tnet=True):
        super().__init__()
        self.l2norm, self.tnet = l2norm, tnet
        self.stn3d = _STN3d()
        self.conv1 = _block(torch.nn.Conv1d(3, 128, 1), 128)
        self.conv2 = _block(torch.nn.Conv1d(128, 256, 1), 256)
        self.fc1 = _block(torch.nn.Linear(256, 128), 128)
        self.fc2 = torch.nn.Sequential(torch.nn.Linear(128, dim))

    def forward(self, x):
        if self.tnet:
            x = torch.bmm(self.stn3d(x), x)
        x = self.conv2(self.conv1(x))
        mx, amx = torch.max(x, 2, keepdim=True)
        f = self.fc2(self.fc1(mx.view(-1, 256)))
        if self.l2norm:
            f = torch.nn.functional.normalize(f, p=2, dim=1)
        return f, mx, amx


__all__ = ["demo_register", "execute_global_registration", "percentile_keep", "PointNetFeature"]
