"""a9: batched weighted Procrustes drop-ins on libpcr (HIP, gfx950).

* ``weighted_icp(src, tgt, weights, _EPS=1e-8) -> (R, t, transformed_src)`` mirrors
  ROPNet/src/models/model_utils.py:105-139 (weighted centroids with
  w/(sum w + eps), Kabsch via torch.svd with the +/-V[:,2] determinant fix).
* ``rigid_fit(X, Y, w, eps=1e-4) -> (R, t)`` mirrors
  c2p-net/deformationpyramid/model/geometry.py:8-34 (|w|-normalised weights,
  f64 SVD on the CPU with diag(1,1,det U det V)), t shaped (B, 3, 1).

Both solve the same optimum (the best proper rotation) with Horn's quaternion
method in f64 on the GPU; the reference's f32 torch results agree to f32
rounding (tests/test_procrustes_golden.py pins this against fixtures generated
by importing the reference).
"""
from __future__ import annotations

import torch

from . import _lib


def procrustes_batch(src, tgt, weights, abs_weights, eps):
    """(B,N,3),(B,N,3),(B,N) -> T (B,3,4) f64 on the GPU: tgt ~ R src + t.
    f64 sources run on f64 inputs (pcr_procrustes_batch_f64), anything else on
    f32 (pcr_procrustes_batch); the sums and the solve are f64 either way."""
    S = torch.as_tensor(src)
    dev = S.device if S.is_cuda else torch.device("cuda", torch.cuda.current_device())
    dt = torch.float64 if S.dtype == torch.float64 else torch.float32
    S = S.to(dev, dt).contiguous()
    G = torch.as_tensor(tgt).to(dev, dt).contiguous()
    W = torch.as_tensor(weights).to(dev, dt).reshape(S.shape[0], S.shape[1]).contiguous()
    if S.dim() != 3 or S.shape[2] != 3 or G.shape != S.shape:
        raise ValueError("src/tgt must both be (B, N, 3)")
    B, N = S.shape[0], S.shape[1]
    T = torch.empty(B, 3, 4, dtype=torch.float64, device=dev)
    with torch.cuda.device(dev):
        _lib.call("pcr_procrustes_batch_f64" if dt == torch.float64 else "pcr_procrustes_batch",
                  _lib.ptr(S), _lib.ptr(G), _lib.ptr(W), B, N,
                  int(abs_weights), float(eps), _lib.ptr(T), _lib.stream_handle(dev))
    return T


def weighted_icp(src, tgt, weights, _EPS=1e-8):
    """Drop-in for ROPNet weighted_icp: returns R (B,3,3), t (B,3), transformed_src."""
    if not src.is_cuda:
        raise _lib.PcrError("weighted_icp: libpcr needs GPU tensors")
    T = procrustes_batch(src, tgt, weights, 0, _EPS)
    R = T[:, :, :3].to(src.dtype)
    t = T[:, :, 3].to(src.dtype)
    transformed_src = torch.matmul(src, R.permute(0, 2, 1).contiguous()) + t.unsqueeze(1)
    return R, t, transformed_src


def rigid_fit(X, Y, w, eps=0.0001):
    """Drop-in for NDP rigid_fit: returns R (B,3,3), t (B,3,1) on X's device."""
    if not X.is_cuda:
        raise _lib.PcrError("rigid_fit: libpcr needs GPU tensors")
    T = procrustes_batch(X, Y, w.reshape(X.shape[0], X.shape[1]), 1, eps)
    return T[:, :, :3].to(X.dtype), T[:, :, 3:4].to(X.dtype)
