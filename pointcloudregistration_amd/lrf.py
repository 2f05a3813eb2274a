"""a4: DIP local reference frames on the GPU (drop-in for dip/lrf.py).

`lrf` mirrors the reference class (dip/lrf.py:4-78): same constructor, and
`get(pt)` returns (patch (patch_size, 3), pt, T (4, 4)).  The frame and patch
come from libpcr (pcr_lrf_count / pcr_lrf_compute).  The reference's
`np.random.choice(ptall.shape[0], patch_size, replace=False)` (dip/lrf.py:76)
is drawn here on the host, from the same global numpy RNG and at the same
point in the call sequence, so a caller that seeds numpy gets the reference's
patches; a whole query set's draws run in one call of libpcr's restatement of
legacy RandomState.choice (pcr_legacy_choice_batch, csrc/legacy_choice.cpp)
instead of one Python call per query.  `get_batch` and `demo_patches` compute many queries in two launches
while drawing the indices in the reference's per-call order.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


def _points(pcd):
    pts = pcd.points if hasattr(pcd, "points") else pcd
    return np.asarray(pts, dtype=np.float64).reshape(-1, 3)


def legacy_choice_batch(pops, k, random_state=None):
    """[np.random.choice(n, k, replace=False) for n in pops] as one (len(pops), k)
    int32 array, drawn by libpcr's host restatement (pcr_legacy_choice_batch) on
    the stream of `random_state` (default: numpy's global RandomState), which is
    left exactly where the Python loop would leave it."""
    rs = random_state if random_state is not None else np.random.mtrand._rand
    name, key, pos, has_gauss, gauss = rs.get_state(legacy=True)
    if name != "MT19937":
        raise ValueError(f"legacy_choice_batch needs an MT19937 RandomState, got {name}")
    key = np.ascontiguousarray(key, dtype=np.uint32).copy()
    pos_c = np.array([pos], np.int32)
    pops = np.ascontiguousarray(pops, dtype=np.int32).reshape(-1)
    out = np.zeros((len(pops), int(k)), np.int32)
    if len(pops):
        _lib.call("pcr_legacy_choice_batch", key.ctypes.data, pos_c.ctypes.data, pops.ctypes.data,
                  len(pops), int(k), out.ctypes.data)
        rs.set_state((name, key, int(pos_c[0]), has_gauss, gauss))
    return out


def _draw(counts, patch_size, choice):
    pops = np.maximum(np.asarray(counts, np.int64), patch_size)
    if choice is None:
        return legacy_choice_batch(pops, patch_size)
    return np.stack([np.asarray(choice(int(c), patch_size), dtype=np.int32) for c in pops])


def _check_sparse(cnt, qn, kernel, allow_sparse):
    """dip/lrf.py:29-30: with fewer than kernel/2 neighbours the reference calls
    search_knn_vector_3d(pt, <float kernel>), which Open3D rejects -> it raises."""
    if allow_sparse:
        return
    bad = [(p, q) for p in range(cnt.shape[0]) for q in range(int(qn[p]))
           if cnt[p, q] < kernel / 2]
    if bad:
        raise ValueError(f"lrf: {len(bad)} queries have fewer than kernel/2 neighbours "
                         f"(first: pair {bad[0][0]} query {bad[0][1]}); the reference raises "
                         "there (dip/lrf.py:29-30). Pass allow_sparse=True for NaN frames.")


def lrf_batch(points, queries, kernel, patch_size, n_pts=None, n_q=None, inds=None,
              choice=None, device=None, allow_sparse=False):
    """Batched frames: points (P,N,3), queries (P,Q,3) (f64, any array type).

    Without `inds`, indices are drawn per query in (p, q) order with
    `choice(n, patch_size)` (default: np.random.choice without replacement).
    Returns (patches (P,Q,ps,3) f64, T (P,Q,4,4) f64, counts (P,Q) int32, inds)."""
    dev = torch.device(device) if device is not None else torch.device("cuda")
    if dev.type != "cuda":
        raise RuntimeError("lrf_batch needs a HIP device: the LRF runs only in libpcr")
    P_ = torch.as_tensor(np.asarray(points, np.float64), device=dev).contiguous()
    Q_ = torch.as_tensor(np.asarray(queries, np.float64), device=dev).contiguous()
    if P_.dim() == 2:
        P_, Q_ = P_.unsqueeze(0), Q_.unsqueeze(0)
    P, N, _ = P_.shape
    Qm = Q_.shape[1]
    if Q_.shape[0] != P or P_.shape[2] != 3 or Q_.shape[2] != 3:
        raise ValueError("points (P,N,3) and queries (P,Q,3) must agree on P")
    ns = None if n_pts is None else torch.as_tensor(np.asarray(n_pts, np.int32), device=dev)
    nq = None if n_q is None else torch.as_tensor(np.asarray(n_q, np.int32), device=dev)
    counts = torch.zeros(P, Qm, dtype=torch.int32, device=dev)
    stream = _lib.stream_handle(dev)
    with torch.cuda.device(dev):
        _lib.call("pcr_lrf_count", _lib.ptr(P_), P, N, _lib.ptr(ns), _lib.ptr(Q_), Qm,
                  _lib.ptr(nq), float(kernel), _lib.ptr(counts), stream)
    cnt = counts.cpu().numpy()
    qn = np.full(P, Qm) if n_q is None else np.minimum(np.asarray(n_q), Qm)
    _check_sparse(cnt, qn, kernel, allow_sparse)
    if inds is None:
        inds = np.zeros((P, Qm, patch_size), np.int32)
        for p in range(P):
            if qn[p] > 0:
                inds[p, :qn[p]] = _draw(cnt[p, :qn[p]], patch_size, choice)
    I_ = torch.as_tensor(np.asarray(inds, np.int32), device=dev).contiguous()
    patches = torch.zeros(P, Qm, patch_size, 3, dtype=torch.float64, device=dev)
    T = torch.zeros(P, Qm, 4, 4, dtype=torch.float64, device=dev)
    kmax = int(cnt.max()) if cnt.size else 0
    with torch.cuda.device(dev):
        _lib.call("pcr_lrf_compute", _lib.ptr(P_), P, N, _lib.ptr(ns), _lib.ptr(Q_), Qm,
                  _lib.ptr(nq), float(kernel), int(patch_size), _lib.ptr(I_), kmax,
                  _lib.ptr(patches), _lib.ptr(T), None, stream)
    return patches, T, counts, inds


class lrf:  # noqa: N801 - the reference's class name (dip/lrf.py:4)
    """Drop-in for dip/lrf.py's lrf class.  `pcd_tree` is accepted and unused:
    the neighbour search runs on the GPU with KDTreeFlann's radius semantics."""

    def __init__(self, pcd, pcd_tree, lrf_kernel, patch_size, viz=False):
        if viz:
            raise NotImplementedError("viz needs Open3D's visualiser (out of scope)")
        self.pcd = pcd
        self.pcd_tree = pcd_tree
        self.patch_kernel = float(lrf_kernel)
        self.patch_size = int(patch_size)
        self._pts = _points(pcd)

    def get(self, pt):
        patches, T, _, _ = lrf_batch(self._pts[None], np.asarray(pt, np.float64)[None, None],
                                     self.patch_kernel, self.patch_size)
        return patches[0, 0].cpu().numpy(), np.asarray(pt), T[0, 0].cpu().numpy()

    def get_batch(self, pts, choice=None):
        """Many queries at once; indices drawn in query order (= a loop of get)."""
        pts = np.asarray(pts, np.float64).reshape(-1, 3)
        patches, T, _, _ = lrf_batch(self._pts[None], pts[None], self.patch_kernel,
                                     self.patch_size, choice=choice)
        return patches[0], T[0]


def demo_patches(pcd1, pcd2, pts1, pts2, lrf_kernel, patch_size, choice=None):
    """dip/demo.py:109-114 in two launches: frames for pts1 in pcd1 and pts2 in
    pcd2, with the choice draws interleaved (frag1 i, frag2 i, frag1 i+1, ...)
    exactly as the demo's loop.  Returns patches1, patches2 as (Q, 3, ps)."""
    a, b = _points(pcd1), _points(pcd2)
    q1, q2 = np.asarray(pts1, np.float64), np.asarray(pts2, np.float64)
    if len(q1) != len(q2):
        raise ValueError("demo.py samples the same number of points from both clouds")
    N = max(len(a), len(b))
    P_ = np.zeros((2, N, 3))
    P_[0, :len(a)], P_[1, :len(b)] = a, b
    Q_ = np.stack([q1, q2])
    ns = np.array([len(a), len(b)], np.int32)
    # phase 1 alone to learn the counts, then draw in the demo's order
    dev = torch.device("cuda")
    Pt = torch.as_tensor(P_, device=dev).contiguous()
    Qt = torch.as_tensor(Q_, device=dev).contiguous()
    nst = torch.as_tensor(ns, device=dev)
    counts = torch.zeros(2, len(q1), dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        _lib.call("pcr_lrf_count", _lib.ptr(Pt), 2, N, _lib.ptr(nst), _lib.ptr(Qt), len(q1), None,
                  float(lrf_kernel), _lib.ptr(counts), _lib.stream_handle(dev))
    cnt = counts.cpu().numpy()
    _check_sparse(cnt, np.array([len(q1), len(q1)]), lrf_kernel, False)
    # the demo's call order: frag1 i, frag2 i, frag1 i+1, ...
    inds = _draw(cnt.T.reshape(-1), patch_size, choice).reshape(len(q1), 2, patch_size)
    inds = np.ascontiguousarray(inds.transpose(1, 0, 2))
    patches, _, _, _ = lrf_batch(P_, Q_, lrf_kernel, patch_size, n_pts=ns, inds=inds,
                                 allow_sparse=True)
    out = patches.transpose(2, 3)  # (2, Q, 3, ps) as demo.py's patchesX[i] = pts.T
    return out[0], out[1]
