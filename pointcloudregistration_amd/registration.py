"""Registration boundary: batched GPU API + Open3D-shaped drop-in façade.

Reference call shapes honoured (Boundary 2):
  * ``registration_ransac_based_on_feature_matching(source, target, source_feature,
    target_feature, mutual_filter, max_correspondence_distance, estimation_method,
    ransac_n, checkers, criteria)`` -> result with ``.transformation``,
    ``.correspondence_set``, ``.fitness``, ``.inlier_rmse``
    (DataPreparation/RANSAC.py:43-52, dip/demo.py:43-52, c2p-net/ngenet/utils/o3d.py:174-184);
  * ``registration_icp(source, target, max_correspondence_distance, init,
    estimation_method[, criteria])`` (DataPreparation/RANSAC.py:61-63);
  * ``register(src, tgt, src_feat, tgt_feat, **params) -> (R, t)`` (north star).

Open3D's RANSAC is OpenMP-parallel with a non-seedable RNG.  Here the
hypothesis stream is Philox keyed by (seed, pair_id, iteration) and the result is
exactly that of the sequential Open3D loop on that stream (oracle_ransac), so it
is reproducible run to run and bit-identical to the CPU restatement.

Every call runs on libpcr (HIP, gfx950); there is no CPU path.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib

# --------------------------------------------------------------------------
# tensor plumbing
# --------------------------------------------------------------------------


def _device():
    if not torch.cuda.is_available():
        raise _lib.PcrError("libpcr needs a ROCm GPU (gfx950); none is visible")
    return torch.device("cuda", torch.cuda.current_device())


def _cuda(x, dtype, device=None):
    if isinstance(x, torch.Tensor):
        t = x
    else:
        t = torch.from_numpy(np.ascontiguousarray(x))
    dev = device or (t.device if t.is_cuda else _device())
    return t.to(device=dev, dtype=dtype).contiguous()


def _batch3(x, name, device=None):
    t = _cuda(x, torch.float32, device)
    if t.dim() == 2:
        t = t.unsqueeze(0)
    if t.dim() != 3 or t.shape[2] != 3:
        raise ValueError(f"{name} must be (P, N, 3) or (N, 3)")
    return t


def _counts(n, P, device):
    if n is None:
        return None
    return _cuda(n, torch.int32, device).reshape(P)


def _stream(device):
    return _lib.stream_handle(device)


@dataclass
class RansacParams:
    """RANSAC parameters with Open3D's names and the reference's defaults
    (RANSAC.py:43-52: mutual, PointToPoint(False), n=3, EdgeLength(0.9),
    Distance(d), RANSACConvergenceCriteria(100000, 0.999))."""
    max_correspondence_distance: float
    edge_length_ratio: float = 0.9
    distance_check: float | None = None   # None -> = max_correspondence_distance
    confidence: float = 0.999
    max_iteration: int = 100000
    ransac_n: int = 3
    mutual_filter: bool = True
    seed: int = 0

    def to_c(self):
        dc = self.max_correspondence_distance if self.distance_check is None else self.distance_check
        return _lib.RansacParams(float(self.max_correspondence_distance),
                                 float(self.edge_length_ratio), float(dc), float(self.confidence),
                                 int(self.max_iteration), int(self.ransac_n),
                                 int(bool(self.mutual_filter)), 0, int(self.seed) & (2**64 - 1))


@dataclass
class IcpParams:
    max_correspondence_distance: float
    relative_fitness: float = 1e-6
    relative_rmse: float = 1e-6
    max_iteration: int = 30

    def to_c(self):
        return _lib.IcpParams(float(self.max_correspondence_distance),
                              float(self.relative_fitness), float(self.relative_rmse),
                              int(self.max_iteration), 0)


@dataclass
class BatchResult:
    """Per-pair results on the device (P = batch)."""
    transformation: torch.Tensor      # (P, 4, 4) f64
    fitness: torch.Tensor             # (P,) f64
    inlier_rmse: torch.Tensor         # (P,) f64
    stats: torch.Tensor               # (P, k) i32 (see pcr_api.h)
    corr_tgt: torch.Tensor | None = None      # (P, Nmax) i32, -1 = no correspondence
    inlier_mask: torch.Tensor | None = None   # (P, ceil(Nmax/32)) i32 bitset

    def correspondence_set(self, p=0):
        """(K, 2) int32 numpy array of (source, target) index pairs of pair p."""
        ct = self.corr_tgt[p].cpu().numpy()
        src = np.nonzero(ct >= 0)[0].astype(np.int32)
        return np.stack([src, ct[src]], axis=1).astype(np.int32)


# --------------------------------------------------------------------------
# batched GPU API
# --------------------------------------------------------------------------


def feature_match(src_feat, tgt_feat, n_src=None, n_tgt=None):
    """Exact feature-space 1-NN both ways: (nn12 (P,N), nn21 (P,M)) int32."""
    F = _cuda(src_feat, torch.float32)
    if F.dim() == 2:
        F = F.unsqueeze(0)
    G = _cuda(tgt_feat, torch.float32, F.device)
    if G.dim() == 2:
        G = G.unsqueeze(0)
    P, N, D = F.shape
    M = G.shape[1]
    if G.shape[0] != P or G.shape[2] != D:
        raise ValueError("src_feat (P,N,D) and tgt_feat (P,M,D) must agree on P and D")
    nn12 = torch.empty(P, N, dtype=torch.int32, device=F.device)
    nn21 = torch.empty(P, M, dtype=torch.int32, device=F.device)
    ns, nt = _counts(n_src, P, F.device), _counts(n_tgt, P, F.device)
    with torch.cuda.device(F.device):
        _lib.call("pcr_feature_match", _lib.ptr(F), _lib.ptr(G), P, N, M, D, _lib.ptr(ns),
                  _lib.ptr(nt), _lib.ptr(nn12), _lib.ptr(nn21), _stream(F.device))
    return nn12, nn21


def correspondences(nn12, nn21, n_src=None, n_tgt=None, mutual_filter=True, ransac_n=3):
    """Mutual filter + ordered compaction -> (corres (P,N,2), n_corres (P,))."""
    nn12 = _cuda(nn12, torch.int32)
    nn21 = _cuda(nn21, torch.int32, nn12.device)
    if nn12.dim() == 1:
        nn12, nn21 = nn12.unsqueeze(0), nn21.unsqueeze(0)
    P, N = nn12.shape
    M = nn21.shape[1]
    corres = torch.empty(P, N, 2, dtype=torch.int32, device=nn12.device)
    ncor = torch.empty(P, dtype=torch.int32, device=nn12.device)
    ns, nt = _counts(n_src, P, nn12.device), _counts(n_tgt, P, nn12.device)
    with torch.cuda.device(nn12.device):
        _lib.call("pcr_correspondences", _lib.ptr(nn12), _lib.ptr(nn21), P, N, M, _lib.ptr(ns),
                  _lib.ptr(nt), int(bool(mutual_filter)), int(ransac_n), _lib.ptr(corres),
                  _lib.ptr(ncor), _stream(nn12.device))
    return corres, ncor


def feature_correspondences(src_feat, tgt_feat, n_src=None, n_tgt=None, mutual_filter=True,
                            ransac_n=3):
    """feature_match + correspondences in one call, without nn21 for every target
    (pcr_feature_correspondences): -> (corres (P,N,2), n_corres (P,), nn12 (P,N)),
    bit-identical to correspondences(*feature_match(...))."""
    F = _cuda(src_feat, torch.float32)
    if F.dim() == 2:
        F = F.unsqueeze(0)
    G = _cuda(tgt_feat, torch.float32, F.device)
    if G.dim() == 2:
        G = G.unsqueeze(0)
    P, N, D = F.shape
    M = G.shape[1]
    if G.shape[0] != P or G.shape[2] != D:
        raise ValueError("src_feat (P,N,D) and tgt_feat (P,M,D) must agree on P and D")
    nn12 = torch.empty(P, N, dtype=torch.int32, device=F.device)
    corres = torch.empty(P, N, 2, dtype=torch.int32, device=F.device)
    ncor = torch.empty(P, dtype=torch.int32, device=F.device)
    ns, nt = _counts(n_src, P, F.device), _counts(n_tgt, P, F.device)
    with torch.cuda.device(F.device):
        _lib.call("pcr_feature_correspondences", _lib.ptr(F), _lib.ptr(G), P, N, M, D, _lib.ptr(ns),
                  _lib.ptr(nt), int(bool(mutual_filter)), int(ransac_n), _lib.ptr(nn12),
                  _lib.ptr(corres), _lib.ptr(ncor), _stream(F.device))
    return corres, ncor, nn12


def _ransac_outputs(P, N, dev, want_corr=True, want_mask=True):
    T = torch.empty(P, 4, 4, dtype=torch.float64, device=dev)
    fr = torch.empty(P, 2, dtype=torch.float64, device=dev)
    st = torch.empty(P, 5, dtype=torch.int32, device=dev)
    ct = torch.empty(P, N, dtype=torch.int32, device=dev) if want_corr else None
    mk = torch.empty(P, (N + 31) // 32, dtype=torch.int32, device=dev) if want_mask else None
    return T, fr, st, ct, mk


def ransac_batch(src, tgt, corres, n_corres, params: RansacParams, n_src=None, n_tgt=None,
                 pair_ids=None, want_corr=True, want_mask=True):
    S = _batch3(src, "src")
    G = _batch3(tgt, "tgt", S.device)
    P, N, M = S.shape[0], S.shape[1], G.shape[1]
    C = _cuda(corres, torch.int32, S.device).reshape(P, -1, 2)
    K = C.shape[1]
    nc = _counts(n_corres, P, S.device)
    pid = None if pair_ids is None else _cuda(pair_ids, torch.int32, S.device).reshape(P)
    T, fr, st, ct, mk = _ransac_outputs(P, N, S.device, want_corr, want_mask)
    cp = params.to_c()
    # count tensors held in locals: a temporary freed before the launch would
    # hand its (reused) block to the next one
    ns, nt = _counts(n_src, P, S.device), _counts(n_tgt, P, S.device)
    with torch.cuda.device(S.device):
        _lib.call("pcr_ransac_batch", _lib.ptr(S), _lib.ptr(G), P, N, M, _lib.ptr(ns), _lib.ptr(nt),
                  _lib.ptr(C), _lib.ptr(nc), K, _lib.ptr(pid), ctypes.byref(cp), _lib.ptr(T),
                  _lib.ptr(fr), _lib.ptr(st), _lib.ptr(ct), _lib.ptr(mk), _stream(S.device))
    return BatchResult(T, fr[:, 0], fr[:, 1], st, ct, mk)


def register_feature_ransac_batch(src, tgt, src_feat, tgt_feat, params: RansacParams,
                                  n_src=None, n_tgt=None, pair_ids=None, want_corr=True,
                                  want_mask=True):
    """Feature matching -> mutual correspondences -> RANSAC for a batch of pairs."""
    S = _batch3(src, "src")
    G = _batch3(tgt, "tgt", S.device)
    F = _cuda(src_feat, torch.float32, S.device)
    H = _cuda(tgt_feat, torch.float32, S.device)
    if F.dim() == 2:
        F, H = F.unsqueeze(0), H.unsqueeze(0)
    P, N, M, D = S.shape[0], S.shape[1], G.shape[1], F.shape[2]
    if F.shape[:2] != (P, N) or H.shape != (P, M, D):
        raise ValueError("features must be (P,N,D) / (P,M,D) matching the clouds")
    pid = None if pair_ids is None else _cuda(pair_ids, torch.int32, S.device).reshape(P)
    T, fr, st, ct, mk = _ransac_outputs(P, N, S.device, want_corr, want_mask)
    cp = params.to_c()
    ns, nt = _counts(n_src, P, S.device), _counts(n_tgt, P, S.device)
    with torch.cuda.device(S.device):
        _lib.call("pcr_register_feature_ransac", _lib.ptr(S), _lib.ptr(G), _lib.ptr(F),
                  _lib.ptr(H), P, N, M, D, _lib.ptr(ns), _lib.ptr(nt), _lib.ptr(pid), ctypes.byref(cp),
                  _lib.ptr(T), _lib.ptr(fr), _lib.ptr(st), _lib.ptr(ct), _lib.ptr(mk),
                  _stream(S.device))
    return BatchResult(T, fr[:, 0], fr[:, 1], st, ct, mk)


def icp_batch(src, tgt, init, params: IcpParams, n_src=None, n_tgt=None, want_corr=True):
    S = _batch3(src, "src")
    G = _batch3(tgt, "tgt", S.device)
    P, N, M = S.shape[0], S.shape[1], G.shape[1]
    I = _cuda(init, torch.float64, S.device).reshape(P, 16)
    T = torch.empty(P, 4, 4, dtype=torch.float64, device=S.device)
    fr = torch.empty(P, 2, dtype=torch.float64, device=S.device)
    st = torch.empty(P, 2, dtype=torch.int32, device=S.device)
    ct = torch.empty(P, N, dtype=torch.int32, device=S.device) if want_corr else None
    cp = params.to_c()
    ns, nt = _counts(n_src, P, S.device), _counts(n_tgt, P, S.device)
    with torch.cuda.device(S.device):
        _lib.call("pcr_icp_batch", _lib.ptr(S), _lib.ptr(G), P, N, M, _lib.ptr(ns), _lib.ptr(nt),
                  _lib.ptr(I), ctypes.byref(cp), _lib.ptr(T), _lib.ptr(fr), _lib.ptr(st),
                  _lib.ptr(ct), _stream(S.device))
    return BatchResult(T, fr[:, 0], fr[:, 1], st, ct)


def transform_batch(xyz, T, out=None):
    """(P,N,3) f32 points through per-pair T (P,4,4) f64: (float)(R p + t) computed in f64."""
    X = _batch3(xyz, "xyz")
    P, N = X.shape[0], X.shape[1]
    M = _cuda(T, torch.float64, X.device).reshape(P, 16)
    if out is None:
        out = torch.empty_like(X)
    with torch.cuda.device(X.device):
        _lib.call("pcr_transform_batch", _lib.ptr(X), P, N, _lib.ptr(M), _lib.ptr(out),
                  _stream(X.device))
    return out


def radius_nn(tgt, queries, r, n_tgt=None, n_q=None):
    """Radius-limited 1-NN of f64 queries (P,Q,3) among targets (P,M,3):
    (idx (P,Q) int32, -1 if none; d2 (P,Q) f64)."""
    G = _batch3(tgt, "tgt")
    Q = _cuda(queries, torch.float64, G.device)
    if Q.dim() == 2:
        Q = Q.unsqueeze(0)
    P, Nq, M = Q.shape[0], Q.shape[1], G.shape[1]
    idx = torch.empty(P, Nq, dtype=torch.int32, device=G.device)
    d2 = torch.empty(P, Nq, dtype=torch.float64, device=G.device)
    nt, nq = _counts(n_tgt, P, G.device), _counts(n_q, P, G.device)
    with torch.cuda.device(G.device):
        _lib.call("pcr_radius_nn", _lib.ptr(G), P, M, _lib.ptr(nt), _lib.ptr(Q), Nq, _lib.ptr(nq),
                  float(r), _lib.ptr(idx),
                  _lib.ptr(d2), _stream(G.device))
    return idx, d2


# --------------------------------------------------------------------------
# Open3D-shaped façade (o3d.pipelines.registration names)
# --------------------------------------------------------------------------


class PointCloud:
    """Minimal stand-in for o3d.geometry.PointCloud: ``.points`` (N, 3), optional
    ``.normals`` / ``.colors``, and the methods the reference's hot-path callers
    use (voxel_down_sample, transform, paint_uniform_color)."""

    def __init__(self, points=None):
        self.points = np.zeros((0, 3)) if points is None else points
        self.normals = None
        self.colors = None

    def has_normals(self):
        return self.normals is not None and len(self.normals) > 0

    def has_colors(self):
        return self.colors is not None and len(self.colors) > 0

    def paint_uniform_color(self, color):
        self.colors = np.tile(np.asarray(color, np.float64).reshape(1, 3), (len(self.points), 1))
        return self

    def voxel_down_sample(self, voxel_size):
        """o3d PointCloud.voxel_down_sample on the GPU (geometry.voxel_down_sample)."""
        from .geometry import voxel_down_sample
        return voxel_down_sample(self, voxel_size)

    def transform(self, T):
        """In place, like Open3D's Transform: p <- ((T00 x + T01 y) + T02 z) + T03
        per row in f64 (the order every kernel of this library uses), normals
        rotated."""
        T = np.asarray(T, np.float64)
        p = np.asarray(self.points, np.float64).reshape(-1, 3)
        x, y, z = p[:, 0], p[:, 1], p[:, 2]
        self.points = np.stack([((T[r, 0] * x + T[r, 1] * y) + T[r, 2] * z) + T[r, 3]
                                for r in range(3)], axis=1)
        if self.has_normals():
            q = np.asarray(self.normals, np.float64).reshape(-1, 3)
            a, b, c = q[:, 0], q[:, 1], q[:, 2]
            self.normals = np.stack([(T[r, 0] * a + T[r, 1] * b) + T[r, 2] * c for r in range(3)], axis=1)
        return self


class Feature:
    """o3d.pipelines.registration.Feature: ``.data`` is (dim, num) like Open3D."""

    def __init__(self, data=None):
        self.data = np.zeros((0, 0)) if data is None else data

    def dimension(self):
        return int(np.asarray(self.data).shape[0])

    def num(self):
        return int(np.asarray(self.data).shape[1])


class TransformationEstimationPointToPoint:
    def __init__(self, with_scaling=False):
        if with_scaling:
            raise NotImplementedError("with_scaling=True (Sim3 Umeyama) is not on the hot path")
        self.with_scaling = False


class CorrespondenceCheckerBasedOnEdgeLength:
    def __init__(self, similarity_threshold=0.9):
        self.similarity_threshold = float(similarity_threshold)


class CorrespondenceCheckerBasedOnDistance:
    def __init__(self, distance_threshold):
        self.distance_threshold = float(distance_threshold)


class RANSACConvergenceCriteria:
    def __init__(self, max_iteration=100000, confidence=0.999):
        self.max_iteration = int(max_iteration)
        self.confidence = float(confidence)


class ICPConvergenceCriteria:
    def __init__(self, relative_fitness=1e-6, relative_rmse=1e-6, max_iteration=30):
        self.relative_fitness = float(relative_fitness)
        self.relative_rmse = float(relative_rmse)
        self.max_iteration = int(max_iteration)


class RegistrationResult:
    def __init__(self, transformation=None, correspondence_set=None, fitness=0.0,
                 inlier_rmse=0.0):
        self.transformation = np.eye(4) if transformation is None else transformation
        self.correspondence_set = (np.zeros((0, 2), np.int32) if correspondence_set is None
                                   else correspondence_set)
        self.fitness = float(fitness)
        self.inlier_rmse = float(inlier_rmse)

    def __repr__(self):
        return (f"RegistrationResult with fitness={self.fitness:e}, inlier_rmse="
                f"{self.inlier_rmse:e}, and correspondence_set size of "
                f"{len(self.correspondence_set)}")


def _points(pc):
    pts = pc.points if hasattr(pc, "points") else pc
    if isinstance(pts, torch.Tensor):
        return pts.reshape(-1, 3)
    return np.asarray(pts, dtype=np.float64).reshape(-1, 3)


def _feature_rows(f):
    """(num, dim) rows of a feature argument: an Open3D-style Feature (``.data`` is
    (dim, num)) is transposed; a raw (N, D) ndarray or tensor passes through (both
    have a ``.data`` attribute of their own, so the test is on the type)."""
    if isinstance(f, (np.ndarray, torch.Tensor)):
        return f
    if hasattr(f, "data"):
        data = f.data
        return data.t() if isinstance(data, torch.Tensor) else np.asarray(data).T
    return np.asarray(f)


def _ransac_params_from_o3d(max_corr, estimation_method, ransac_n, checkers, criteria, mutual,
                            seed):
    if estimation_method is not None and getattr(estimation_method, "with_scaling", False):
        raise NotImplementedError("with_scaling=True is not supported")
    edge, dist = -1.0, -1.0
    for c in checkers or []:
        if isinstance(c, CorrespondenceCheckerBasedOnEdgeLength):
            edge = c.similarity_threshold
        elif isinstance(c, CorrespondenceCheckerBasedOnDistance):
            dist = c.distance_threshold
        else:
            raise NotImplementedError(f"checker {type(c).__name__} is not supported")
    crit = criteria or RANSACConvergenceCriteria()
    return RansacParams(max_correspondence_distance=float(max_corr), edge_length_ratio=edge,
                        distance_check=dist, confidence=crit.confidence,
                        max_iteration=crit.max_iteration, ransac_n=int(ransac_n),
                        mutual_filter=bool(mutual), seed=int(seed))


def _to_result(br: BatchResult):
    T = br.transformation[0].cpu().numpy()
    return RegistrationResult(T, br.correspondence_set(0), float(br.fitness[0].item()),
                              float(br.inlier_rmse[0].item()))


def registration_ransac_based_on_feature_matching(source, target, source_feature, target_feature,
                                                  mutual_filter, max_correspondence_distance,
                                                  estimation_method=None, ransac_n=3,
                                                  checkers=None, criteria=None, seed=0):
    """Drop-in for o3d.pipelines.registration.registration_ransac_based_on_feature_matching."""
    prm = _ransac_params_from_o3d(max_correspondence_distance, estimation_method, ransac_n,
                                  checkers, criteria, mutual_filter, seed)
    src, tgt = _points(source), _points(target)
    fs, ft = _feature_rows(source_feature), _feature_rows(target_feature)
    br = register_feature_ransac_batch(src, tgt, fs, ft, prm, want_mask=False)
    return _to_result(br)


def registration_ransac_based_on_correspondence(source, target, corres,
                                                max_correspondence_distance,
                                                estimation_method=None, ransac_n=3,
                                                checkers=None, criteria=None, seed=0):
    """Drop-in for o3d.pipelines.registration.registration_ransac_based_on_correspondence."""
    prm = _ransac_params_from_o3d(max_correspondence_distance, estimation_method, ransac_n,
                                  checkers, criteria, False, seed)
    src, tgt = _points(source), _points(target)
    c = np.asarray(corres, dtype=np.int32).reshape(1, -1, 2)
    br = ransac_batch(src, tgt, c, np.array([c.shape[1]], np.int32), prm, want_mask=False)
    return _to_result(br)


def registration_icp(source, target, max_correspondence_distance, init=None,
                     estimation_method=None, criteria=None):
    """Drop-in for o3d.pipelines.registration.registration_icp (point-to-point)."""
    if estimation_method is not None and not isinstance(estimation_method,
                                                        TransformationEstimationPointToPoint):
        raise NotImplementedError("only TransformationEstimationPointToPoint is supported")
    crit = criteria or ICPConvergenceCriteria()
    init = np.eye(4) if init is None else np.asarray(init, dtype=np.float64)
    prm = IcpParams(float(max_correspondence_distance), crit.relative_fitness,
                    crit.relative_rmse, crit.max_iteration)
    br = icp_batch(_points(source), _points(target), init.reshape(1, 4, 4), prm)
    return _to_result(br)


def register(src, tgt, src_feat, tgt_feat, max_correspondence_distance, mutual_filter=True,
             ransac_n=3, edge_length_ratio=0.9, distance_check=None, max_iteration=100000,
             confidence=0.999, seed=0):
    """Rigid registration src -> tgt from per-point features: returns (R (3,3), t (3,)) f64
    numpy arrays with tgt ~ R @ src + t (north-star register(src, tgt) -> (R, t))."""
    prm = RansacParams(max_correspondence_distance, edge_length_ratio, distance_check,
                       confidence, max_iteration, ransac_n, mutual_filter, seed)
    br = register_feature_ransac_batch(src, tgt, src_feat, tgt_feat, prm, want_corr=False,
                                       want_mask=False)
    T = br.transformation[0].cpu().numpy()
    return T[:3, :3].copy(), T[:3, 3].copy()
