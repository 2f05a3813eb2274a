"""numpy front-end of the CPU oracle (liboracle.so built from pcr_oracle.c).

TEST INFRASTRUCTURE ONLY -- used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker.  Nothing in the product imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def nnd_forward(xyz1, xyz2):
    """Restatement of my_lib.cpp:28-60: returns dist1, dist2, idx1, idx2."""
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    b, n, m = xyz1.shape[0], xyz1.shape[1], xyz2.shape[1]
    d1 = np.zeros((b, n), np.float32)
    d2 = np.zeros((b, m), np.float32)
    i1 = np.zeros((b, n), np.int32)
    i2 = np.zeros((b, m), np.int32)
    lib().oracle_nnd_forward(_p(xyz1), _p(xyz2), b, n, m, _p(d1), _p(d2), _p(i1), _p(i2))
    return d1, d2, i1, i2


def nnd_backward(xyz1, xyz2, gd1, gd2, idx1, idx2):
    """Restatement of my_lib.cpp:64-133: returns gradxyz1, gradxyz2."""
    xyz1, xyz2, gd1, gd2 = _f32(xyz1), _f32(xyz2), _f32(gd1), _f32(gd2)
    idx1, idx2 = _i32(idx1), _i32(idx2)
    b, n, m = xyz1.shape[0], xyz1.shape[1], xyz2.shape[1]
    g1 = np.zeros((b, n, 3), np.float32)
    g2 = np.zeros((b, m, 3), np.float32)
    lib().oracle_nnd_backward(_p(xyz1), _p(xyz2), _p(gd1), _p(gd2), _p(idx1), _p(idx2),
                              b, n, m, _p(g1), _p(g2))
    return g1, g2


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _setup_sigs():
    L = lib()
    c = ctypes
    L.oracle_det_log.restype = c.c_double
    L.oracle_det_log.argtypes = [c.c_double]
    L.oracle_est_k.restype = c.c_double
    L.oracle_est_k.argtypes = [c.c_double, c.c_int, c.c_double]
    L.oracle_radius_thr.restype = c.c_double
    L.oracle_radius_thr.argtypes = [c.c_double]
    L.oracle_procrustes_batch.argtypes = [c.c_void_p] * 3 + [c.c_int, c.c_int, c.c_int, c.c_double, c.c_void_p]
    L.oracle_ransac.restype = c.c_int
    L.oracle_ransac.argtypes = ([c.c_void_p, c.c_int, c.c_void_p, c.c_int, c.c_void_p, c.c_int,
                                 c.c_double, c.c_int, c.c_double, c.c_double, c.c_int, c.c_double,
                                 c.c_uint64, c.c_uint32, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p])
    L.oracle_icp.restype = c.c_int
    L.oracle_icp.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_int, c.c_void_p, c.c_double,
                             c.c_int, c.c_double, c.c_double, c.c_void_p, c.c_void_p, c.c_void_p]
    L.oracle_icp_trace.restype = c.c_int
    L.oracle_icp_trace.argtypes = L.oracle_icp.argtypes + [c.c_void_p, c.c_void_p]
    L.oracle_radius_nn.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_int, c.c_double, c.c_int,
                                   c.c_void_p, c.c_void_p]
    L.oracle_featnn.argtypes = [c.c_void_p, c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_void_p]
    L.oracle_corres.restype = c.c_int
    L.oracle_corres.argtypes = [c.c_void_p, c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_void_p]
    L.oracle_philox.argtypes = [c.c_uint64, c.c_uint32, c.c_uint32, c.c_uint32, c.c_void_p]
    L.oracle_horn_rotation.argtypes = [c.c_void_p, c.c_void_p]
    L.oracle_voxel_down_sample.restype = c.c_int
    L.oracle_voxel3i_map_order.restype = None
    L.oracle_voxel3i_map_order.argtypes = [c.c_void_p, c.c_int, c.c_void_p]
    L.oracle_voxel_down_sample.argtypes = [c.c_void_p, c.c_int, c.c_double, c.c_void_p, c.c_void_p,
                                           c.c_void_p, c.c_void_p, c.c_void_p]
    L.oracle_xs_sum.restype = c.c_double
    L.oracle_xs_sum.argtypes = [c.c_void_p, c.c_int]
    L.oracle_lrf_count.restype = c.c_int
    L.oracle_lrf_count.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_double]
    L.oracle_lrf.restype = c.c_int
    L.oracle_lrf.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_double, c.c_int, c.c_void_p,
                             c.c_void_p, c.c_void_p]
    return L


_sigs = None


def L():
    global _sigs
    if _sigs is None:
        _sigs = _setup_sigs()
    return _sigs


def det_log(x):
    return L().oracle_det_log(float(x))


def est_k(w, n, conf):
    return L().oracle_est_k(float(w), int(n), float(conf))


def philox(seed, pair, itr, block=0):
    out = np.zeros(4, np.uint32)
    L().oracle_philox(seed, pair, itr, block, _p(out))
    return out


def voxel_down_sample(points, voxel_size, normals=None, colors=None):
    """Open3D PointCloud::VoxelDownSample restated (oracle/voxel_oracle.cpp):
    (points, normals or None, colors or None) in the map's iteration order."""
    p = _f64(points).reshape(-1, 3)
    n = p.shape[0]
    nr = None if normals is None else _f64(normals).reshape(-1, 3)
    cl = None if colors is None else _f64(colors).reshape(-1, 3)
    op = np.zeros((max(n, 1), 3))
    on = np.zeros((max(n, 1), 3)) if nr is not None else None
    oc = np.zeros((max(n, 1), 3)) if cl is not None else None
    k = L().oracle_voxel_down_sample(_p(p), n, float(voxel_size), _p(nr) if nr is not None else None,
                                     _p(cl) if cl is not None else None, _p(op),
                                     _p(on) if on is not None else None, _p(oc) if oc is not None else None)
    if k < 0:
        raise ValueError("voxel_down_sample: voxel_size <= 0 or too small")
    return op[:k].copy(), (on[:k].copy() if on is not None else None), (oc[:k].copy() if oc is not None else None)


def voxel3i_map_order(xyz):
    """iteration order of std::unordered_map<Vector3i, ., hash_eigen> for the keys
    (K, 3) int32 inserted in row order (the real container)"""
    xyz = _i32(xyz).reshape(-1, 3)
    out = np.zeros(xyz.shape[0], np.int32)
    L().oracle_voxel3i_map_order(_p(xyz), xyz.shape[0], _p(out))
    return out


def xs_sum(v):
    """Exact fixed-point sum of f64 terms rounded once (the ICP Umeyama sums)."""
    v = _f64(v).reshape(-1)
    return float(L().oracle_xs_sum(_p(v), v.shape[0]))


def horn_rotation(S):
    S = _f64(S).reshape(9)
    R = np.zeros(9, np.float64)
    L().oracle_horn_rotation(_p(S), _p(R))
    return R.reshape(3, 3)


def procrustes_batch(src, tgt, w, absw, eps):
    """(B,N,3),(B,N,3),(B,N) -> T (B,3,4) f64 (weighted_icp: absw=0,eps=1e-8;
    rigid_fit: absw=1, eps=1e-4)."""
    src, tgt, w = _f32(src), _f32(tgt), _f32(w)
    b, n = src.shape[0], src.shape[1]
    T = np.zeros((b, 3, 4), np.float64)
    L().oracle_procrustes_batch(_p(src), _p(tgt), _p(w), b, n, int(absw), float(eps), _p(T))
    return T


def featnn(F, G):
    F, G = _f32(F), _f32(G)
    nn = np.zeros(F.shape[0], np.int32)
    L().oracle_featnn(_p(F), _p(G), F.shape[0], G.shape[0], F.shape[1], _p(nn))
    return nn


def vote(source, target, source_feats, target_feats, voxel_size):
    """c2p-net/ngenet/models/vote.py:12-37 restated: the three nearest-target
    searches by the exact 1-NN (featnn; get_coor_points :6-9), then the f32
    distance tests and the in-place h-row replacement.  Returns
    [source, target, fs_h, ft_h] like the reference (fs_h / ft_h are copies
    here) and the replaced mask."""
    tgt = np.asarray(target, np.float32)
    fs = [np.array(f, np.float32) for f in source_feats]
    ft = [np.array(f, np.float32) for f in target_feats]
    i1, i2, i3 = (featnn(a, b) for a, b in zip(fs, ft))
    y1, y2, y3 = tgt[i1], tgt[i2], tgt[i3]

    def dist(a, b):
        d = a - b
        return np.sqrt((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2])

    thr = np.float32(voxel_size * 2)
    sel_h = (dist(y1, y2) < thr) | (dist(y1, y3) < thr)
    sel_m = dist(y2, y3) < thr
    rep = ~sel_h & sel_m
    fs[0][rep] = fs[1][rep]
    ft[0][i2[rep]] = ft[1][i2[rep]]
    return [source, target, fs[0], ft[0]], rep


def corres(nn12, nn21, mutual=True, ransac_n=3):
    nn12, nn21 = _i32(nn12), _i32(nn21)
    out = np.zeros((nn12.shape[0], 2), np.int32)
    k = L().oracle_corres(_p(nn12), _p(nn21), nn12.shape[0], int(mutual), int(ransac_n), _p(out))
    return out[:k].copy()


def radius_nn(tgt, queries, r, use_grid=True):
    tgt, q = _f64(tgt), _f64(queries)
    idx = np.zeros(q.shape[0], np.int32)
    d2 = np.zeros(q.shape[0], np.float64)
    L().oracle_radius_nn(_p(tgt), tgt.shape[0], _p(q), q.shape[0], float(r), int(use_grid),
                         _p(idx), _p(d2))
    return idx, d2


def ransac(src, tgt, corr, max_corr_dist, ransac_n=3, edge_ratio=0.9, dist_check=None,
           max_iteration=100000, confidence=0.999, seed=0, pair_id=0):
    """Returns dict(T (4,4), fitness, inlier_rmse, correspondence_set (K,2), iters,
    validated, best_itr, found)."""
    src, tgt, corr = _f32(src), _f32(tgt), _i32(corr).reshape(-1, 2)
    if dist_check is None:
        dist_check = max_corr_dist
    T = np.zeros(16, np.float64)
    fr = np.zeros(2, np.float64)
    co = np.zeros((src.shape[0], 2), np.int32)
    st = np.zeros(4, np.int32)
    nc = L().oracle_ransac(_p(src), src.shape[0], _p(tgt), tgt.shape[0], _p(corr), corr.shape[0],
                           float(max_corr_dist), int(ransac_n), float(edge_ratio), float(dist_check),
                           int(max_iteration), float(confidence), int(seed), int(pair_id),
                           _p(T), _p(fr), _p(co), _p(st))
    return dict(T=T.reshape(4, 4), fitness=fr[0], inlier_rmse=fr[1],
                correspondence_set=co[:nc].copy(), iters=int(st[0]), validated=int(st[1]),
                best_itr=int(st[2]), found=int(st[3]))


def icp(src, tgt, max_corr_dist, init=None, max_iteration=30, relative_fitness=1e-6,
        relative_rmse=1e-6):
    src, tgt = _f32(src), _f32(tgt)
    init = np.eye(4) if init is None else init
    init = _f64(init).reshape(16)
    T = np.zeros(16, np.float64)
    fr = np.zeros(2, np.float64)
    it = np.zeros(1, np.int32)
    nc = L().oracle_icp(_p(src), src.shape[0], _p(tgt), tgt.shape[0], _p(init),
                        float(max_corr_dist), int(max_iteration), float(relative_fitness),
                        float(relative_rmse), _p(T), _p(fr), _p(it))
    return dict(T=T.reshape(4, 4), fitness=fr[0], inlier_rmse=fr[1], n_corr=nc, iters=int(it[0]))


def icp_trace(src, tgt, max_corr_dist, init=None, max_iteration=30, relative_fitness=1e-6,
              relative_rmse=1e-6):
    """oracle.icp plus, per iteration, the f64 working copy the Umeyama step saw
    (iters, n, 3) and its correspondences (iters, n) (-1 = no target within d)."""
    src, tgt = _f32(src), _f32(tgt)
    n = src.shape[0]
    init = _f64(np.eye(4) if init is None else init).reshape(16)
    T = np.zeros(16, np.float64)
    fr = np.zeros(2, np.float64)
    it = np.zeros(1, np.int32)
    P = np.zeros((max_iteration, n, 3), np.float64)
    cj = np.full((max_iteration, n), -1, np.int32)
    nc = L().oracle_icp_trace(_p(src), n, _p(tgt), tgt.shape[0], _p(init), float(max_corr_dist),
                              int(max_iteration), float(relative_fitness), float(relative_rmse),
                              _p(T), _p(fr), _p(it), _p(P), _p(cj))
    k = int(it[0])
    return dict(T=T.reshape(4, 4), fitness=fr[0], inlier_rmse=fr[1], n_corr=nc, iters=k,
                P=P[:k].copy(), cj=cj[:k].copy())


def ransac_sample(seed, pair_id, itr, K, ransac_n=3):
    """The correspondence indices hypothesis `itr` draws (sample_indices in
    pcr_oracle.c: Philox4x32-10 words scaled to [0, K))."""
    out = []
    for j in range(ransac_n):
        if j % 4 == 0:
            w = philox(seed, pair_id, itr, j >> 2)
        out.append(int((int(w[j & 3]) * int(K)) >> 32))
    return np.array(out, np.int32)


def lrf_count(pts, q, kernel):
    """Radius-neighbour count of lrf.get (dip/lrf.py:21), incl. the first hit."""
    pts, q = _f64(pts), _f64(q)
    return int(L().oracle_lrf_count(_p(pts), len(pts), _p(q), float(kernel)))


def lrf(pts, q, kernel, patch_size, inds):
    """dip/lrf.py:19-78 with the caller's choice indices: (k, patch (ps,3), T (4,4))."""
    pts, q = _f64(pts), _f64(q)
    inds = _i32(inds)
    patch = np.zeros((patch_size, 3), np.float64)
    T = np.zeros(16, np.float64)
    k = L().oracle_lrf(_p(pts), len(pts), _p(q), float(kernel), int(patch_size), _p(inds),
                       _p(patch), _p(T))
    return int(k), patch, T.reshape(4, 4)


# ---------------------------------------------------------------------------
# a10: NDP per-level warp, numpy f64 restatement of
# c2p-net/deformationpyramid/model/nets.py NDPLayer.forward (:111-140),
# posenc (:164-177), get_Rotation axis_angle (:144-161) -> rigid_body.exp_so3 /
# skew (:89-95, :113-119), MLP (:295-304), Deformation_Pyramid.warp (:36-48).
# Floating point: the GPU (f32) is held to 1e-5 of it (north_star tolerance).
# ---------------------------------------------------------------------------
def ndp_level(p, x, m, k0):
    """One NDPLayer (SE3, axis_angle). p: dict of the layer's state_dict arrays."""
    x = np.asarray(x, np.float64)
    w = float(2.0 ** (m + k0))
    pe = np.concatenate([np.sin(x[:, 0:1] * w), np.cos(x[:, 0:1] * w),
                         np.sin(x[:, 1:2] * w), np.cos(x[:, 1:2] * w),
                         np.sin(x[:, 2:3] * w), np.cos(x[:, 2:3] * w)], axis=1)
    f = lambda k: np.asarray(p[k], np.float64)  # noqa: E731
    h = np.maximum(pe @ f("input.0.weight").T + f("input.0.bias"), 0.0)
    i = 0
    while f"mlp.pts_linears.{i}.weight" in p:
        h = np.maximum(h @ f(f"mlp.pts_linears.{i}.weight").T + f(f"mlp.pts_linears.{i}.bias"), 0.0)
        i += 1
    t = 0.001 * (h @ f("trn_branch.weight").T + f("trn_branch.bias"))
    r = 0.001 * (h @ f("rot_brach.weight").T + f("rot_brach.bias"))
    th = np.linalg.norm(r, axis=-1, keepdims=True)
    wv = r / th
    z = np.zeros(len(x))
    K = np.stack([z, -wv[:, 2], wv[:, 1], wv[:, 2], z, -wv[:, 0], -wv[:, 1], wv[:, 0], z],
                 -1).reshape(-1, 3, 3)
    R = np.eye(3)[None] + np.sin(th)[..., None] * K + (1 - np.cos(th))[..., None] * (K @ K)
    xn = (R @ x[..., None])[..., 0] + t
    nr = None
    if "nr_branch.weight" in p:
        s = 1.0 / (1.0 + np.exp(-(0.001 * (h @ f("nr_branch.weight").T + f("nr_branch.bias")))))
        xn = x + s * (xn - x)
        nr = s[:, 0]
    return xn, nr


def ndp_warp(levels, x, k0=-8, max_level=None, min_level=0):
    """Deformation_Pyramid.warp: levels[i] is level i's state dict (m = i + 1)."""
    if max_level is None:
        max_level = len(levels) - 1
    data = {}
    for i in range(min_level, max_level + 1):
        x, nr = ndp_level(levels[i], x, i + 1, k0)
        data[i] = (x, nr)
    return x, data


# ---------------------------------------------------------------------------
# f2: KPConv grid subsampling / radius neighbours (ngenet/cpp_wrappers)
# ---------------------------------------------------------------------------

def _size_t(f):
    """(size_t)f for float32 f as g++ emits it on x86-64: below 2^63 through the
    signed conversion, so -1.0f -> 2^64 - 1 (cvttss2si)."""
    f = np.asarray(f, np.float32)
    return f.astype(np.float64).astype(np.int64).view(np.uint64)


def voxel_keys(points, dl):
    """Per-point mapIdx of one cloud, grid_subsampling.cpp:17-54, in float32:
    origin = floor(min * (1/dl)) * dl, iX = (size_t)floor((x - origin.x) / dl),
    mapIdx = iX + NX*iY + NX*NY*iZ in size_t (wrapping) arithmetic."""
    p = np.asarray(points, np.float32).reshape(-1, 3)
    dl = np.float32(dl)
    inv = np.float32(1.0) / dl
    mn, mx = p.min(0), p.max(0)  # cloud.cpp:27-68 (finite inputs)
    org = (np.floor(mn * inv) * dl).astype(np.float32)
    nx = _size_t(np.floor((mx[0] - org[0]) / dl)) + np.uint64(1)
    ny = _size_t(np.floor((mx[1] - org[1]) / dl)) + np.uint64(1)
    i = _size_t(np.floor((p - org) / dl))
    with np.errstate(over="ignore"):
        return (i[:, 0] + nx * i[:, 1]) + (nx * ny) * i[:, 2]


def grid_subsample(points, batches, dl, features=None, max_p=0, order=None):
    """batch_grid_subsampling (grid_subsampling.cpp:109-211) restated with numpy.

    Voxel sums are float32 additions in input order (np.add.at is sequential,
    SampledData::update_* :41-79), barycentre = sum * float32(1.0 / count),
    features f / float32(count) (:86-95).  The emission order of the reference
    is the iteration order of its unordered_map; `order(keys)` must return it
    for the distinct keys given in first-occurrence order (e.g. the product's
    pcr_voxel_map_order, itself checked against the compiled reference);
    without it voxels come out in first-occurrence order."""
    p = np.asarray(points, np.float32).reshape(-1, 3)
    f = None if features is None else np.asarray(features, np.float32).reshape(p.shape[0], -1)
    bl = np.asarray(batches, np.int64).reshape(-1)
    cap = p.shape[0] if max_p < 1 else int(max_p)
    out_p, out_f, out_len = [], [], []
    o = 0
    for L in bl:
        bp = p[o:o + L]
        if L == 0:
            out_len.append(0)
            continue
        keys = voxel_keys(bp, dl)
        uk, first, inv = np.unique(keys, return_index=True, return_inverse=True)
        rank = np.argsort(first, kind="stable")           # voxel ids in first-occurrence order
        vox_of_rank = rank
        sums = np.zeros((len(uk), 3), np.float32)
        np.add.at(sums, inv.reshape(-1), bp)
        cnt = np.bincount(inv.reshape(-1), minlength=len(uk))
        seq = np.arange(len(uk)) if order is None else np.asarray(order(uk[vox_of_rank]))
        sel = vox_of_rank[seq][:cap]
        scale = (1.0 / cnt[sel].astype(np.float64)).astype(np.float32)
        out_p.append(sums[sel] * scale[:, None])
        if f is not None:
            fs = np.zeros((len(uk), f.shape[1]), np.float32)
            np.add.at(fs, inv.reshape(-1), f[o:o + L])
            out_f.append(fs[sel] / cnt[sel].astype(np.float32)[:, None])
        out_len.append(len(sel))
        o += L
    P = np.concatenate(out_p) if out_p else np.zeros((0, 3), np.float32)
    res = (P, np.asarray(out_len, np.int32))
    if f is not None:
        res = res + (np.concatenate(out_f) if out_f else np.zeros((0, f.shape[1]), np.float32),)
    return res


def radius_neighbors(queries, supports, q_batches, s_batches, radius):
    """batch_nanoflann_neighbors (neighbors.cpp:211-332) restated brute force:
    per query, the supports of its batch with float32 ((dx*dx + dy*dy) + dz*dz)
    < radius*radius (L2_Simple_Adaptor::evalMetric, RadiusResultSet::addPoint),
    ascending distance, equal distances by index, padded with len(supports).
    Returns (rows (nq, max_count) int32, distances as a list of arrays).
    Not restated: the reference's order among EQUAL distances (nanoflann's
    leaf-visit order permuted by std::sort, neighbors.cpp:298 via
    nanoflann.hpp radiusSearch) -- tie-bearing cases are checked against the
    compiled reference (oracle/_ref/libref_kpconv.so) instead."""
    q = np.asarray(queries, np.float32).reshape(-1, 3)
    s = np.asarray(supports, np.float32).reshape(-1, 3)
    qb = np.asarray(q_batches, np.int64)
    sb = np.asarray(s_batches, np.int64)
    r2 = np.float32(radius) * np.float32(radius)
    rows, dists = [], []
    qo = so = 0
    for b in range(len(qb)):
        S = s[so:so + sb[b]]
        for i in range(qo, qo + qb[b]):
            d = q[i] - S
            dd = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
            j = np.nonzero(dd < r2)[0]
            o = np.lexsort((j, dd[j]))
            rows.append(j[o] + so)
            dists.append(dd[j][o])
        qo += qb[b]
        so += sb[b]
    mc = max((len(r) for r in rows), default=0)
    out = np.full((len(rows), mc), s.shape[0], np.int32)
    for i, r in enumerate(rows):
        out[i, :len(r)] = r
    return out, dists


# --------------------------------------------------------------------------
# f1: normals + FPFH (fpfh_oracle.c; Open3D restated, parity vs Open3D unpinned)
# --------------------------------------------------------------------------

def _fpfh_sigs():
    Lb = lib()
    c = ctypes
    for f in ("oracle_det_acos", "oracle_det_cos"):
        getattr(Lb, f).restype = c.c_double
        getattr(Lb, f).argtypes = [c.c_double]
    Lb.oracle_det_atan2.restype = c.c_double
    Lb.oracle_det_atan2.argtypes = [c.c_double, c.c_double]
    Lb.oracle_hybrid_search.argtypes = [c.c_void_p, c.c_int, c.c_double, c.c_int, c.c_void_p,
                                        c.c_void_p, c.c_void_p]
    Lb.oracle_estimate_normals.argtypes = [c.c_void_p, c.c_int, c.c_double, c.c_int, c.c_void_p,
                                           c.c_void_p]
    Lb.oracle_fpfh.argtypes = [c.c_void_p, c.c_void_p, c.c_int, c.c_double, c.c_int, c.c_void_p,
                               c.c_void_p]
    Lb.oracle_fast_eigen3x3.argtypes = [c.c_void_p, c.c_void_p]
    Lb.oracle_pair_features.argtypes = [c.c_void_p] * 5
    return Lb


_fs = None


def FL():
    global _fs
    if _fs is None:
        _fs = _fpfh_sigs()
    return _fs


def det_atan2(y, x):
    return FL().oracle_det_atan2(float(y), float(x))


def det_acos(x):
    return FL().oracle_det_acos(float(x))


def det_cos(x):
    return FL().oracle_det_cos(float(x))


def hybrid_search(pts, radius, max_nn):
    """KDTreeFlann::SearchHybrid(points[i], radius, max_nn) for every point:
    (idx (n,K) int32 -1 padded, d2 (n,K) f64, counts (n,))."""
    p = _f32(pts).reshape(-1, 3)
    n = p.shape[0]
    idx = np.zeros((n, max_nn), np.int32)
    d2 = np.zeros((n, max_nn), np.float64)
    cnt = np.zeros(n, np.int32)
    FL().oracle_hybrid_search(_p(p), n, float(radius), int(max_nn), _p(idx), _p(d2), _p(cnt))
    return idx, d2, cnt


def estimate_normals(pts, radius, max_nn, prior=None):
    p = _f32(pts).reshape(-1, 3)
    out = np.zeros((p.shape[0], 3), np.float64)
    pr = None if prior is None else _f64(prior).reshape(-1, 3)
    FL().oracle_estimate_normals(_p(p), p.shape[0], float(radius), int(max_nn),
                                 None if pr is None else _p(pr), _p(out))
    return out


def fpfh(pts, normals, radius, max_nn):
    """(spfh (n,33), fpfh (n,33)) f64 (Open3D Feature::data_ transposed)."""
    p = _f32(pts).reshape(-1, 3)
    nm = _f64(normals).reshape(-1, 3)
    sp = np.zeros((p.shape[0], 33), np.float64)
    fp = np.zeros((p.shape[0], 33), np.float64)
    FL().oracle_fpfh(_p(p), _p(nm), p.shape[0], float(radius), int(max_nn), _p(sp), _p(fp))
    return sp, fp


def fast_eigen3x3(C):
    C = _f64(C).reshape(9)
    v = np.zeros(3, np.float64)
    FL().oracle_fast_eigen3x3(_p(C), _p(v))
    return v


def pair_features(p1, n1, p2, n2):
    f = np.zeros(4, np.float64)
    FL().oracle_pair_features(_p(_f64(p1)), _p(_f64(n1)), _p(_f64(p2)), _p(_f64(n2)), _p(f))
    return f
