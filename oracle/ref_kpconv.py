"""TEST INFRASTRUCTURE ONLY: ctypes access to the reference's own KPConv helpers.

oracle/_ref/libref_kpconv.so is built by oracle/build_ref.sh from the reference
sources in place (c2p-net/ngenet/cpp_wrappers: grid_subsampling.cpp,
neighbors.cpp + vendored nanoflann, cloud.cpp) plus oracle/ref_kpconv.cpp, our
marshalling in place of the CPython wrapper.cpp files.  The functions below
mirror the wrappers' Python signatures and error behaviour
(cpp_subsampling/wrapper.cpp:59-330, cpp_neighbors/wrapper.cpp:63-230):
inputs converted to float32 / int32 C-contiguous, RuntimeError("Error") on an
empty result.  Only tests/, smoke() and bench.py's cpu_baseline leg use it.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_ref", "libref_kpconv.so")
_lib = None


def available():
    return os.path.exists(LIB_PATH)


def _load():
    global _lib
    if _lib is None:
        lib = ctypes.CDLL(LIB_PATH)
        P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        lib.ref_subsample_batch.argtypes = [P, I, P, I, P, I, F, I, P, P, P]
        lib.ref_subsample_batch.restype = I
        lib.ref_batch_neighbors.argtypes = [P, I, P, I, P, P, I, F, P]
        lib.ref_batch_neighbors.restype = I
        lib.ref_free.argtypes = [P]
        _lib = lib
    return _lib


def _arr(x, dt, shape1=None):
    a = np.ascontiguousarray(np.asarray(x), dtype=dt)
    if shape1 is not None and (a.ndim != 2 or a.shape[1] != shape1):
        raise RuntimeError(f"Wrong dimensions : shape is not (N, {shape1})")
    return a


def _take(ptr, count, dt):
    lib = _load()
    addr = ptr.value
    out = np.ctypeslib.as_array(ctypes.cast(addr, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                shape=(max(count, 1),))[:count].copy()
    lib.ref_free(addr)
    return out


def subsample_batch(points, batches, features=None, sampleDl=0.1, max_p=0):
    """cpp_subsampling.subsample_batch (points / features only)."""
    lib = _load()
    pts = _arr(points, np.float32, 3)
    bl = _arr(batches, np.int32).reshape(-1)
    n = pts.shape[0]
    fd = 0
    f = None
    if features is not None:
        f = _arr(features, np.float32)
        if f.ndim == 1:
            f = f.reshape(-1, 1)
        fd = f.shape[1]
    op, ob, of = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    m = lib.ref_subsample_batch(pts.ctypes.data, n, bl.ctypes.data, bl.shape[0],
                                f.ctypes.data if f is not None else None, fd, float(sampleDl),
                                int(max_p), ctypes.byref(op), ctypes.byref(ob),
                                ctypes.byref(of) if f is not None else None)
    s_pts = _take(op, 3 * m, np.float32).reshape(m, 3)
    s_len = _take(ob, bl.shape[0], np.int32)
    s_feat = _take(of, m * fd, np.float32).reshape(m, fd) if f is not None else None
    if m < 1:
        raise RuntimeError("Error")
    return (s_pts, s_len) if f is None else (s_pts, s_len, s_feat)


def batch_query(queries, supports, q_batches, s_batches, radius=0.1):
    """cpp_neighbors.batch_query."""
    lib = _load()
    q = _arr(queries, np.float32, 3)
    s = _arr(supports, np.float32, 3)
    qb = _arr(q_batches, np.int32).reshape(-1)
    sb = _arr(s_batches, np.int32).reshape(-1)
    if qb.shape[0] != sb.shape[0]:
        raise RuntimeError("Wrong number of batch elements: different for queries and supports ")
    out = ctypes.c_void_p()
    mc = lib.ref_batch_neighbors(q.ctypes.data, q.shape[0], s.ctypes.data, s.shape[0],
                                 qb.ctypes.data, sb.ctypes.data, qb.shape[0], float(radius),
                                 ctypes.byref(out))
    res = _take(out, q.shape[0] * mc, np.int32).reshape(q.shape[0], mc)
    if res.size < 1:
        raise RuntimeError("Error")
    return res


def pyramid(points, lengths, normals, architecture, first_subsampling_dl, conv_radius,
            neighborhood_limits):
    """The reference's collate_fn layer loop (c2p-net/ngenet/data/dataloader.py:116-167)
    over the compiled reference helpers, numpy in / numpy out (int64 indices)."""
    pts = np.asarray(points, np.float32)
    nrm = np.asarray(normals, np.float32)
    lens = np.asarray(lengths, np.int32)
    r_normal = first_subsampling_dl * conv_radius
    out = {k: [] for k in ("points", "neighbors", "pools", "upsamples", "stacked_lengths", "normals")}
    layer = 0

    def nb(q, s, qb, sb, r, mx):
        inds = batch_query(q, s, qb, sb, radius=r)
        return inds[:, :mx] if mx > 0 else inds

    for block_i, block in enumerate(architecture):
        if "upsample" in block:
            break
        conv_i = pool_i = up_i = None
        if "strided" in block or "upsample" in architecture[block_i + 1]:
            conv_i = nb(pts, pts, lens, lens, r_normal, neighborhood_limits[layer])
        if "strided" in block:
            voxel_size = 2 * r_normal / conv_radius
            new_pts, new_len, new_nrm = subsample_batch(pts, lens, features=nrm, sampleDl=voxel_size)
            pool_i = nb(new_pts, pts, new_len, lens, r_normal, neighborhood_limits[layer])
            up_i = nb(pts, new_pts, lens, new_len, 2 * r_normal, neighborhood_limits[layer])
        if conv_i is not None:
            out["points"].append(pts)
            out["stacked_lengths"].append(lens)
            out["normals"].append(nrm)
            out["neighbors"].append(conv_i.astype(np.int64))
        if pool_i is not None:
            out["pools"].append(pool_i.astype(np.int64))
            out["upsamples"].append(up_i.astype(np.int64))
            pts, lens, nrm = new_pts, new_len, new_nrm
            r_normal *= 2
            layer += 1
    return out
