"""f2: KPConv input pyramid helpers on the GPU (drop-in for ngenet's cpp_wrappers).

Mirrors of the reference's Python-facing functions:

* ``subsample_batch``  -- cpp_subsampling.subsample_batch
  (c2p-net/ngenet/cpp_wrappers/cpp_subsampling/wrapper.cpp:59-330)
* ``batch_query``      -- cpp_neighbors.batch_query
  (cpp_neighbors/wrapper.cpp:63-230)
* ``batch_grid_subsampling`` / ``batch_neighbors`` -- the dataloader wrappers
  (c2p-net/ngenet/data/dataloader.py:12-66), returning torch tensors.

Same argument names, defaults and results (subsampled points and features
bit-identical and in the same order; neighbour rows identical, including the
reference's order among exactly equal distances, which the library replays on
the host for the rows that hold them, see DESIGN.md "f2"), RuntimeError("Error") on an
empty result like the wrappers.  The work runs in libpcr (pcr_grid_subsample,
pcr_radius_count / pcr_radius_neighbors); there is no CPU path.  numpy / CPU
inputs give numpy outputs (as the reference); CUDA tensors stay on the device.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib


def _device(*xs):
    for x in xs:
        if isinstance(x, torch.Tensor) and x.is_cuda:
            return x.device, True
    return torch.device("cuda", torch.cuda.current_device()), False


def _points(x, dev, name, ncol=3):
    t = torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x)
    t = t.to(device=dev, dtype=torch.float32).contiguous()
    if ncol is not None and (t.dim() != 2 or t.shape[1] != ncol):
        raise RuntimeError(f"Wrong dimensions : {name}.shape is not (N, {ncol})")
    return t


def _lengths(x, name):
    a = x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)
    a = np.ascontiguousarray(a, dtype=np.int32)
    if a.ndim != 1:
        raise RuntimeError(f"Wrong dimensions : {name}.shape is not (B,) ")
    return a


def _out(t, on_device):
    return t if on_device else t.cpu().numpy()


def subsample_batch(points, batches, features=None, classes=None, sampleDl=0.1,
                    method="barycenters", max_p=0, verbose=0):
    """Barycentric voxel-grid subsampling of a stack of clouds.

    Returns (s_points (M,3) f32, s_len (B,) int32[, s_features (M,d) f32])."""
    if method not in ("barycenters", "voxelcenters"):
        raise RuntimeError('Error parsing method. Valid method names are "barycenters" and '
                           '"voxelcenters" ')
    if classes is not None:
        # the label vote (grid_subsampling.cpp:97-102) is unused by ngenet's callers
        raise NotImplementedError("subsample_batch: classes are not supported")
    dev, on_dev = _device(points, features)
    pts = _points(points, dev, "points")
    bl = _lengths(batches, "batches")
    n = pts.shape[0]
    feat, fdim = None, 0
    if features is not None:
        feat = _points(features, dev, "features", None)
        if feat.dim() == 1:
            feat = feat.reshape(-1, 1)
        if feat.dim() != 2 or feat.shape[0] != n:
            raise RuntimeError("Wrong dimensions : features.shape is not (N, d)")
        fdim = feat.shape[1]
    out_p = torch.empty((max(n, 1), 3), dtype=torch.float32, device=dev)
    out_f = torch.empty((max(n, 1), max(fdim, 1)), dtype=torch.float32, device=dev) if feat is not None else None
    out_len = np.zeros(bl.shape[0], np.int32)
    total = ctypes.c_int32(0)
    with torch.cuda.device(dev):
        _lib.call("pcr_grid_subsample", _lib.ptr(pts), n, bl.ctypes.data, bl.shape[0],
                  _lib.ptr(feat), fdim, float(sampleDl), int(max_p), _lib.ptr(out_p),
                  _lib.ptr(out_f), out_len.ctypes.data, ctypes.byref(total),
                  _lib.stream_handle(dev))
    m = total.value
    if m < 1:
        raise RuntimeError("Error")
    s_len = torch.from_numpy(out_len).to(dev) if on_dev else out_len
    res = (_out(out_p[:m], on_dev), s_len)
    if feat is not None:
        res = res + (_out(out_f[:m, :fdim], on_dev),)
    return res


def _neighbors(queries, supports, q_batches, s_batches, radius, max_nn):
    dev, on_dev = _device(queries, supports)
    q = _points(queries, dev, "query")
    s = _points(supports, dev, "support")
    qb = _lengths(q_batches, "queries_batches")
    sb = _lengths(s_batches, "supports_batches")
    if qb.shape[0] != sb.shape[0]:
        raise RuntimeError("Wrong number of batch elements: different for queries and supports ")
    nq, ns = q.shape[0], s.shape[0]
    mc = ctypes.c_int32(0)
    stream = _lib.stream_handle(dev)
    with torch.cuda.device(dev):
        _lib.call("pcr_radius_count", _lib.ptr(q), nq, _lib.ptr(s), ns, qb.ctypes.data,
                  sb.ctypes.data, qb.shape[0], float(radius), None, ctypes.byref(mc), stream)
        width = mc.value if max_nn <= 0 else min(mc.value, int(max_nn))
        out = torch.empty((nq, width), dtype=torch.int32, device=dev)
        if nq * width > 0:
            _lib.call("pcr_radius_neighbors", _lib.ptr(q), nq, _lib.ptr(s), ns, qb.ctypes.data,
                      sb.ctypes.data, qb.shape[0], float(radius), width, _lib.ptr(out), None,
                      stream)
    return out, mc.value, on_dev


def batch_query(queries, supports, q_batches, s_batches, radius=0.1):
    """Radius neighbours of every query among the supports of its batch:
    (Nq, max_count) int32 rows by ascending distance, padded with len(supports)."""
    out, mc, on_dev = _neighbors(queries, supports, q_batches, s_batches, radius, 0)
    if out.numel() < 1:
        raise RuntimeError("Error")
    return _out(out, on_dev)


def batch_neighbors(batch_queries, batch_supports, q_batches, s_batches, radius, max_nn):
    """dataloader.py:12-25: batch_query truncated to max_nn columns (if > 0), as a
    torch tensor (on the GPU when the inputs are CUDA tensors)."""
    out, mc, on_dev = _neighbors(batch_queries, batch_supports, q_batches, s_batches, radius,
                                 max_nn)
    if mc * out.shape[0] < 1:
        raise RuntimeError("Error")
    return out if on_dev else out.cpu()


def batch_grid_subsampling(points, batches_len, features=None, labels=None, sampleDl=0.1,
                           max_p=0, verbose=0, random_grid_orient=True):
    """dataloader.py:28-66 (points / features) returning torch tensors."""
    if labels is not None:
        raise NotImplementedError("batch_grid_subsampling: labels are not supported")
    res = subsample_batch(points, batches_len, features=features, sampleDl=sampleDl,
                          max_p=max_p, verbose=verbose)
    return tuple(r if isinstance(r, torch.Tensor) else torch.from_numpy(r) for r in res)


def collate_fn(list_data, config, neighborhood_limits, device=None):
    """dataloader.py:69-182 (collate_fn): stacks the items' clouds (src, tgt per
    item) and builds the KPConv input pyramid -- conv neighbours, strided grid
    subsampling with normals, pooling and upsampling neighbours per layer --
    with every neighbour search and subsampling in libpcr.  Arrays stay on the
    GPU between layers; the returned dict has the reference's keys and, as the
    reference, CPU tensors unless `device` names a CUDA device."""
    pts_l, raw_l, feats_l, norm_l, lens, transf_l, coors_l = [], [], [], [], [], [], []
    for item in list_data:
        pts_l += [item["src_points"], item["tgt_points"]]
        raw_l += [item["src_points_raw"], item["tgt_points_raw"]]
        feats_l += [item["src_feats"], item["tgt_feats"]]
        norm_l += [item["src_normals"], item["tgt_normals"]]
        lens += [len(item["src_points"]), len(item["tgt_feats"])]  # (:98-99, as the reference)
        transf_l.append(item["transf"])
        coors_l.append(torch.from_numpy(np.asarray(item["coors"])).long())
    dev = torch.device("cuda", torch.cuda.current_device())
    cat = lambda xs: torch.from_numpy(np.concatenate(xs, axis=0).astype(np.float32))  # noqa: E731
    points = cat(pts_l).to(dev)
    normals = cat(norm_l).to(dev)
    lengths = np.asarray(lens, np.int32)
    stack = pyramid(points, lengths, normals, config.architecture, config.first_subsampling_dl,
                    config.conv_radius, neighborhood_limits)
    out_dev = torch.device(device) if device is not None else torch.device("cpu")
    mv = lambda t: t.to(out_dev)  # noqa: E731
    return {
        "points": [mv(t) for t in stack["points"]],
        "neighbors": [mv(t) for t in stack["neighbors"]],
        "pools": [mv(t) for t in stack["pools"]],
        "upsamples": [mv(t) for t in stack["upsamples"]],
        "stacked_lengths": [mv(t) for t in stack["stacked_lengths"]],
        "feats": mv(cat(feats_l)),
        "normals": [mv(t) for t in stack["normals"]],
        "coors": coors_l,
        "transf": mv(torch.from_numpy(np.array(transf_l).astype(np.float32))),
        "batched_points_raw": mv(cat(raw_l)),
    }


def pyramid(points, lengths, normals, architecture, first_subsampling_dl, conv_radius,
            neighborhood_limits):
    """The layer loop of collate_fn (dataloader.py:116-167) on device tensors:
    points (N,3) f32 CUDA, lengths (B,) host int32, normals (N,3) f32 CUDA.
    Returns lists of CUDA tensors (neighbour indices int64, as .long() there)."""
    lengths = torch.as_tensor(np.asarray(lengths, np.int32))
    r_normal = first_subsampling_dl * conv_radius
    out = {"points": [], "neighbors": [], "pools": [], "upsamples": [], "stacked_lengths": [],
           "normals": []}
    layer = 0
    for block_i, block in enumerate(architecture):
        if "upsample" in block:
            break
        conv_i = pool_i = up_i = None
        if "strided" in block or "upsample" in architecture[block_i + 1]:
            conv_i = batch_neighbors(points, points, lengths, lengths, r_normal,
                                     neighborhood_limits[layer])
        if "strided" in block:
            voxel_size = 2 * r_normal / conv_radius
            new_points, new_len, new_normals = subsample_batch(points, lengths, features=normals,
                                                               sampleDl=voxel_size)
            new_len = new_len.cpu()
            pool_i = batch_neighbors(new_points, points, new_len, lengths, r_normal,
                                     neighborhood_limits[layer])
            up_i = batch_neighbors(points, new_points, lengths, new_len, 2 * r_normal,
                                   neighborhood_limits[layer])
        if conv_i is not None:
            out["points"].append(points)
            out["stacked_lengths"].append(lengths)
            out["normals"].append(normals)
            out["neighbors"].append(conv_i.long())
        if pool_i is not None:
            out["pools"].append(pool_i.long())
            out["upsamples"].append(up_i.long())
            points, lengths, normals = new_points, new_len, new_normals
            r_normal *= 2
            layer += 1
    return out
