"""f3: the on-disk formats around the path and their batched producers.

* RANSAC dataset dict (DataPreparation/RANSAC.py:102-131): keys ``source``,
  ``target``, ``src_normals``, ``tgt_normals``, ``transformation``,
  ``inlier_rmse``, ``inlier_ratio``, ``correspondence`` -- one list entry per kept
  pair, pairs with fewer than 1000 ICP correspondences dropped (:109-110),
  ``inlier_ratio = len(correspondence_set) / len(target)`` (:116).  Read by
  DataPreparation/CPD.py:27-28 and dip/preprocess_correspondences.py:24-25.
  ``ransac_dataset`` builds it from batched GPU results; ``save_pickle`` /
  ``load_pickle`` write and read the same pickle (pickle executes code on load:
  only open files you produced yourself).
* Ground-truth correspondences of dip/preprocess_correspondences.py:45-58: per
  pair, ICP (point-to-point, identity init) of ``source.transform(T)`` against
  ``target`` with threshold 0.7 ('original') / 0.03, and its correspondence set.
  ``icp_correspondences`` runs all pairs in one ICP launch: the source is passed
  untransformed with ``init = T``, which applies T in f64 inside the kernel --
  the coordinates Open3D's ``transform`` produces -- and returns the same sets.
  The reference stores them in an hdf5 file (one gzip dataset per pair);
  ``save_correspondences`` writes that layout when h5py is importable and an
  ``.npz`` with the same dataset names otherwise (h5py is not in this image).
"""
from __future__ import annotations

import pickle

import numpy as np
import torch

from . import registration as reg

RANSAC_KEYS = ("source", "target", "src_normals", "tgt_normals", "transformation",
               "inlier_rmse", "inlier_ratio", "correspondence")


def ransac_dataset(sources, targets, src_normals, tgt_normals, icp_results, min_corr=1000):
    """The RANSAC.py dict from per-pair clouds / normals (lists of (n, 3) arrays) and
    ICP results (objects with .transformation, .inlier_rmse, .correspondence_set,
    e.g. RegistrationResult or (T, rmse, corr) tuples)."""
    data = {k: [] for k in RANSAC_KEYS}
    for s, t, ns, nt, r in zip(sources, targets, src_normals, tgt_normals, icp_results):
        if isinstance(r, tuple):
            T, rmse, corr = r
        else:
            T, rmse, corr = r.transformation, r.inlier_rmse, r.correspondence_set
        corr = np.asarray(corr)
        if len(corr) < min_corr:
            continue
        data["source"].append(np.asarray(s, dtype=np.float64))
        data["target"].append(np.asarray(t, dtype=np.float64))
        data["src_normals"].append(np.asarray(ns, dtype=np.float64))
        data["tgt_normals"].append(np.asarray(nt, dtype=np.float64))
        data["inlier_ratio"].append(len(corr) / len(t))
        data["inlier_rmse"].append(float(rmse))
        data["transformation"].append(np.asarray(T, dtype=np.float64))
        data["correspondence"].append(corr)
    return data


def save_pickle(path, data):
    with open(path, "wb") as f:
        pickle.dump(data, f)


def load_pickle(path):
    """Load a dataset pickle this package (or the reference) wrote.  Pickle runs code
    from the file: never point this at files from an untrusted source."""
    with open(path, "rb") as f:
        return pickle.load(f)


def _pad(clouds):
    n = np.array([len(c) for c in clouds], np.int32)
    out = np.zeros((len(clouds), max(int(n.max()), 1), 3), np.float32)
    for i, c in enumerate(clouds):
        out[i, :len(c)] = np.asarray(c, dtype=np.float32)
    return out, n


def icp_correspondences(data, threshold, criteria=None):
    """Correspondence sets (list of (K, 2) int32) of preprocess_correspondences.py for
    every pair of a RANSAC / CPD dataset dict, in one batched ICP launch."""
    crit = criteria or reg.ICPConvergenceCriteria()
    S, ns = _pad(data["source"])
    G, nt = _pad(data["target"])
    T = np.stack([np.asarray(t, dtype=np.float64) for t in data["transformation"]])
    prm = reg.IcpParams(float(threshold), crit.relative_fitness, crit.relative_rmse,
                        crit.max_iteration)
    br = reg.icp_batch(S, G, T, prm, n_src=ns, n_tgt=nt, want_corr=True)
    return [br.correspondence_set(p) for p in range(len(ns))]


def save_correspondences(path, corrs):
    """hdf5 with datasets '0', '1', ... (gzip) like preprocess_correspondences.py:48-58
    when h5py is available, else an .npz with the same names."""
    try:
        import h5py
    except ImportError:
        h5py = None
    if h5py is not None and not str(path).endswith(".npz"):
        with h5py.File(path, "w") as f:
            for i, c in enumerate(corrs):
                f.create_dataset(str(i), data=np.asarray(c), compression="gzip")
        return path
    path = str(path) if str(path).endswith(".npz") else str(path) + ".npz"
    np.savez_compressed(path, **{str(i): np.asarray(c) for i, c in enumerate(corrs)})
    return path


def load_correspondences(path):
    if str(path).endswith(".npz"):
        with np.load(path) as z:
            return [z[str(i)] for i in range(len(z.files))]
    import h5py
    with h5py.File(path, "r") as f:
        return [np.asarray(f[str(i)]) for i in range(len(f.keys()))]


__all__ = ["RANSAC_KEYS", "ransac_dataset", "save_pickle", "load_pickle", "icp_correspondences",
           "save_correspondences", "load_correspondences"]
