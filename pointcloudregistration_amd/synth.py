"""Synthetic TOF/PC-style cloud pairs with ground truth.

There is no network and the reference's real clouds are not available, so the
benchmark and tests use a procedural closed surface (a lobed, organ-like blob in
[-1, 1]^3) sampled twice with partial overlap:

* a pool of surface points U; target = U[idx_t] + jitter, source =
  R^-1 (U[idx_s] - t) + jitter, so tgt ~ R src + t on the overlap;
* R from three axis angles U(0, max_angle) composed Rx Ry Rz and t ~ U(-0.5, 0.5)^3
  (ROPNet/src/utils/process.py:68-80 generate_random_rotation_matrix /
  generate_random_tranlation_vector);
* jitter N(0, sigma) clipped (DataPreparation/Augment.py:58-66);
* per-point descriptors (D = 32, NgeNet final_feats_dim, c2p-net/config/MRI.yaml:9)
  = a N(0,1) code per underlying surface point + N(0, feat_noise) per cloud.

Pair p of a batch uses numpy default_rng(base_seed + p), so shards on different
ranks generate disjoint, reproducible pairs.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def surface_points(rng, n):
    """n points on a lobed closed surface, area-weighted by rejection."""
    out = []
    need = n
    while need > 0:
        m = int(need * 1.6) + 64
        z = rng.uniform(-1.0, 1.0, m)
        phi = rng.uniform(0.0, 2 * np.pi, m)
        s = np.sqrt(1.0 - z * z)
        d = np.stack([s * np.cos(phi), s * np.sin(phi), z], axis=1)   # uniform on sphere
        th = np.arccos(np.clip(z, -1, 1))
        r = 1.0 + 0.25 * np.sin(3 * th) * np.cos(2 * phi) + 0.12 * np.cos(5 * phi) * s
        # rejection on the radial scale factor ~ area element r^2
        keep = rng.uniform(0, 1.45 ** 2, m) < r * r
        p = d[keep] * r[keep, None] * np.array([0.95, 0.62, 0.5])
        out.append(p)
        need -= p.shape[0]
    return np.concatenate(out)[:n]


def rotation_xyz(ax, ay, az):
    cx, sx, cy, sy, cz, sz = np.cos(ax), np.sin(ax), np.cos(ay), np.sin(ay), np.cos(az), np.sin(az)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rx @ (Ry @ Rz)


@dataclass
class PairBatch:
    src: np.ndarray        # (P, N, 3) f32
    tgt: np.ndarray        # (P, M, 3) f32
    src_feat: np.ndarray   # (P, N, D) f32
    tgt_feat: np.ndarray   # (P, M, D) f32
    R: np.ndarray          # (P, 3, 3) f64  tgt ~ R src + t
    t: np.ndarray          # (P, 3) f64
    src_uid: np.ndarray    # (P, N) i32 underlying surface point id
    tgt_uid: np.ndarray    # (P, M) i32


def make_pair(seed, n=8192, m=8192, d=32, overlap_pool=1.45, max_angle_deg=45.0,
              trans=0.5, sigma=0.001, clip=0.005, feat_noise=0.05):
    rng = np.random.default_rng(seed)
    pool_n = int(max(n, m) * overlap_pool)
    U = surface_points(rng, pool_n)
    code = rng.standard_normal((pool_n, d)).astype(np.float32)
    ang = rng.uniform(0.0, 1.0, 3) * np.deg2rad(max_angle_deg)
    R = rotation_xyz(*ang)
    t = rng.uniform(-trans, trans, 3)
    ids = rng.permutation(pool_n)[:n]
    idt = rng.permutation(pool_n)[:m]
    jit_s = np.clip(rng.normal(0.0, sigma, (n, 3)), -clip, clip)
    jit_t = np.clip(rng.normal(0.0, sigma, (m, 3)), -clip, clip)
    tgt = (U[idt] + jit_t).astype(np.float32)
    src = ((U[ids] - t) @ R + jit_s).astype(np.float32)     # R^T (u - t) == R^-1 (u - t)
    fs = (code[ids] + rng.normal(0.0, feat_noise, (n, d))).astype(np.float32)
    ft = (code[idt] + rng.normal(0.0, feat_noise, (m, d))).astype(np.float32)
    return src, tgt, fs, ft, R, t, ids.astype(np.int32), idt.astype(np.int32)


def deform_field(u, amp):
    """A smooth non-rigid displacement (C5: the intra-operative surface is a
    deformed copy of the pre-operative one): sinusoids of ~2.5 rad per unit,
    faded in along x by a logistic ramp, so one end of the blob stays rigid
    (RANSAC finds its inliers there) and the other moves by up to ~amp."""
    u = np.asarray(u, np.float64)
    ramp = 1.0 / (1.0 + np.exp(-6.0 * u[:, 0]))
    f = np.stack([np.sin(2.5 * u[:, 1] + 0.3), np.sin(2.5 * u[:, 2] + 1.1),
                  np.sin(2.5 * u[:, 0] + 2.0)], axis=1)
    return amp * ramp[:, None] * f


def make_c5_pair(seed, n=20000, m=20000, d=32, deform=0.15, feat_noise=0.5, **kw):
    """make_pair with the target deformed by deform_field before the rigid
    motion is undone on the source: tgt = U + f(U) + jitter, src = R^-1 (U - t) +
    jitter.  Returns a PairBatch of one pair (R, t = the rigid part)."""
    src, tgt, fs, ft, R, t, ids, idt = make_pair(seed, n, m, d, feat_noise=feat_noise, **kw)
    rng = np.random.default_rng(seed)
    pool_n = int(max(n, m) * kw.get("overlap_pool", 1.45))
    U = surface_points(rng, pool_n)
    tgt = (tgt + deform_field(U[idt], deform)).astype(np.float32)
    return PairBatch(*[np.stack([x]) for x in (src, tgt, fs, ft, R, t, ids, idt)])


def make_batch(pairs, n=8192, m=8192, d=32, base_seed=1000, first_pair=0, **kw):
    outs = [make_pair(base_seed + first_pair + p, n, m, d, **kw) for p in range(pairs)]
    return PairBatch(*[np.stack([o[k] for o in outs]) for k in range(8)])


def rre_rte(R_pred, t_pred, R_gt, t_gt):
    """RRE (deg) / RTE with ROPNet's definitions (ROPNet/src/metrics/metrics.py:6-33):
    RRE = arccos(clip((tr(R_gt^T R) - 1)/2)), RTE = |R_gt^T (t - t_gt)| = |t - t_gt|."""
    R_pred, R_gt = np.asarray(R_pred, np.float64), np.asarray(R_gt, np.float64)
    rel = np.matmul(np.swapaxes(R_gt, -1, -2), R_pred)
    tr = rel[..., 0, 0] + rel[..., 1, 1] + rel[..., 2, 2]
    rre = np.degrees(np.arccos(np.clip((tr - 1) / 2, -1, 1)))
    d = np.asarray(t_pred, np.float64) - np.asarray(t_gt, np.float64)
    rte = np.linalg.norm(np.squeeze(np.swapaxes(R_gt, -1, -2) @ d[..., None], -1), axis=-1)
    return rre, rte
