"""Generate golden fixtures by IMPORTING the reference's own Python code (read-only,
no bytecode written) in the build container.  Outputs are data (inputs + the
reference's outputs); the reference itself never travels.

  weighted_icp     ROPNet/src/models/model_utils.py:105-139
  rigid_fit        c2p-net/deformationpyramid/model/geometry.py:8-34
  Error_R/Error_t  ROPNet/src/metrics/metrics.py:6-33
  get_coor_points  c2p-net/ngenet/models/vote.py:6-9
  vote             c2p-net/ngenet/models/vote.py:12-37
  lrf.get          dip/lrf.py:19-78
  NDP warp         c2p-net/deformationpyramid/model/nets.py:10-177 (small config)

`open3d` is not installed: an EMPTY placeholder module satisfies the top-level
`import open3d` of those files (none of the functions used here calls into it).
For lrf.get, the KD-tree is an argument of the class (lrf.py:11); it is given a
brute-force radius search object (ascending d^2, strict <, ties by index), so
the LRF math is pinned while Open3D's neighbour order is not (Open3D absent).

    python tests/golden/make_golden_py.py
"""
import os
import sys
import types

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.modules.setdefault("open3d", types.ModuleType("open3d"))


def _imp_ropnet():
    sys.path.insert(0, f"{REF}/ROPNet/src")
    from models.model_utils import weighted_icp
    from metrics.metrics import Error_R, Error_t
    return weighted_icp, Error_R, Error_t


def _imp_ndp():
    sys.path.insert(0, f"{REF}/c2p-net/deformationpyramid")
    from model.geometry import rigid_fit
    from model.nets import Deformation_Pyramid
    return rigid_fit, Deformation_Pyramid


def _rot(rng):
    q = rng.standard_normal(4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def procrustes_cases():
    weighted_icp, Error_R, Error_t = _imp_ropnet()
    rigid_fit, _ = _imp_ndp()
    rng = np.random.default_rng(2024)
    out = {}
    B, M = 4, 358   # ROPNet test: N2 = 0.4 * 896 (configs/arguments.py:29,35)
    cases = {}
    src = rng.standard_normal((B, M, 3)).astype(np.float32)
    Rs = np.stack([_rot(rng) for _ in range(B)])
    ts = rng.uniform(-0.5, 0.5, (B, 3))
    tgt_clean = (np.einsum("bij,bnj->bni", Rs, src) + ts[:, None]).astype(np.float32)
    cases["noiseless"] = (src, tgt_clean, np.ones((B, M), np.float32))
    noisy = (tgt_clean + rng.normal(0, 0.02, tgt_clean.shape)).astype(np.float32)
    cases["noisy_weighted"] = (src, noisy, rng.random((B, M)).astype(np.float32))
    refl = src.copy()
    refl[..., 2] *= -1                      # mirrored target: H has det < 0
    cases["reflection"] = (src, refl, np.ones((B, M), np.float32))
    flat = src.copy()
    flat[..., 2] = 0.0                       # coplanar (rank-2 H)
    cases["coplanar"] = (flat, (np.einsum("bij,bnj->bni", Rs, flat) + ts[:, None]).astype(np.float32),
                         rng.random((B, M)).astype(np.float32))
    for name, (s, t, w) in cases.items():
        R, tt, ts_ = weighted_icp(torch.from_numpy(s), torch.from_numpy(t), torch.from_numpy(w))
        out[f"wicp/{name}/src"], out[f"wicp/{name}/tgt"], out[f"wicp/{name}/w"] = s, t, w
        out[f"wicp/{name}/R"], out[f"wicp/{name}/t"] = R.numpy(), tt.numpy()
        out[f"wicp/{name}/transformed"] = ts_.numpy()
        R2, t2 = rigid_fit(torch.from_numpy(s), torch.from_numpy(t), torch.from_numpy(w)[..., None])
        out[f"rfit/{name}/R"], out[f"rfit/{name}/t"] = R2.numpy(), t2.numpy()
    # metrics (ROPNet Error_R / Error_t), isotropic errors in degrees / units
    R1 = np.stack([_rot(rng) for _ in range(8)])
    R2 = np.stack([_rot(rng) for _ in range(8)])
    R2[0] = R1[0]
    t1, t2 = rng.normal(size=(8, 3)), rng.normal(size=(8, 3))
    out["metrics/R1"], out["metrics/R2"], out["metrics/t1"], out["metrics/t2"] = R1, R2, t1, t2
    out["metrics/err_R"] = Error_R(R1, R2)
    out["metrics/err_t"] = Error_t(t1, t2, R2)
    return out


def vote_cases():
    sys.path.insert(0, f"{REF}/c2p-net")
    from ngenet.models.vote import get_coor_points
    rng = np.random.default_rng(7)
    out = {}
    for name, (n, m, d) in {"h32": (600, 700, 32), "d8": (400, 350, 8)}.items():
        fs = rng.standard_normal((n, d)).astype(np.float32)
        ft = rng.standard_normal((m, d)).astype(np.float32)
        tgt = rng.random((m, 3)).astype(np.float32)
        _, inds = get_coor_points(fs, ft, tgt, False)
        out[f"vote/{name}/fs"], out[f"vote/{name}/ft"], out[f"vote/{name}/inds"] = fs, ft, inds
    out.update(vote_full_case())
    return out


def vote_full_case():
    """vote() itself on a case built so that every branch occurs: targets with
    near twins (distinct indices closer than 2 voxel), sources whose m / l
    levels agree on a target while h points elsewhere (replaced), h agreeing
    too (kept), and sources with three unrelated levels."""
    from ngenet.models.vote import vote
    rng = np.random.default_rng(19)
    n, m, d, voxel = 300, 350, 16, 0.025
    tgt = rng.random((m, 3)).astype(np.float32)
    tgt[300:] = tgt[:50] + rng.uniform(-0.02, 0.02, (50, 3)).astype(np.float32)
    ft = [rng.standard_normal((m, d)).astype(np.float32) for _ in range(3)]
    t_of = rng.integers(0, m, n)
    t_twin = np.where(t_of < 50, t_of + 300, t_of)
    kind = rng.integers(0, 4, n)  # 0 all agree, 1 h off, 2 all off, 3 l on the twin
    fs = [rng.standard_normal((n, d)).astype(np.float32) for _ in range(3)]
    for lvl in range(3):
        for i in range(n):
            k = kind[i]
            j = t_of[i]
            if k == 2 or (k == 1 and lvl == 0):
                continue
            if k == 3 and lvl == 2:
                j = t_twin[i]
            fs[lvl][i] = ft[lvl][j] + np.float32(0.05) * rng.standard_normal(d).astype(np.float32)
    src = rng.random((n, 3)).astype(np.float32)
    out = {"vote/full/src": src, "vote/full/tgt": tgt, "vote/full/voxel": np.array(voxel)}
    for lvl, nm in enumerate("hml"):
        out[f"vote/full/fs_{nm}"], out[f"vote/full/ft_{nm}"] = fs[lvl].copy(), ft[lvl].copy()
    res = vote(src.copy(), tgt.copy(), [f.copy() for f in fs], [f.copy() for f in ft], voxel, False)
    out["vote/full/fs_h_out"], out["vote/full/ft_h_out"] = res[2], res[3]
    return out


class _Cloud:
    def __init__(self, pts):
        self.points = pts


class _BruteRadiusTree:
    """radius search with Open3D's return shape (k, idx, dist2); ascending d^2,
    strict d^2 < r^2, ties by index (Open3D's own order is unpinned)."""

    def __init__(self, pts):
        self.pts = np.asarray(pts, np.float64)

    def search_radius_vector_3d(self, q, r):
        d2 = ((self.pts - np.asarray(q, np.float64)[None]) ** 2).sum(1)
        idx = np.nonzero(d2 < r * r)[0]
        order = np.lexsort((idx, d2[idx]))
        idx = idx[order]
        return len(idx), list(idx), list(d2[idx])


def lrf_cases():
    sys.path.insert(0, f"{REF}/dip")
    import lrf as lrf_mod
    rng = np.random.default_rng(11)
    out = {}
    # DIP config (dip/demo.py:11-19): lrf_kernel = 3*sqrt(3), patch 256, mm-scale cloud
    pts = (rng.random((3000, 3)) * np.array([30.0, 20.0, 15.0])).astype(np.float64)
    kernel = 3 * np.sqrt(3)
    L = lrf_mod.lrf(_Cloud(pts), _BruteRadiusTree(pts), kernel, 256)
    qi = rng.choice(3000, 48, replace=False)
    patches, Ts = [], []
    for k, i in enumerate(qi):
        np.random.seed(1000 + k)
        p, _, T = L.get(pts[i])
        patches.append(p)
        Ts.append(T)
    out["lrf/pts"], out["lrf/qi"] = pts, qi.astype(np.int64)
    out["lrf/kernel"] = np.array(kernel)
    out["lrf/patches"], out["lrf/T"] = np.stack(patches), np.stack(Ts)
    return out


def ndp_cases():
    _, Deformation_Pyramid = _imp_ndp()
    torch.manual_seed(3)
    out = {}
    # small config for a compact fixture (weights stored); m=3 levels, width 32
    ndp = Deformation_Pyramid(depth=3, width=32, device="cpu", k0=-8, m=3,
                              rotation_format="axis_angle", nonrigidity_est=True, motion="SE3")
    for lvl, layer in enumerate(ndp.pyramid):
        for k, v in layer.state_dict().items():
            # perturb so the warp is far from identity (fresh init gives ~1e-3 motion)
            out[f"ndp/l{lvl}/{k}"] = v.numpy() * np.float32(3.0) if v.dim() > 1 else v.numpy()
        layer.load_state_dict({k: torch.from_numpy(out[f"ndp/l{lvl}/{k}"]) for k in layer.state_dict()})
    x = torch.from_numpy(np.random.default_rng(5).uniform(-1, 1, (500, 3)).astype(np.float32))
    with torch.no_grad():
        y, data = ndp.warp(x)
    out["ndp/x"], out["ndp/y"] = x.numpy(), y.numpy()
    for lvl in range(3):
        out[f"ndp/level{lvl}"] = data[lvl][0].numpy()
        if data[lvl][1] is not None:
            out[f"ndp/nonrigid{lvl}"] = data[lvl][1].numpy()
    return out


def main():
    np.savez_compressed(os.path.join(HERE, "procrustes_golden.npz"), **procrustes_cases())
    np.savez_compressed(os.path.join(HERE, "vote_golden.npz"), **vote_cases())
    np.savez_compressed(os.path.join(HERE, "lrf_golden.npz"), **lrf_cases())
    np.savez_compressed(os.path.join(HERE, "ndp_golden.npz"), **ndp_cases())
    for f in ("procrustes", "vote", "lrf", "ndp"):
        print(f, os.path.getsize(os.path.join(HERE, f"{f}_golden.npz")))


if __name__ == "__main__":
    main()
