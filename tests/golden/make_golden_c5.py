"""Golden vectors for C5 at its own configuration (BASELINE configs[4]):
c2p-net/testScript.py:161-192 -> deformationpyramid/model/registration.py:149-289
on one 20,000-point pair, NDP m = 9, width 128, depth 3, 40 iterations with the
early-stop rule of config/NDP.yaml:8-32.

Two parts, both computed here in the build container:

1. the rigid stage by the build's ORACLE chain (oracle/: test infrastructure):
   vote (ngenet/models/vote.py:12-37) -> exact feature 1-NN both ways -> mutual
   filter -> feature RANSAC at d = voxel = 0.025 (o3d.py:164-184 with the
   dist_thresh of testScript.py:112-114,178) -> estimate = T source (f64, then f32
   as `.float()`) -> inds = np.unique of the correspondence sources
   (testScript.py:183).  Stored: T, the inlier sources, SHA-256 of the estimate.
   The 20k x 20k screens take seconds here; the GPU test compares against these
   numbers instead of re-running the oracle on the box.
2. the NDP stage by the REFERENCE's own Deformation_Pyramid (nets.py, imported
   from /root/reference) run through the loop of optimize_deformation_pyramid
   (:196-270 restated as in make_golden_ndp_opt.py) on the CPU in f32, fed with
   part 1's estimate / target / inds.  pytorch3d is absent: its knn_points
   Chamfer is restated as the exact squared 1-NN distance (argmin by chunks,
   then the distance recomputed from the gathered neighbour so autograd sees
   the same graph as knn_points' gather).  Stored: the losses of every
   iteration of every level, every 10th row of each level's warped samples and
   of the final warp, the initial weights (checked equal to the build's mirror
   under the same torch seed; if equal only their checksum is kept).

Nothing from the reference is stored except these numbers.
Usage: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_c5.py
"""
import hashlib
import os
import sys
import time
import types

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.modules.setdefault("open3d", types.ModuleType("open3d"))

# config/NDP.yaml:8-32 (early stop active, as the reference runs it)
CFG = dict(iters=40, lr=0.01, max_break_count=15, break_threshold_ratio=0.001, w_reg=0.05,
           m=9, k0=-8, depth=3, width=128)
N_PTS, SEED, LEVEL_SEED, VOXEL, RANSAC_SEED, TORCH_SEED, ROW_STEP = 20000, 515, 5, 0.025, 1, 7, 10


def c5_inputs():
    """The bench's C5 pair (bench.measure_c5): synth.make_c5_pair(515) (target
    non-rigidly deformed by up to ~0.15), three feature levels h / m / l = f,
    f + N(0, 0.6), f + N(0, 0.6) from default_rng(5)."""
    from pointcloudregistration_amd import synth
    B = synth.make_c5_pair(SEED, n=N_PTS, m=N_PTS, d=32)
    rng = np.random.default_rng(LEVEL_SEED)

    def lv(f):
        return [f] + [(f + rng.normal(0, 0.6, f.shape)).astype(np.float32) for _ in range(2)]
    return B, lv(B.src_feat[0]), lv(B.tgt_feat[0])


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def knn_sq(x, y, chunk=2048):
    """squared 1-NN distance of every row of x in y (exact direct form), with
    the autograd graph of a gather: argmin without grad, then (x - y[idx])^2."""
    with torch.no_grad():
        idx = torch.empty(x.shape[0], dtype=torch.long)
        for a in range(0, x.shape[0], chunk):
            d = ((x[a:a + chunk, None, :] - y[None, :, :]) ** 2).sum(-1)
            idx[a:a + chunk] = d.argmin(1)
    return ((x - y[idx]) ** 2).sum(-1)


def trunc_chamfer(x, y, trunc=1e9):
    """loss.py:60-218 (batch 1, squared distances, mean over the full length)."""
    cx, cy = knn_sq(x, y), knn_sq(y, x)
    cx = torch.where(cx >= trunc, torch.zeros_like(cx), cx)
    cy = torch.where(cy >= trunc, torch.zeros_like(cy), cy)
    return cx.sum() / x.shape[0] + cy.sum() / y.shape[0]


def rigid_stage(B, fs, ft):
    import oracle as O
    src, tgt = B.src[0], B.tgt[0]
    out, rep = O.vote(src, tgt, fs, ft, VOXEL)
    fs_h, ft_h = out[2], out[3]
    co = O.corres(O.featnn(fs_h, ft_h), O.featnn(ft_h, fs_h), True, 3)
    r = O.ransac(src, tgt, co, VOXEL, dist_check=VOXEL, seed=RANSAC_SEED, pair_id=0)
    T = r["T"]
    p = src.astype(np.float64)
    est = np.stack([((T[k, 0] * p[:, 0] + T[k, 1] * p[:, 1]) + T[k, 2] * p[:, 2]) + T[k, 3]
                    for k in range(3)], axis=1).astype(np.float32)
    inds = np.unique(r["correspondence_set"][:, 0]).astype(np.int64)
    return dict(T=T, est=est, inds=inds, replaced=int(rep.sum()), n_corres=int(len(co)),
                ransac=r, fs_h=fs_h, ft_h=ft_h)


def main():
    t0 = time.time()
    B, fs, ft = c5_inputs()
    rs = rigid_stage(B, fs, ft)
    print(f"rigid stage {time.time() - t0:.1f}s: corres {rs['n_corres']}, inliers {len(rs['inds'])}, "
          f"replaced {rs['replaced']}, iters {rs['ransac']['iters']}", flush=True)
    sys.path.insert(0, f"{REF}/c2p-net/deformationpyramid")
    from model.nets import Deformation_Pyramid
    c = CFG
    torch.manual_seed(TORCH_SEED)
    NDP = Deformation_Pyramid(depth=c["depth"], width=c["width"], device="cpu", k0=c["k0"], m=c["m"],
                              nonrigidity_est=c["w_reg"] > 0, rotation_format="axis_angle",
                              motion="SE3")
    # the build's mirror under the same seed: same initial weights?
    from pointcloudregistration_amd import ndp_opt
    torch.manual_seed(TORCH_SEED)
    mine = ndp_opt.DeformationPyramid(c["depth"], c["width"], torch.device("cpu"), c["k0"], c["m"],
                                      c["w_reg"] > 0)
    init = {}
    same = True
    for lvl, (a, b) in enumerate(zip(NDP.pyramid, mine.pyramid)):
        sa, sb = a.state_dict(), b.state_dict()
        same = same and list(sa) == list(sb) and all(torch.equal(sa[k], sb[k]) for k in sa)
        for k, v in sa.items():
            init[f"init/l{lvl}/{k}"] = v.numpy().copy()
    out = {"seeds": np.array([N_PTS, SEED, LEVEL_SEED, RANSAC_SEED, TORCH_SEED, ROW_STEP]),
           "voxel": np.float64(VOXEL),
           "inputs_sha": np.array(sha(B.src[0], B.tgt[0], *fs, *ft)),
           "T": rs["T"], "inds": rs["inds"], "estimate_sha": np.array(sha(rs["est"])),
           "vote_sha": np.array(sha(rs["fs_h"], rs["ft_h"])),
           "ransac_stats": np.array([rs["ransac"]["iters"], rs["ransac"]["validated"],
                                     rs["ransac"]["best_itr"], rs["n_corres"]]),
           "init_sha": np.array(sha(*[init[k] for k in sorted(init)])),
           "init_from_mirror_seed": np.array(same)}
    if not same:
        out.update(init)
    print("initial weights equal the mirror's under the same seed:", same, flush=True)
    est_t, tgt_t = torch.from_numpy(rs["est"]), torch.from_numpy(B.tgt[0])
    inds = torch.from_numpy(rs["inds"])
    src_mean = est_t.mean(dim=0, keepdims=True)
    tgt_mean = tgt_t.mean(dim=0, keepdims=True)
    src_pcd, tgt_pcd = est_t - src_mean, tgt_t - tgt_mean
    s_sample, t_sample = src_pcd, tgt_pcd
    BCE = torch.nn.BCELoss()
    torch.set_num_threads(os.cpu_count() or 8)
    for level in range(NDP.n_hierarchy):
        NDP.gradient_setup(optimized_level=level)
        optimizer = torch.optim.Adam(NDP.pyramid[level].parameters(), lr=c["lr"])
        break_counter, loss_prev, losses = 0, 1e+6, []
        for it in range(c["iters"]):
            s_sample_warped, data = NDP.warp(s_sample, max_level=level, min_level=level)
            loss = trunc_chamfer(s_sample_warped[inds], t_sample, trunc=1e+9)
            if level > 0 and c["w_reg"] > 0:
                nonrigidity = data[level][1]
                loss = loss + c["w_reg"] * BCE(nonrigidity, torch.zeros_like(nonrigidity))
            losses.append(loss.item())
            if loss.item() < 1e-4:
                break
            if abs(loss_prev - loss.item()) < loss_prev * c["break_threshold_ratio"]:
                break_counter += 1
            if break_counter >= c["max_break_count"]:
                break
            loss_prev = loss.item()
            optimizer.zero_grad()
            loss.backward()
            optimizer.step()
        out[f"loss/l{level}"] = np.array(losses)
        out[f"hist/l{level}"] = (s_sample_warped + tgt_mean).detach().numpy()[::ROW_STEP].copy()
        s_sample = s_sample_warped.detach()
        print(f"level {level}: {len(losses)} iterations, loss {losses[0]:.6g} -> {losses[-1]:.6g} "
              f"({time.time() - t0:.0f}s)", flush=True)
    NDP.gradient_setup(optimized_level=-1)
    with torch.no_grad():
        warped_pcd, _ = NDP.warp(src_pcd)
    out["warped"] = (warped_pcd + tgt_mean).numpy()[::ROW_STEP].copy()
    path = os.path.join(HERE, "c5_golden.npz")
    np.savez_compressed(path, **out)
    print(path, os.path.getsize(path), f"{time.time() - t0:.0f}s")


if __name__ == "__main__":
    main()
