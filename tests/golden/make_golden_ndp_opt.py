"""Golden vectors for f4 (the NDP level optimisation), generated in the build
container by running the reference's own Deformation_Pyramid
(c2p-net/deformationpyramid/model/nets.py, imported from /root/reference) through
the loop of Registration.optimize_deformation_pyramid
(model/registration.py:171-285, no landmarks) on the CPU in f32.

registration.py itself cannot be imported here: its loss module needs pytorch3d
(absent).  The loop below restates :196-270 line for line; the truncated
Chamfer (model/loss.py:60-218 with pytorch3d knn_points) is restated as squared
1-NN distances by brute force.  Stored: the initial weights of every level, the
inputs, the loss of every iteration of every level, the per-level warped samples
and the final warp.  Nothing from the reference is stored except these numbers.

Usage: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_ndp_opt.py
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

CFG = dict(iters=15, lr=0.01, max_break_count=15, break_threshold_ratio=0.001, w_reg=0.05,
           m=3, k0=-8, depth=3, width=128)


def trunc_chamfer(x, y, trunc=1e9):
    """loss.py:60-218 for (1, P1, 3) / (1, P2, 3), point mean over the full length."""
    d = ((x[0][:, None, :] - y[0][None, :, :]) ** 2).sum(-1)
    cx, cy = d.min(1)[0], d.min(0)[0]
    cx = torch.where(cx >= trunc, torch.zeros_like(cx), cx)
    cy = torch.where(cy >= trunc, torch.zeros_like(cy), cy)
    return cx.sum() / x.shape[1] + cy.sum() / y.shape[1]


def main():
    sys.path.insert(0, f"{REF}/c2p-net/deformationpyramid")
    from model.nets import Deformation_Pyramid
    torch.manual_seed(7)
    rng = np.random.default_rng(7)
    n, m = 1300, 1200
    u = rng.uniform(-1, 1, (n, 3))
    src = (u / np.linalg.norm(u, axis=1, keepdims=True) * 0.6).astype(np.float32)
    w = rng.uniform(-1, 1, (m, 3))
    w = w / np.linalg.norm(w, axis=1, keepdims=True) * 0.6
    tgt = (w + 0.04 * np.sin(3 * w[:, [1, 2, 0]]) + np.array([0.3, -0.1, 0.2])).astype(np.float32)
    inds = np.sort(rng.choice(n, 1100, replace=False)).astype(np.int64)
    c = CFG
    NDP = Deformation_Pyramid(depth=c["depth"], width=c["width"], device="cpu", k0=c["k0"], m=c["m"],
                              nonrigidity_est=c["w_reg"] > 0, rotation_format="axis_angle",
                              motion="SE3")
    out = {"src": src, "tgt": tgt, "inds": inds}
    for lvl, layer in enumerate(NDP.pyramid):
        for k, v in layer.state_dict().items():
            out[f"init/l{lvl}/{k}"] = v.numpy().copy()
    src_t, tgt_t = torch.from_numpy(src), torch.from_numpy(tgt)
    src_mean = src_t.mean(dim=0, keepdims=True)
    tgt_mean = tgt_t.mean(dim=0, keepdims=True)
    src_pcd, tgt_pcd = src_t - src_mean, tgt_t - tgt_mean
    s_sample, t_sample = src_pcd, tgt_pcd
    BCE = torch.nn.BCELoss()
    for level in range(NDP.n_hierarchy):
        NDP.gradient_setup(optimized_level=level)
        optimizer = torch.optim.Adam(NDP.pyramid[level].parameters(), lr=c["lr"])
        break_counter, loss_prev, losses = 0, 1e+6, []
        for it in range(c["iters"]):
            s_sample_warped, data = NDP.warp(s_sample, max_level=level, min_level=level)
            loss = trunc_chamfer(s_sample_warped[None, inds], t_sample[None], trunc=1e+9)
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
        out[f"hist/l{level}"] = (s_sample_warped + tgt_mean).detach().numpy()
        s_sample = s_sample_warped.detach()
    NDP.gradient_setup(optimized_level=-1)
    with torch.no_grad():
        warped_pcd, _ = NDP.warp(src_pcd)
    out["warped"] = (warped_pcd + tgt_mean).numpy()
    np.savez_compressed(os.path.join(HERE, "ndp_opt_golden.npz"), **out)
    print({k: np.round(v, 6).tolist() for k, v in out.items() if k.startswith("loss")})
    print(os.path.getsize(os.path.join(HERE, "ndp_opt_golden.npz")))


if __name__ == "__main__":
    main()
