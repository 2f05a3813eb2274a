"""How far the REFERENCE's own C5 NDP trajectory moves under a change that is
mathematically nothing: the same loop as tests/golden/make_golden_c5.py (the
reference's Deformation_Pyramid imported from /root/reference, CPU f32), with
the Chamfer subset `inds` in another order -- so only the f32 summation order of
the losses and of the gradient scatter changes.  Prints the per-level maximum
relative loss deviation from the committed golden (c5_golden.npz).  Test
infrastructure (build container only): it sizes the tolerance of
tests/test_c5_full_gpu.py, whose GPU path sums the gradient exactly.

    PYTHONDONTWRITEBYTECODE=1 python tools/c5_ref_spread.py [levels] [seed]
"""
import json
import os
import sys
import time

sys.dont_write_bytecode = True
import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import make_golden_c5 as G  # noqa: E402


def main():
    levels = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    pseed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    g = np.load(os.path.join(ROOT, "tests", "golden", "c5_golden.npz"))
    B, fs, ft = G.c5_inputs()
    rs = G.rigid_stage(B, fs, ft)
    sys.path.insert(0, f"{G.REF}/c2p-net/deformationpyramid")
    from model.nets import Deformation_Pyramid
    c = G.CFG
    torch.manual_seed(G.TORCH_SEED)
    NDP = Deformation_Pyramid(depth=c["depth"], width=c["width"], device=torch.device("cpu"), k0=c["k0"],
                              m=c["m"], nonrigidity_est=c["w_reg"] > 0, rotation_format="axis_angle",
                              motion="SE3")
    est_t, tgt_t = torch.from_numpy(rs["est"]), torch.from_numpy(B.tgt[0])
    inds = torch.from_numpy(np.random.default_rng(pseed).permutation(rs["inds"]))
    s_sample = est_t - est_t.mean(dim=0, keepdims=True)
    t_sample = tgt_t - tgt_t.mean(dim=0, keepdims=True)
    BCE = torch.nn.BCELoss()
    torch.set_num_threads(os.cpu_count() or 8)
    out = []
    t0 = time.time()
    for level in range(levels):
        NDP.gradient_setup(optimized_level=level)
        opt = torch.optim.Adam(NDP.pyramid[level].parameters(), lr=c["lr"])
        brk, prev, losses = 0, 1e+6, []
        for it in range(c["iters"]):
            warped, data = NDP.warp(s_sample, max_level=level, min_level=level)
            loss = G.trunc_chamfer(warped[inds], t_sample, trunc=1e+9)
            if level > 0 and c["w_reg"] > 0:
                nr = data[level][1]
                loss = loss + c["w_reg"] * BCE(nr, torch.zeros_like(nr))
            losses.append(loss.item())
            if loss.item() < 1e-4:
                break
            if abs(prev - loss.item()) < prev * c["break_threshold_ratio"]:
                brk += 1
            if brk >= c["max_break_count"]:
                break
            prev = loss.item()
            opt.zero_grad()
            loss.backward()
            opt.step()
        want = g[f"loss/l{level}"]
        k = min(len(want), len(losses))
        rel = np.abs(np.array(losses[:k]) - want[:k]) / np.abs(want[:k])
        out.append({"level": level, "evaluated": [len(losses), len(want)], "max_rel": float(rel.max())})
        print(json.dumps(out[-1]), f"{time.time() - t0:.0f}s", flush=True)
        s_sample = warped.detach()


if __name__ == "__main__":
    main()
