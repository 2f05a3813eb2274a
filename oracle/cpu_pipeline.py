"""CPU-baseline worker for bench.py (TEST/MEASUREMENT INFRASTRUCTURE ONLY).

One process = one host core: runs the oracle's C restatement of the C4 per-pair
pipeline (oracle/pcr_oracle.c: featnn both ways -> mutual corres -> sequential
RANSAC -> ICP -> nnd Chamfer of the aligned pair) single-threaded on the pairs
assigned to it (pair w, w + W, w + 2W, ... of the input file) until its time
budget is spent, then writes its per-pair transforms and its own elapsed time.

bench.py starts W of these as child processes BEFORE it touches the GPU, so the
pairs run in parallel across the host cores ("pairs spread across all
host cores"); the reference's own RANSAC.py loop is one pair at a time on one
core (DataPreparation/RANSAC.py:109-122).

usage: python cpu_pipeline.py IN_DIR OUT.npz WORKER NWORKERS BUDGET_S
(IN_DIR holds one .npy per array, memory-mapped by every worker)
"""
import os
import sys
import time

os.environ["OMP_NUM_THREADS"] = "1"   # before liboracle (OpenMP featnn) loads

import numpy as np  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import oracle  # noqa: E402


def run_pair(z, p):
    src, tgt = np.array(z["src"][p]), np.array(z["tgt"][p])
    fs, ft = np.array(z["src_feat"][p]), np.array(z["tgt_feat"][p])
    d_r, d_i = float(z["ransac_d"]), float(z["icp_d"])
    nn12 = oracle.featnn(fs, ft)
    nn21 = oracle.featnn(ft, fs)
    co = oracle.corres(nn12, nn21, True, 3)
    r = oracle.ransac(src, tgt, co, d_r, 3, 0.9, None, 100000, 0.999, int(z["seed"]),
                      int(z["pair_ids"][p]))
    ic = oracle.icp(src, tgt, d_i, init=r["T"])
    T = ic["T"]
    aligned = (src.astype(np.float64) @ T[:3, :3].T + T[:3, 3]).astype(np.float32)
    oracle.nnd_forward(aligned[None], tgt[None])
    return r["T"], T


def main():
    inp, out, w, W, budget = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), \
        float(sys.argv[5])
    z = {f[:-4]: np.load(os.path.join(inp, f), mmap_mode="r") for f in os.listdir(inp)
         if f.endswith(".npy")}
    P = z["src"].shape[0]
    oracle.lib()
    done, Tr, Ti = [], [], []
    t0 = time.perf_counter()
    p = w
    while p < P and (time.perf_counter() - t0 < budget or not done):
        a, b = run_pair(z, p)
        done.append(p)
        Tr.append(a)
        Ti.append(b)
        p += W
    el = time.perf_counter() - t0
    np.savez(out, pairs=np.array(done, np.int32), T_ransac=np.array(Tr).reshape(-1, 4, 4),
             T_icp=np.array(Ti).reshape(-1, 4, 4), elapsed=np.float64(el))


if __name__ == "__main__":
    main()
