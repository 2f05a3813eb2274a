"""Benchmark driver (contract: one JSON line on rank 0).

python bench.py [--gpus N] [--steps K] [--warmup W] [--pairs P] [--points NPTS]

Workload (BASELINE.json configs[3]): P synthetic TOF/PC-style
cloud pairs of NPTS points per GPU rank (weak scaling: pair ids are
rank*P .. rank*P+P-1), inputs resident in HBM.  One step = one pass of the hot
path over the batch.  Multi-GPU: one process per GPU (torchrun), no data-path
collective, barrier + synchronize around the timed loop, max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MI355X_PEAK_FP32_TFLOPS = 157.3   # vector & f32-MFMA peak (MI355X_MICROARCH.md)
MI355X_PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=256)
    ap.add_argument("--points", type=int, default=8192)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, world):
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def make_clouds(pairs, npts, rank):
    """Synthetic pair batch generated on the GPU (seeded per rank)."""
    g = torch.Generator(device="cuda").manual_seed(1000 + rank)
    src = torch.rand(pairs, npts, 3, device="cuda", generator=g) * 2 - 1
    tgt = torch.rand(pairs, npts, 3, device="cuda", generator=g) * 2 - 1
    return src, tgt


def cpu_baseline_nnd(npts, budget_s=12.0):
    """Reference CPU nndistance (oracle/_ref, compiled from the reference's
    my_lib.cpp) on a bounded sample of the same workload, single thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle", "_ref"))
    try:
        import torch_nndistance_ref as ref
        kind = "reference"
        fwd = ref.nnd_forward
    except ImportError:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        kind = "port"

        def fwd(a, b, d1, d2, i1, i2):
            r = oracle.nnd_forward(a.numpy(), b.numpy())
            d1.copy_(torch.from_numpy(r[0]))
            return 1
    torch.set_num_threads(1)
    rng = np.random.default_rng(0)
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s or done == 0:
        a = torch.from_numpy(rng.random((1, npts, 3), dtype=np.float32) * 2 - 1)
        b = torch.from_numpy(rng.random((1, npts, 3), dtype=np.float32) * 2 - 1)
        d1, d2 = torch.zeros(1, npts), torch.zeros(1, npts)
        i1 = torch.zeros(1, npts, dtype=torch.int32)
        i2 = torch.zeros(1, npts, dtype=torch.int32)
        fwd(a, b, d1, d2, i1, i2)
        done += 1
    el = time.perf_counter() - t0
    return {"value": done / el, "unit": "pairs/s", "cores": 1, "kind": kind,
            "sample": f"{done} pairs x {npts} pts nndistance forward (both directions), "
                      f"single thread, {el:.1f}s"}


def main():
    args = parse()
    rank, world, local = dist_setup()
    from pointcloudregistration_amd import nndistance as nd

    P, N = args.pairs, args.points
    src, tgt = make_clouds(P, N, rank)
    d1 = torch.empty(P, N, device="cuda")
    d2 = torch.empty(P, N, device="cuda")
    i1 = torch.empty(P, N, dtype=torch.int32, device="cuda")
    i2 = torch.empty(P, N, dtype=torch.int32, device="cuda")

    def step():
        nd.nnd_forward_cuda(src, tgt, d1, d2, i1, i2)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    wall = max_over_ranks(wall, world)
    kern_ms = ev0.elapsed_time(ev1) / args.steps   # nnd kernel(s) per step, same stream

    total_pairs = P * world * args.steps
    value = total_pairs / wall
    # roofline of the dominant kernel (nnd sweep): 2*N*M pair evals x 8 flops per pair
    flops = 2.0 * N * N * 8 * P
    achieved = flops / (kern_ms * 1e-3) / 1e12
    out = {
        "metric": "TOF/PC pairs/sec (8192 pts)",
        "value": value,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (uniform clouds generated on device, seeded per rank)",
        "config": {"workload": "c4_chamfer_leg", "pairs_per_gpu": P, "points": N,
                   "parallelism": f"pair-sharded x{world}"},
        "roofline": {"bound": "valu", "achieved": achieved, "peak": MI355X_PEAK_FP32_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / MI355X_PEAK_FP32_TFLOPS,
                     "traffic": None, "kernel": "nnd_fwd_kernel",
                     "kernel_ms": kern_ms},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_nnd(N)
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
