"""Pair sharding across GPUs + the single result gather.

Cloud pairs are independent, so the data path has no collective: rank r of W
owns pairs [first_r, first_r + count_r) (generated or loaded locally) and runs
the whole pipeline on its own GPU.  The only exchange is one all-gather of the
fixed-size per-pair result records (40 f64 = 320 B per pair) to every rank --
RCCL over xGMI with the "nccl" backend on ROCm, gloo on CPU for tests.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import threading
import time

import torch
import torch.distributed as dist


def shard(total_pairs: int, world: int, rank: int):
    """Contiguous balanced split: (first, count) for `rank` (strong-scaling helper)."""
    base, rem = divmod(total_pairs, world)
    count = base + (1 if rank < rem else 0)
    first = rank * base + min(rank, rem)
    return first, count


def weak_shard(pairs_per_rank: int, rank: int):
    """Weak scaling: every rank owns `pairs_per_rank` distinct pairs."""
    return rank * pairs_per_rank, pairs_per_rank


def gather_records(rec: torch.Tensor, world: int, rows: int | None = None):
    """All-gather the ranks' (P_r, W) record blocks; returns (world*rows, W) on every
    rank, rank r's records at rows [r*rows, r*rows + P_r) (zero padding after them).
    `rows` >= every P_r (default: this rank's P, i.e. equal shards)."""
    rows = rec.shape[0] if rows is None else int(rows)
    if rows < rec.shape[0]:
        raise ValueError(f"rows={rows} < this rank's {rec.shape[0]} records")
    if rows > rec.shape[0]:
        pad = torch.zeros((rows - rec.shape[0],) + tuple(rec.shape[1:]), dtype=rec.dtype,
                          device=rec.device)
        rec = torch.cat([rec, pad], 0)
    if world == 1:
        return rec
    rec = rec.contiguous()
    if dist.get_backend() == "nccl":
        out = torch.empty((world * rec.shape[0],) + tuple(rec.shape[1:]), dtype=rec.dtype,
                          device=rec.device)
        dist.all_gather_into_tensor(out, rec)
        return out
    parts = [torch.empty_like(rec) for _ in range(world)]
    dist.all_gather(parts, rec)
    return torch.cat(parts, 0)


def launch_local_ranks(cmd, world: int, timeout=1800.0):
    """Start `world` copies of `cmd` as rank processes of one node (RANK, LOCAL_RANK,
    WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT): what
    torchrun --nproc-per-node would do, for a parent that must not touch the GPU
    itself.  Returns (exit code, rank 0's stdout): 0 only if every rank exited 0.
    Every rank is polled: as soon as ANY rank exits non-zero the others (blocked
    in a collective, waiting for it) are ended, and so are all of them after
    `timeout` seconds (None: no limit)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs, out = [], []
    rcs = [None] * world
    reader = None
    try:
        for r in range(world):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                       LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=str(port))
            procs.append(subprocess.Popen(cmd, env=env,
                                          stdout=subprocess.PIPE if r == 0 else None))
        # rank 0's stdout is drained on a thread so a full pipe never blocks it
        reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read()), daemon=True)
        reader.start()
        deadline = None if timeout is None else time.monotonic() + timeout
        while True:
            rcs = [p.poll() for p in procs]
            if all(c is not None for c in rcs) or any(c not in (None, 0) for c in rcs):
                break
            if deadline is not None and time.monotonic() > deadline:
                print(f"launch_local_ranks: timeout after {timeout} s", file=sys.stderr)
                break
            time.sleep(0.1)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        rcs = [p.wait() for p in procs]  # a killed rank reports a negative code
        if reader is not None:
            reader.join(timeout=10)
    rc = 0 if all(c == 0 for c in rcs) else 1
    if rc:
        print(f"launch_local_ranks: rank exit codes {rcs}", file=sys.stderr)
    return rc, (out[0] if out else b"").decode("utf-8", "replace")
