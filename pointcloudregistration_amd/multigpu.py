"""Pair sharding across GPUs + the single result gather.

Cloud pairs are independent, so the data path has no collective: rank r of W
owns pairs [first_r, first_r + count_r) (generated or loaded locally) and runs
the whole pipeline on its own GPU.  The only exchange is one all-gather of the
fixed-size per-pair result records (40 f64 = 320 B per pair) to every rank --
RCCL over xGMI with the "nccl" backend on ROCm, gloo on CPU for tests.
"""
from __future__ import annotations

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


def gather_records(rec: torch.Tensor, world: int):
    """All-gather equal-size (P, W) record blocks; returns (world*P, W) on every rank."""
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
