"""CPU: the N>1 data path (pair sharding + the single records all-gather) with
world_size 2 over gloo."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pointcloudregistration_amd.multigpu import gather_records, shard, weak_shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, P = weak_shard(3, rank)
    rec = torch.arange(P * 40, dtype=torch.float64).reshape(P, 40) + 1000 * (first + 1)
    allrec = gather_records(rec, world)
    out[rank] = allrec.clone()
    dist.destroy_process_group()


def test_shard_partitions():
    for total in (0, 1, 7, 256, 1001):
        for world in (1, 2, 3, 8):
            spans = [shard(total, world, r) for r in range(world)]
            assert sum(c for _, c in spans) == total
            pos = 0
            for f, c in spans:
                assert f == pos
                pos += c


def test_gather_records_gloo_world2():
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    a, b = out[0], out[1]
    assert torch.equal(a, b) and a.shape == (6, 40)
    assert torch.all(a[:3, 0] >= 1000) and torch.all(a[3:, 0] >= 4000)
