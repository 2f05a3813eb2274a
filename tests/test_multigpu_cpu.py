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


_RANK_SCRIPT = r"""
import os, sys, json
import torch, torch.distributed as dist
sys.path.insert(0, {root!r})
from pointcloudregistration_amd.multigpu import gather_records, shard
world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
dist.init_process_group("gloo")
total = 5                                   # uneven: 3 + 2 pairs
first, P = shard(total, world, rank)
rows = -(-total // world)
rec = torch.arange(P, dtype=torch.float64)[:, None].repeat(1, 40) + first
allrec = gather_records(rec, world, rows)
if rank == 0:
    print(json.dumps({{"world": world, "col0": allrec[:, 0].tolist()}}))
dist.destroy_process_group()
sys.exit(int(os.environ.get("FAIL_RANK", "-1")) == rank)
"""


def test_launch_local_ranks_gloo_world2(tmp_path):
    """bench.py --gpus N without torchrun: the parent starts N rank processes
    (multigpu.launch_local_ranks) that rendezvous on 127.0.0.1; rank 0's line is
    relayed; uneven shards are padded to equal gather blocks."""
    import json
    import sys

    from pointcloudregistration_amd.multigpu import launch_local_ranks
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT.format(root=root))
    rc, out = launch_local_ranks([sys.executable, str(script)], 2, timeout=120)
    assert rc == 0
    line = json.loads(out.strip().splitlines()[-1])
    assert line["world"] == 2
    assert line["col0"] == [0.0, 1.0, 2.0, 3.0, 4.0, 0.0]


def test_launch_local_ranks_reports_failure(tmp_path, monkeypatch):
    import sys

    from pointcloudregistration_amd.multigpu import launch_local_ranks
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT.format(root=root))
    monkeypatch.setenv("FAIL_RANK", "1")
    rc, _ = launch_local_ranks([sys.executable, str(script)], 2, timeout=120)
    assert rc != 0


def test_bench_rejects_world_mismatch():
    """--gpus must match a launcher's WORLD_SIZE (else the line would mislabel n_gpus)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
