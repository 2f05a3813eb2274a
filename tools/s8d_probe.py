"""Probe of the s8d job's stream layout (bench.py measure_s8d_job): one 256-pair
job from pinned host inputs, chunked, with the chunk pipelines on the current
stream ("cur") or on their own streams ("lanes"), printing the median job ms per
variant.  usage: python tools/s8d_probe.py [pairs]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloudregistration_amd import _lib, synth  # noqa: E402
from pointcloudregistration_amd.pipeline import PairPipeline, default_params  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 256
B = synth.make_batch(P, n=8192, m=8192, d=32, base_seed=1000, feat_noise=1.0)
params = default_params(seed=0)
ids = np.arange(P, dtype=np.int32)


def variant(C, L, on_cur, runs=8, copy_prio=0):
    bounds = [P * c // C for c in range(C + 1)]
    hosts, devs, pipes = [], [], []
    for c in range(C):
        a, b = bounds[c], bounds[c + 1]
        h = [torch.from_numpy(np.ascontiguousarray(x[a:b])).pin_memory()
             for x in (B.src, B.tgt, B.src_feat, B.tgt_feat)]
        d = [torch.empty(t.shape, dtype=t.dtype, device="cuda") for t in h]
        hosts.append(h)
        devs.append(d)
        pipes.append(PairPipeline(*d, params, pair_ids=ids[a:b], context=c % L))
    copy_s = torch.cuda.Stream(priority=copy_prio)
    comp = torch.cuda.current_stream()
    lanes = [comp if (on_cur and k == 0) else torch.cuda.Stream() for k in range(L)]
    ev = [torch.cuda.Event() for _ in range(C)]
    rec = torch.empty((P, 40), dtype=torch.float64, device="cuda")
    if L > 1:
        _lib.call("pcr_set_concurrency", L)

    def job():
        for s in lanes:
            if s is not comp:
                s.wait_stream(comp)
        with torch.cuda.stream(copy_s):
            for c in range(C):
                for d, h in zip(devs[c], hosts[c]):
                    d.copy_(h, non_blocking=True)
                ev[c].record(copy_s)
        th = time.perf_counter()
        for c in range(C):
            s = lanes[c % L]
            s.wait_event(ev[c])
            with torch.cuda.stream(s):
                pipes[c].run()
                rec[bounds[c]:bounds[c + 1]].copy_(pipes[c].records())
        th = time.perf_counter() - th
        for s in lanes:
            if s is not comp:
                comp.wait_stream(s)
        torch.cuda.synchronize()
        return th

    for _ in range(3):
        job()
    ts, hs = [], []
    for _ in range(runs):
        t0 = time.perf_counter()
        hs.append(job())
        ts.append(time.perf_counter() - t0)
    if L > 1:
        _lib.call("pcr_set_concurrency", 1)
    print(f"C={C} L={L} lane0={'cur' if on_cur else 'own'} copy_prio={copy_prio}: job {np.median(ts) * 1e3:.2f} ms "
          f"(min {min(ts) * 1e3:.2f}), host enqueue {np.median(hs) * 1e3:.2f} ms", flush=True)
    del pipes
    torch.cuda.empty_cache()


import bench  # noqa: E402

r = bench.measure_s8d_job(B, params, ids, 1, P)
print("bench.measure_s8d_job first:", round(r["ms_per_job"], 2), flush=True)
variant(4, 1, True)
r = bench.measure_s8d_job(B, params, ids, 1, P)
print("bench.measure_s8d_job after:", round(r["ms_per_job"], 2), flush=True)
pipe = PairPipeline(B.src, B.tgt, B.src_feat, B.tgt_feat, params, pair_ids=ids)
for _ in range(200):
    pipe.run()
torch.cuda.synchronize()
del pipe
torch.cuda.empty_cache()
r = bench.measure_s8d_job(B, params, ids, 1, P)
print("bench.measure_s8d_job after 200 full steps:", round(r["ms_per_job"], 2), flush=True)
variant(4, 1, True)
