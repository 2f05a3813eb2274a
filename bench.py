"""Benchmark driver (contract: one JSON line on rank 0).

python bench.py [--gpus N] [--steps K] [--warmup W] [--pairs P] [--points NPTS]

Workload = BASELINE.json configs[3]: a job of P (default 256)
synthetic TOF/PC-style cloud pairs of NPTS points with D=32 descriptors, split
over the ranks as SURVEY §8e prescribes (rank r owns a contiguous shard of
~P/N pairs, generated locally; strong scaling), inputs resident in HBM.
One step = the whole pair pipeline over the shard (pointcloudregistration_amd/
pipeline.py): exact mutual feature NN -> RANSAC (RANSAC.py parameters) -> ICP
-> nnd Chamfer quality, then the RCCL all-gather of the per-pair records.
Multi-GPU: one process per GPU -- under torchrun, or started by this script
itself when --gpus N > 1 is given without a launcher -- barrier + synchronize
around the timed loop, max over ranks; value = all pairs of the job / that time.
Beside it: the PCIe-inclusive rate (host-resident inputs, `host_resident`), weak
scaling at N > 1 (P pairs on every rank), the pair-parallel CPU baseline and the
C2 / a4 / a10 / f1 / f2 / f4 / C5 side measurements at N = 1.
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

PEAK_F32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32 MFMA = f32 vector peak
# dense f16/bf16 MFMA: v_mfma_f32_32x32x16_f16 = 32768 flop / 32 cycles / SIMD,
# 1024 SIMDs x 2.4 GHz (MI355X_MICROARCH.md "Peak BF16/FP16 MFMA ~2.5 PF dense")
PEAK_F16_MFMA_TFLOPS = 2516.6
PEAK_HBM_GBS = 8000.0
PEAK_LDS_GBS = 256 * 256 * 2.4   # 256 CUs x 256 B/clk (ds_read_b64/b128) x 2.4 GHz, in GB/s


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=256,
                    help="pairs in the WHOLE job (SURVEY 8e: 256 split over the ranks)")
    ap.add_argument("--points", type=int, default=8192)
    ap.add_argument("--dim", type=int, default=32)
    ap.add_argument("--feat-noise", type=float, default=1.0)
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-resident", action="store_true",
                    help="skip the PCIe-inclusive (host-resident inputs) measurement")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the C2 / a4 / a10 / f1 / f4 side measurements")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as one captured HIP graph (measured: no gain at 256 pairs, "
                         "slower at 32 / 64 where the cooperative launches are recorded)")
    ap.add_argument("--s8d-chunks", type=int, default=0,
                    help="s8d_job: copy chunks per rank (0: by shard size)")
    ap.add_argument("--s8d-lanes", type=int, default=0,
                    help="s8d_job: chunk pipelines in flight (0: 1)")
    ap.add_argument("--streams", type=int, default=1,
                    help="split the rank's shard into this many sub-batches run concurrently on "
                         "their own HIP streams (1..4)")
    return ap.parse_args()


def launch_ranks(args):
    """`python bench.py --gpus N` without a launcher: start N rank processes BEFORE
    this process touches the GPU, relay rank 0's JSON line, exit non-zero if any
    rank fails (multigpu.launch_local_ranks).  Under torchrun the env already names
    the rank and this is not used."""
    from pointcloudregistration_amd.multigpu import launch_local_ranks
    rc, out0 = launch_local_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                  args.gpus)
    sys.stdout.write(out0)
    sys.stdout.flush()
    return rc


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


CPU_WORKER_CAP = 16  # the GPU box's host share per GPU (os.cpu_count() shows the whole machine)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(batch, params, budget_s, pair_ids):
    """The oracle's C restatement of the same per-pair pipeline (oracle/pcr_oracle.c:
    featnn both ways -> mutual corres -> sequential RANSAC -> ICP -> nnd Chamfer),
    pair-parallel: one single-threaded worker process per host core
    (oracle/cpu_pipeline.py), each taking pairs w, w+W, ... of the workload for
    ~budget_s seconds.  Runs before this process touches the GPU (the workers are
    plain child processes).  value = sum over workers of pairs / own elapsed."""
    import shutil
    import subprocess
    import tempfile
    aff = len(os.sched_getaffinity(0))
    W = max(1, min(aff, CPU_WORKER_CAP))
    k = min(batch.src.shape[0], 8 * W)
    tmp = tempfile.mkdtemp(prefix="pcr_cpu_")
    try:
        inp = os.path.join(tmp, "in")
        os.mkdir(inp)
        arrays = dict(src=batch.src[:k], tgt=batch.tgt[:k], src_feat=batch.src_feat[:k],
                      tgt_feat=batch.tgt_feat[:k], pair_ids=np.asarray(pair_ids[:k], np.int32),
                      ransac_d=np.float64(params.ransac.max_correspondence_distance),
                      icp_d=np.float64(params.icp.max_correspondence_distance),
                      seed=np.int64(params.ransac.seed))
        for name, arr in arrays.items():
            np.save(os.path.join(inp, name + ".npy"), arr)
        env = dict(os.environ, OMP_NUM_THREADS="1")
        worker = os.path.join(ROOT, "oracle", "cpu_pipeline.py")
        procs = [subprocess.Popen([sys.executable, worker, inp, os.path.join(tmp, f"o{w}.npz"),
                                   str(w), str(W), str(budget_s)], env=env) for w in range(W)]
        rcs = [p.wait() for p in procs]
        if any(rcs):
            raise RuntimeError(f"cpu baseline workers failed: {rcs}")
        rate, done, Ts = 0.0, 0, {}
        for w in range(W):
            z = np.load(os.path.join(tmp, f"o{w}.npz"))
            n = len(z["pairs"])
            rate += n / float(z["elapsed"])
            done += n
            for i, p in enumerate(z["pairs"]):
                Ts[int(p)] = (z["T_ransac"][i], z["T_icp"][i])
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return ({"value": rate, "unit": "pairs/s", "cores": W, "affinity_cpus": aff,
             "cpu_model": _cpu_model(), "kind": "port",
             "per_gpu_share": {"value": rate, "cores": W,
                               "note": "the GPU box's host share per GPU (16 cores); the pool "
                                       "forbids more workers than that"},
             "whole_host_extrapolated": {"value": rate * aff / W, "cores": aff,
                                         "note": "per-worker rate x every affinity core (pair-"
                                                 "parallel, no shared state: linear in cores "
                                                 "up to memory bandwidth); not measured"},
             "sample": f"{done} of the workload's pairs ({batch.src.shape[1]} pts, D="
                       f"{batch.src_feat.shape[2]}) through the oracle pipeline (featnn x2, "
                       f"mutual corres, RANSAC, ICP, Chamfer), {W} single-threaded worker "
                       f"processes for ~{budget_s:.0f} s each; value = sum of per-worker rates"},
            Ts)


def _events_ms(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def _graph_ms(fn, reps):
    """Device time per call: `reps` calls captured in one HIP graph and replayed
    (no host dispatch between the launches -- what a caller that captures or
    batches its calls pays); the eager per-call time is _events_ms."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(4):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (4 * reps)


def measure_lrf(with_cpu):
    """a4 on the C3 shape (dip/demo.py: 2 clouds, 2048 sampled points each,
    kernel 3*sqrt(3), patch 256): synthetic surface clouds of 20k points scaled
    to ~170 neighbours per ball.  GPU time = both phases (count + frames) for
    4096 queries; the host choice draws are timed separately."""
    from pointcloudregistration_amd import _lib, synth
    from pointcloudregistration_amd import lrf as L
    rng = np.random.default_rng(77)
    clouds = np.stack([synth.surface_points(rng, 20000) * 40.0 for _ in range(2)])
    qidx = np.stack([rng.choice(20000, 2048, replace=False) for _ in range(2)])
    qs = np.stack([clouds[p][qidx[p]] for p in range(2)])
    ker, ps = 3.0 * np.sqrt(3.0), 256
    P_ = torch.as_tensor(clouds, device="cuda").contiguous()
    Q_ = torch.as_tensor(qs, device="cuda").contiguous()
    counts = torch.zeros(2, 2048, dtype=torch.int32, device="cuda")
    st = _lib.stream_handle()
    _lib.call("pcr_lrf_count", _lib.ptr(P_), 2, 20000, None, _lib.ptr(Q_), 2048, None, ker,
              _lib.ptr(counts), st)
    cnt = counts.cpu().numpy()
    # the draws in demo.py's order (frag1 i, frag2 i, ...): libpcr's restatement
    # of legacy RandomState.choice (the product path) and numpy's own loop
    np.random.seed(3)
    t0 = time.perf_counter()
    inds = L.legacy_choice_batch(np.maximum(cnt.T.reshape(-1), ps), ps)
    host_ms = (time.perf_counter() - t0) * 1e3
    inds = np.ascontiguousarray(inds.reshape(2048, 2, ps).transpose(1, 0, 2))
    np.random.seed(3)
    t0 = time.perf_counter()
    ref = np.stack([np.random.choice(max(int(cnt[p, i]), ps), ps, replace=False)
                    for i in range(2048) for p in range(2)])
    numpy_ms = (time.perf_counter() - t0) * 1e3
    draws_equal = bool(np.array_equal(ref.reshape(2048, 2, ps).transpose(1, 0, 2), inds))
    I_ = torch.as_tensor(inds, device="cuda").contiguous()
    patches = torch.empty(2, 2048, ps, 3, dtype=torch.float64, device="cuda")
    T = torch.empty(2, 2048, 16, dtype=torch.float64, device="cuda")
    kmax = int(cnt.max())

    def run():
        _lib.call("pcr_lrf_count", _lib.ptr(P_), 2, 20000, None, _lib.ptr(Q_), 2048, None, ker,
                  _lib.ptr(counts), st)
        _lib.call("pcr_lrf_compute", _lib.ptr(P_), 2, 20000, None, _lib.ptr(Q_), 2048, None, ker,
                  ps, _lib.ptr(I_), kmax, _lib.ptr(patches), _lib.ptr(T), None, st)
    ms = _events_ms(run, 5)
    # algorithmic work: two f64 sweeps of the cloud per query (3 sub, 3 mul, 2 add)
    flops = 4096 * 2 * 20000 * 8.0
    res = {"workload": "C3 DIP: 2 clouds x 20000 pts, 2 x 2048 queries, kernel 3*sqrt(3), patch 256",
           "gpu_ms": ms, "queries_per_s": 4096 / (ms * 1e-3), "host_choice_ms": host_ms,
           "host_choice_numpy_loop_ms": numpy_ms, "host_choice_equal_to_numpy": draws_equal,
           "median_neighbours": float(np.median(cnt)),
           "roofline": {"bound": "valu-f64", "achieved_tflops": flops / (ms * 1e-3) / 1e12,
                        "peak_tflops": 78.6, "note": "brute-force f64 sweeps; cloud is L2-resident"}}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        t0 = time.perf_counter()
        n = 64
        for i in range(n):
            O.lrf(clouds[0], qs[0][i], ker, ps, inds[0][i])
        cpu_ms = (time.perf_counter() - t0) * 1e3 / n
        res["cpu_baseline"] = {"ms_per_query": cpu_ms, "cores": 1, "kind": "port",
                               "sample": f"{n} queries through oracle_lrf (brute-force radius)",
                               "reference_measured_ms_per_query": 0.47}
    return res


def measure_ndp(with_cpu):
    """a10 on the C5 shape (config/NDP.yaml: width 128, depth 3, m 9 levels,
    k0 -8, SE3 axis_angle, nonrigidity on levels > 0) over 20000 points."""
    from pointcloudregistration_amd import ndp
    rng = np.random.default_rng(5)
    W, n = 128, 20000
    levels = []
    for i in range(9):
        sd = {"input.0.weight": rng.normal(0, 0.5, (W, 6)), "input.0.bias": rng.normal(0, .1, W)}
        for k in range(2):
            sd[f"mlp.pts_linears.{k}.weight"] = rng.normal(0, 1 / np.sqrt(W), (W, W))
            sd[f"mlp.pts_linears.{k}.bias"] = rng.normal(0, .1, W)
        for b in ("rot_brach", "trn_branch"):
            sd[f"{b}.weight"] = rng.normal(0, 1, (3, W))
            sd[f"{b}.bias"] = rng.normal(0, .1, 3)
        if i > 0:
            sd["nr_branch.weight"] = rng.normal(0, 1, (1, W))
            sd["nr_branch.bias"] = rng.normal(0, .1, 1)
        levels.append({k: torch.as_tensor(v.astype(np.float32), device="cuda")
                       for k, v in sd.items()})
    x = torch.as_tensor(rng.uniform(-1, 1, (n, 3)).astype(np.float32), device="cuda")
    pyr = ndp.PreparedPyramid(levels)
    ms = _events_ms(lambda: pyr.warp(x, per_level=False), 10)
    flops = n * 9 * 2.0 * (6 * W + 2 * W * W + 7 * W)
    res = {"workload": "C5 NDP warp: 20000 pts x 9 levels, width 128, depth 3 (random init)",
           "gpu_ms": ms, "point_levels_per_s": n * 9 / (ms * 1e-3),
           "roofline": {"bound": "mfma", "achieved": flops / (ms * 1e-3) / 1e12,
                        "peak": PEAK_F32_MFMA_TFLOPS, "unit": "TFLOP/s",
                        "frac": flops / (ms * 1e-3) / 1e12 / PEAK_F32_MFMA_TFLOPS,
                        "kernel": "ndp_warp_kernel<4> (v_mfma_f32_32x32x2_f32)"}}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        lv = [{k: v.cpu().numpy() for k, v in L.items()} for L in levels]
        xc = x.cpu().numpy()
        t0 = time.perf_counter()
        O.ndp_warp(lv, xc)
        res["cpu_baseline"] = {"ms": (time.perf_counter() - t0) * 1e3,
                               "cores": int(os.environ.get("OMP_NUM_THREADS", "1")),
                               "kind": "port", "sample": "numpy f64 oracle, the full warp",
                               "reference_measured_ms": 137.0}
    return res


def measure_fpfh(with_cpu):
    """f1 on the C1 shape (DataPreparation/RANSAC.py:12-64, voxel 0.01: normals
    r 0.04 / 30, FPFH r 0.07 / 100, feature RANSAC d 0.04 mutual, ICP d 0.02) for
    one 1024-point pair, end to end through the Open3D-shaped drop-ins; plus the
    batched normals+FPFH kernels on 64 clouds x 8192 points (C4 cloud shape)."""
    from pointcloudregistration_amd import features as F
    from pointcloudregistration_amd import registration as reg
    from pointcloudregistration_amd import synth
    rng = np.random.default_rng(1)
    tgt = (synth.surface_points(rng, 1024) * 0.5).astype(np.float32)
    R = synth.rotation_xyz(*np.deg2rad(rng.uniform(-90, 90, 3)))
    t = rng.uniform(-1.5, 1.5, 3)
    src = ((tgt.astype(np.float64) @ R.T + t)
           + np.clip(rng.normal(0, 0.001, tgt.shape), -0.005, 0.005)).astype(np.float32)
    voxel, d = 0.01, 0.04

    def c1():
        s_pcd, t_pcd = reg.PointCloud(src), reg.PointCloud(tgt)
        s_pcd, s_f = F.preprocess_point_cloud(s_pcd, voxel)
        t_pcd, t_f = F.preprocess_point_cloud(t_pcd, voxel)
        res = reg.registration_ransac_based_on_feature_matching(
            s_pcd, t_pcd, s_f, t_f, True, d, reg.TransformationEstimationPointToPoint(False), 3,
            [reg.CorrespondenceCheckerBasedOnEdgeLength(0.9),
             reg.CorrespondenceCheckerBasedOnDistance(d)],
            reg.RANSACConvergenceCriteria(100000, 0.999))
        return reg.registration_icp(s_pcd, t_pcd, 0.02, res.transformation,
                                    reg.TransformationEstimationPointToPoint())
    icp = c1()
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        c1()
    torch.cuda.synchronize()
    c1_ms = (time.perf_counter() - t0) * 1e3 / reps
    rre, rte = synth.rre_rte(icp.transformation[None, :3, :3], icp.transformation[None, :3, 3],
                             R.T[None], (-R.T @ t)[None])
    # batched kernels: normals (r 0.04, 30) + FPFH (r 0.07, 100) on 64 x 8192 points
    P, N = 64, 8192
    clouds = np.stack([synth.surface_points(np.random.default_rng(100 + p), N) for p in range(P)])
    X = torch.as_tensor(clouds.astype(np.float32), device="cuda")

    def batch():
        nm = F.estimate_normals_batch(X, 0.04, 30)
        return F.compute_fpfh_batch(X, nm, 0.07, 100)
    ms = _events_ms(batch, 3)
    _, _, cnt = F.hybrid_search_batch(X, 0.07, 100)
    res = {"workload": "C1 RANSAC.py: 2 x 1024 pts, normals + FPFH + feature RANSAC + ICP (wall "
                       "clock, host-synchronous drop-ins); batch: 64 x 8192 pts normals + FPFH",
           "c1_ms_per_pair": c1_ms, "c1_rre_deg": float(rre[0]), "c1_rte": float(rte[0]),
           "c1_fitness": icp.fitness,
           "batch_gpu_ms": ms, "batch_points_per_s": P * N / (ms * 1e-3),
           "batch_median_fpfh_neighbours": float(cnt.float().median().item())}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        t0 = time.perf_counter()
        ns, nt = O.estimate_normals(src, 4 * voxel, 30), O.estimate_normals(tgt, 4 * voxel, 30)
        fs = O.fpfh(src, ns, 7 * voxel, 100)[1].astype(np.float32)
        ft = O.fpfh(tgt, nt, 7 * voxel, 100)[1].astype(np.float32)
        corr = O.corres(O.featnn(fs, ft), O.featnn(ft, fs), True, 3)
        o = O.ransac(src, tgt, corr, d, dist_check=d)
        oi = O.icp(src, tgt, 0.02, o["T"])
        cpu_ms = (time.perf_counter() - t0) * 1e3
        res["cpu_baseline"] = {"c1_ms_per_pair": cpu_ms, "cores": 1, "kind": "port",
                               "sample": "one C1 pair through the oracle (brute-force search)",
                               "T_icp_bitexact": bool(np.array_equal(oi["T"], icp.transformation))}
    return res


def measure_ndp_opt(with_cpu):
    """f4 on the C5 shape (config/NDP.yaml: 9 levels x 40 iterations, width 128,
    depth 3, w_reg 0.05) for a 20k-point pair with 5k Chamfer indices: the
    graph-captured optimisation vs the reference's loop structure run eagerly on
    the same GPU (torch Adam, loss.item() every iteration, same warp/Chamfer ops)."""
    from pointcloudregistration_amd import ndp_opt
    from pointcloudregistration_amd.chamfer import compute_truncated_chamfer_distance
    rng = np.random.default_rng(9)
    n = 20000
    u = rng.standard_normal((n, 3))
    src = (u / np.linalg.norm(u, axis=1, keepdims=True)).astype(np.float32)
    w = rng.standard_normal((n, 3))
    w = w / np.linalg.norm(w, axis=1, keepdims=True)
    tgt = (w + 0.05 * np.sin(3 * w[:, [1, 2, 0]])).astype(np.float32)
    inds = np.sort(rng.choice(n, 5000, replace=False))
    cfg = ndp_opt.NDPConfig(max_break_count=10**6)  # run all 9 x 40 iterations
    S, G = torch.from_numpy(src).cuda(), torch.from_numpy(tgt).cuda()

    def fresh():
        torch.manual_seed(0)
        return ndp_opt.DeformationPyramid(3, 128, torch.device("cuda"), -8, 9, True)
    ndp_opt.optimize_deformation_pyramid(S, G, inds, cfg, NDP=fresh())  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, _, _, info = ndp_opt.optimize_deformation_pyramid(S, G, inds, cfg, NDP=fresh())
    torch.cuda.synchronize()
    graph_ms = (time.perf_counter() - t0) * 1e3
    replay_ms = float(sum(i.get("replay_ms", 0.0) for i in info))
    evaluated = int(sum(i["evaluated"] for i in info))
    # f4 roofline: per iteration the level's forward, data backward and weight
    # gradients over all n points, each 2 * (6W + 2W^2 + 7W) = 68,864 flops per
    # point at W = 128, on the f32 MFMA (157.3 TF)
    flop_it = 3 * 2 * (6 * 128 + 2 * 128 * 128 + 7 * 128) * n
    f4_roof = {"bound": "mfma", "unit": "TFLOP/s", "peak": 157.3,
               "flop_per_iteration": flop_it, "iterations": evaluated,
               "achieved": flop_it * evaluated / (replay_ms * 1e-3) / 1e12 if replay_ms > 0 else None,
               "replay_ms": replay_ms,
               "note": "algorithmic flops of the MLP forward + data backward + weight gradients "
                       "(the Chamfer and Adam are extra) / the summed graph replay time of the levels"}
    if f4_roof["achieved"] is not None:
        f4_roof["frac"] = f4_roof["achieved"] / f4_roof["peak"]

    def reference_style(P):
        s = S - S.mean(0, keepdim=True)
        t = G - G.mean(0, keepdim=True)
        I = torch.as_tensor(inds, device="cuda")
        for level in range(P.n_hierarchy):
            P.gradient_setup(level)
            opt = torch.optim.Adam(P.pyramid[level].parameters(), lr=cfg.lr)
            prev, bc = 1e6, 0
            for _ in range(cfg.iters):
                x, data = P.warp(s, max_level=level, min_level=level)
                loss = compute_truncated_chamfer_distance(x[None, I], t[None], trunc=1e9)
                if level > 0:
                    nr = data[level][1]
                    loss = loss + cfg.w_reg * torch.nn.functional.binary_cross_entropy(
                        nr, torch.zeros_like(nr))
                L = loss.item()
                if L < 1e-4:
                    break
                if abs(prev - L) < prev * cfg.break_threshold_ratio:
                    bc += 1
                prev = L
                opt.zero_grad()
                loss.backward()
                opt.step()
            s = x.detach()
    reference_style(fresh())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reference_style(fresh())
    torch.cuda.synchronize()
    eager_ms = (time.perf_counter() - t0) * 1e3
    res = {"workload": "C5 NDP optimisation: 20000-pt pair, 5000 Chamfer indices, 9 levels x 40 "
                       "iterations (width 128, depth 3), wall clock",
           "graph_ms": graph_ms, "reference_loop_on_gpu_ms": eager_ms, "roofline": f4_roof,
           "iterations_per_s": 9 * 40 / (graph_ms * 1e-3), "speedup_vs_reference_loop": eager_ms / graph_ms}
    if with_cpu:
        P = ndp_opt.DeformationPyramid(3, 128, "cpu", -8, 9, True)
        Sc, Gc = torch.from_numpy(src), torch.from_numpy(tgt)
        x = Sc - Sc.mean(0, keepdim=True)
        y = Gc - Gc.mean(0, keepdim=True)
        P.gradient_setup(1)
        opt = torch.optim.Adam(P.pyramid[1].parameters(), lr=cfg.lr)
        reps = 2
        t0 = time.perf_counter()
        for _ in range(reps):
            xw, data = P.warp(x, max_level=1, min_level=1)
            d1 = torch.cdist(xw[inds], y).min(1)[0] ** 2
            d2 = torch.cdist(y, xw[inds]).min(1)[0] ** 2
            loss = d1.mean() + d2.mean()
            opt.zero_grad()
            loss.backward()
            opt.step()
        it_ms = (time.perf_counter() - t0) * 1e3 / reps
        res["cpu_baseline"] = {"ms_extrapolated": it_ms * 9 * 40, "ms_per_iteration": it_ms,
                               "cores": torch.get_num_threads(), "kind": "port",
                               "sample": f"{reps} iterations of one level on the CPU (torch, cdist "
                                         "Chamfer), x 360"}
    return res


def measure_c5(with_cpu):
    """C5 end to end (c2p-net/testScript.py:161-196) on one 20k-point pair (the
    target non-rigidly deformed, synth.make_c5_pair -- the pair of
    tests/golden/c5_golden.npz): vote over three 32-d feature levels -> mutual
    feature RANSAC at d = 0.025 -> estimate -> NDP 9 levels x <= 40 iterations
    (width 128, config/NDP.yaml's early stop, which now stops the work) on the
    unique inlier sources; wall clock per stage, inputs resident on the device."""
    from pointcloudregistration_amd import c2p, ndp_opt, registration as reg, synth
    B = synth.make_c5_pair(515, n=20000, m=20000, d=32)
    rng = np.random.default_rng(5)

    def lv(f):
        return [f] + [(f + rng.normal(0, 0.6, f.shape)).astype(np.float32) for _ in range(2)]
    fs, ft = lv(B.src_feat[0]), lv(B.tgt_feat[0])
    dev = torch.device("cuda")
    S, G = torch.from_numpy(B.src[0]).to(dev), torch.from_numpy(B.tgt[0]).to(dev)
    FS = [torch.from_numpy(f).to(dev) for f in fs]
    FT = [torch.from_numpy(f).to(dev) for f in ft]
    cfg = ndp_opt.NDPConfig()  # config/NDP.yaml
    voxel = 0.025

    def run():
        a, b = [f.clone() for f in FS], [f.clone() for f in FT]
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        _, _, fs_h, ft_h = c2p.vote(S, G, a, b, voxel)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        prm = reg.RansacParams(max_correspondence_distance=voxel, distance_check=voxel, seed=1)
        br = reg.register_feature_ransac_batch(S, G, fs_h, ft_h, prm, want_mask=False)
        est = reg.transform_batch(S.unsqueeze(0), br.transformation)[0]
        corrs = torch.nonzero(br.corr_tgt[0] >= 0).flatten().cpu().numpy()
        t.append(time.perf_counter())
        torch.manual_seed(0)
        P = ndp_opt.DeformationPyramid(3, 128, dev, -8, 9, True)
        w, _, _, info = ndp_opt.optimize_deformation_pyramid(est, G, corrs, cfg, NDP=P)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        return np.diff(t) * 1e3, br, len(corrs), info
    run()
    ms, br, k, info = run()
    T = br.transformation[0].cpu().numpy()
    rre, rte = synth.rre_rte(T[:3, :3], T[:3, 3], B.R[0], B.t[0])
    res = {"workload": "C5 flow: one 20000-pt pair, vote (3 x 32-d levels) -> feature RANSAC "
                       "d=0.025 -> NDP 9 x 40 on the inlier sources, wall clock",
           "ms": float(ms.sum()), "vote_ms": float(ms[0]), "ransac_ms": float(ms[1]),
           "ndp_ms": float(ms[2]), "inlier_sources": int(k), "rre_deg": float(rre),
           "rte": float(rte), "ndp_iterations_evaluated": [int(i["evaluated"]) for i in info]}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        rows = 500
        t0 = time.perf_counter()
        O.vote(None, B.tgt[0], [f[:rows] for f in fs], ft, voxel)
        vote_s = (time.perf_counter() - t0) * (20000 / rows)
        res["cpu_baseline"] = {"vote_ms_extrapolated": vote_s * 1e3, "cores": 1, "kind": "port",
                               "sample": f"oracle vote on {rows} of 20000 source rows "
                                         "(3 exact f64 1-NN screens + the tests), x 40"}
    return res


def measure_c3(with_cpu):
    """C3 end to end (dip/demo.py:64-178) on one pair of 40k-point mm-scale clouds:
    voxel_down_sample(1.0) -> 2 x 2048 samples -> LRF patches (3*sqrt(3), 256) ->
    descriptor network (PointNetFeature, seeded random init, D = 64, torch) ->
    5th-percentile filter -> feature RANSAC at 1.5; wall clock of the whole call."""
    from pointcloudregistration_amd import dip, synth
    rng = np.random.default_rng(31)
    U = synth.surface_points(rng, 60000) * 40.0
    R = synth.rotation_xyz(*np.deg2rad(rng.uniform(-30, 30, 3)))
    t = rng.uniform(-10, 10, 3)
    src = U[rng.permutation(60000)[:40000]] + rng.normal(0, 0.05, (40000, 3))
    tgt = (U[rng.permutation(60000)[:40000]] + rng.normal(0, 0.05, (40000, 3))) @ R.T + t
    torch.manual_seed(1)
    net = dip.PointNetFeature(64).cuda().eval()
    np.random.seed(5)
    dip.demo_register(src, tgt, net, seed=3)
    torch.cuda.synchronize()
    np.random.seed(5)
    t0 = time.perf_counter()
    out = dip.demo_register(src, tgt, net, seed=3)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    T = out["result"].transformation
    rre, rte = synth.rre_rte(T[:3, :3], T[:3, 3], R, t)
    res = {"workload": "C3 DIP demo: 2 x 40000-pt clouds (mm), voxel 1.0 -> 2 x 2048 LRF "
                       "patches -> D=64 descriptors (seeded random-init PointNetFeature) -> 5th pct filter "
                       "-> feature RANSAC d=1.5, wall clock",
           "ms": ms, "downsampled_points": [len(out["pcd1"].points), len(out["pcd2"].points)],
           "inlier_correspondences": int(len(out["result"].correspondence_set)),
           "rre_deg": float(rre), "rte_mm": float(rte)}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        ker, ps = 3.0 * np.sqrt(3.0), 256
        t0 = time.perf_counter()
        d1, _, _ = O.voxel_down_sample(src, 1.0)
        d2, _, _ = O.voxel_down_sample(tgt, 1.0)
        t_vox = time.perf_counter() - t0
        q = d1[out["inds1"][:128]]
        t0 = time.perf_counter()
        for i in range(128):
            c = O.lrf_count(d1, q[i], ker)
            O.lrf(d1, q[i], ker, ps, np.random.choice(max(c, ps), ps, replace=False))
        t_lrf = (time.perf_counter() - t0) * 4096 / 128
        g1, g2 = out["good1"], out["good2"]
        a = d1[out["inds1"]][g1].astype(np.float32)
        b = d2[out["inds2"]][g2].astype(np.float32)
        fa, fb = out["desc1"][g1].astype(np.float32), out["desc2"][g2].astype(np.float32)
        t0 = time.perf_counter()
        co = O.corres(O.featnn(fa, fb), O.featnn(fb, fa), True, 3)
        O.ransac(a, b, co, 1.5, dist_check=1.5, seed=3)
        t_reg = time.perf_counter() - t0
        res["cpu_baseline"] = {"ms": (t_vox + t_lrf + t_reg) * 1e3, "voxel_ms": t_vox * 1e3,
                               "lrf_ms_extrapolated": t_lrf * 1e3, "match_ransac_ms": t_reg * 1e3,
                               "cores": 1, "kind": "port",
                               "sample": "oracle voxel x2, LRF on 128 of 4096 queries (x 32), "
                                         "featnn x2 + RANSAC; the descriptor network is not timed"}
    return res


def measure_voxel(with_cpu):
    """f2: Open3D voxel_down_sample of 16 clouds of 200k points (3DMatch-like
    extent, 2.5 cm voxels: o3d.py / DataPreparation callers) in one batched call,
    vs the oracle's C++ restatement (one thread) on one cloud."""
    from pointcloudregistration_amd import geometry, synth
    rng = np.random.default_rng(21)
    clouds = [(synth.surface_points(rng, 200000) * 2.0).astype(np.float64) for _ in range(16)]
    dev = torch.device("cuda")
    C = [torch.from_numpy(c).to(dev) for c in clouds]
    geometry.voxel_down_sample_batch(C, 0.025)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        outs = geometry.voxel_down_sample_batch(C, 0.025)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / reps
    res = {"workload": "f2 voxel_down_sample: 16 clouds x 200000 pts, voxel 0.025, one batched call",
           "ms": ms, "points_per_s": 16 * 200000 / (ms * 1e-3),
           "out_points": int(sum(o[0].shape[0] for o in outs))}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        t0 = time.perf_counter()
        O.voxel_down_sample(clouds[0], 0.025)
        s = time.perf_counter() - t0
        res["cpu_baseline"] = {"points_per_s": 200000 / s, "cores": 1, "kind": "port",
                               "sample": "oracle (C++ unordered_map restatement) on 1 of the 16 clouds"}
    return res


def measure_c2(with_cpu):
    """C2 (BASELINE configs[1]): dip/torch-nndistance Chamfer forward on 2 x 4096
    random points (test.py:8-9 shape, U[0,1)^3, default_rng(0)), the drop-in's
    default path (certified grid) and the brute-force kernel, beside the
    reference's own CPU extension (dip/torch-nndistance/src/my_lib.cpp:28-60,
    compiled unmodified into oracle/_ref by oracle/build_ref.sh) on one core."""
    from pointcloudregistration_amd import nndistance as nd
    rng = np.random.default_rng(0)
    N = 4096
    x1 = rng.random((1, N, 3), dtype=np.float32)
    x2 = rng.random((1, N, 3), dtype=np.float32)
    t1, t2 = torch.from_numpy(x1).cuda(), torch.from_numpy(x2).cuda()
    d1, d2 = torch.empty(1, N, device="cuda"), torch.empty(1, N, device="cuda")
    i1 = torch.empty(1, N, dtype=torch.int32, device="cuda")
    i2 = torch.empty(1, N, dtype=torch.int32, device="cuda")
    res = {"workload": "C2: nnd forward, B=1, 4096 x 4096 (both directions), U[0,1)^3"}
    outs = {}
    old = os.environ.get("PCR_NND_ALGO")
    try:
        for algo in ("grid", "brute"):
            os.environ["PCR_NND_ALGO"] = algo
            call = lambda: nd.nnd_forward_cuda(t1, t2, d1, d2, i1, i2)  # noqa: E731
            res[f"eager_ms_{algo}"] = _events_ms(call, 50)  # incl. the Python wrapper's dispatch
            res[f"gpu_ms_{algo}"] = _graph_ms(call, 50)
            outs[algo] = [x.cpu().numpy() for x in (d1, d2, i1, i2)]
    finally:
        if old is None:
            os.environ.pop("PCR_NND_ALGO", None)
        else:
            os.environ["PCR_NND_ALGO"] = old
    evals = 2.0 * N * N
    res["pair_evals_per_s_brute"] = evals / (res["gpu_ms_brute"] * 1e-3)
    # brute force: 8 flops per pair evaluation (3 sub, 3 mul, 2 add; no FMA: bit-exact form)
    tf = evals * 8 / (res["gpu_ms_brute"] * 1e-3) / 1e12
    res["roofline_brute"] = {"bound": "valu-f32", "achieved": tf, "peak": PEAK_F32_MFMA_TFLOPS,
                             "unit": "TFLOP/s", "frac": tf / PEAK_F32_MFMA_TFLOPS,
                             "note": "one launch of 1 pair: 32 KB of inputs, far from filling "
                                     "256 CUs; 8 flops/pair-eval, no FMA contraction; gpu_ms = "
                                     "device time per call from a graph of 50 calls, eager_ms = "
                                     "one Python call at a time"}
    res["grid_equals_brute"] = all(np.array_equal(a, b) for a, b in zip(outs["grid"], outs["brute"]))
    if with_cpu:
        ref = None
        try:
            sys.path.insert(0, os.path.join(ROOT, "oracle", "_ref"))
            import torch_nndistance_ref as ref  # the reference's my_lib.cpp, compiled here
        except ImportError:
            ref = None
        c1, c2 = torch.from_numpy(x1), torch.from_numpy(x2)
        e1, e2 = torch.zeros(1, N), torch.zeros(1, N)
        j1, j2 = torch.zeros(1, N, dtype=torch.int32), torch.zeros(1, N, dtype=torch.int32)
        reps = 3
        if ref is not None:
            ref.nnd_forward(c1, c2, e1, e2, j1, j2)
            t0 = time.perf_counter()
            for _ in range(reps):
                ref.nnd_forward(c1, c2, e1, e2, j1, j2)
            cpu_ms = (time.perf_counter() - t0) * 1e3 / reps
            kind, got = "reference", [e1.numpy(), e2.numpy(), j1.numpy(), j2.numpy()]
        else:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O
            t0 = time.perf_counter()
            for _ in range(reps):
                got = list(O.nnd_forward(x1, x2))
            cpu_ms = (time.perf_counter() - t0) * 1e3 / reps
            kind = "port"
        res["cpu_baseline"] = {"ms": cpu_ms, "cores": 1, "kind": kind,
                               "sample": "the same 4096 x 4096 forward, "
                                         + ("oracle/_ref torch_nndistance_ref.nnd_forward "
                                            "(reference my_lib.cpp)" if kind == "reference"
                                            else "oracle nnd_forward (C restatement)")}
        res["gpu_vs_cpu_bitexact"] = all(np.array_equal(a, b) for a, b in zip(outs["grid"], got))
        res["speedup_vs_cpu"] = cpu_ms / res["gpu_ms_grid"]
    return res


TRAFFIC_DIR = "profiles"


def _traffic_file():
    """Newest committed PMC traffic summary (profiles/rNN/vMM_pmc_traffic.json)."""
    return _newest("pmc_traffic.json")


# the pair count of the launches the traffic counters are quoted for (set by
# main: tools/pmc_traffic.sh profiles the default 256-pair bench)
_TRAFFIC_PAIRS = {"launch": 256}


def _pmc_traffic(kernel, *more):
    """HBM bytes per launch (fetch + write) of the kernel whose name holds `kernel`
    (and every string of `more`) from the newest committed PMC summary
    (tools/pmc_traffic.sh on this bench, 256 pairs), scaled by the pair ratio
    when this run's launches cover another pair count, or None when absent."""
    f = _traffic_file()
    if f is None:
        return None
    try:
        with open(f) as fh:
            d = json.load(fh)
        ks = d["kernels"]
        prof_pairs = int(d.get("pairs", 256))
    except (OSError, ValueError, KeyError):
        return None
    ratio = _TRAFFIC_PAIRS["launch"] / prof_pairs
    for k, v in ks.items():
        if kernel in k and all(m in k for m in more):
            # the largest launch (RANSAC's gated second round is a near-empty
            # launch of the same kernel; older summaries have the mean only)
            f = v.get("fetch_size_bytes_max", v.get("fetch_size_bytes", 0.0))
            w = v.get("write_size_bytes_max", v.get("write_size_bytes", 0.0))
            return (f + w) * ratio
    return None


def _traffic_source():
    f = _traffic_file()
    if not f:
        return None
    src = os.path.relpath(f, ROOT)
    if _TRAFFIC_PAIRS["launch"] != 256:
        src += f" (256-pair counters scaled {_TRAFFIC_PAIRS['launch']}/256)"
    return src


L2_HIT_CYC = 200        # MI355X_MICROARCH.md: global_load_dword L2-hit latency ~180-225 cycles
CLOCK_GHZ_PEAK = 2.4
WAVES_PER_SIMD = 8      # nng_query<1>: 39 VGPRs -> the 8-wave cap (guide: min(8, 512/alloc))


def grid_walk_replay(q, c, max_ring=3):
    """Host replay of nng_query's ring walk (nnd_grid.hip:186-288) for queries q
    against cloud c: per query the cells probed and points read before its answer
    is certified.  Cell size as nng_bbox (nnd_grid.hip:82-97); hash collisions
    ignored.  A query certifies after the first ring k whose (2k+1)^3 block faces
    lie farther than its true nearest neighbour (scipy cKDTree); past max_ring it
    reads all of c (the fallback scan, 4 loads in flight per round trip).
    Returns per-query dependent round trips (one per probed cell for its slot
    starts + one per point read) in the kernel's slot (cell-sorted) order."""
    from scipy.spatial import cKDTree
    q = q.astype(np.float64)
    c32 = c.astype(np.float32)
    lo, hi = c32.min(0).astype(np.float64), c32.max(0).astype(np.float64)
    e = hi - lo
    m = e.max()
    cell = float(np.float32(0.6 * np.cbrt(np.prod(np.maximum(e, 1e-3 * m)) / len(c))))
    cc = np.floor(c.astype(np.float64) / cell).astype(np.int64)
    key = lambda x, y, z: (x * 1_000_003 + y) * 1_000_033 + z  # noqa: E731
    uk, cnt = np.unique(key(cc[:, 0], cc[:, 1], cc[:, 2]), return_counts=True)
    dstar = cKDTree(c.astype(np.float64)).query(q)[0]
    qc = np.floor(q / cell).astype(np.int64)
    f0 = np.minimum(q - qc * cell, (qc + 1) * cell - q).min(1)
    kdone = np.maximum(np.ceil((dstar - f0) / cell), 0).astype(np.int64)
    trips = np.zeros(len(q))
    for k in range(max_ring + 1):
        sel = np.nonzero(kdone == k)[0]
        if not len(sel):
            continue
        pts = np.zeros(len(sel))
        r = np.arange(-k, k + 1)
        for dx in r:
            for dy in r:
                for dz in r:
                    kk = key(qc[sel, 0] + dx, qc[sel, 1] + dy, qc[sel, 2] + dz)
                    pos = np.clip(np.searchsorted(uk, kk), 0, len(uk) - 1)
                    pts += np.where(uk[pos] == kk, cnt[pos], 0)
        trips[sel] = (2 * k + 1) ** 3 + pts
    far = kdone > max_ring
    trips[far] = 7 ** 3 + len(c) / 4.0
    S = 256
    while S < len(c):
        S <<= 1
    k = ((qc[:, 0] & 1023) | ((qc[:, 1] & 1023) << 10) | ((qc[:, 2] & 1023) << 20)).astype(np.uint64)
    for sh, mul in ((16, 0x85ebca6b), (13, 0xc2b2ae35), (16, None)):  # nng.h nhash (murmur3 fmix32)
        k ^= k >> np.uint64(sh)
        if mul is not None:
            k = (k * np.uint64(mul)) & np.uint64(0xffffffff)
    qh = (k & np.uint64(S - 1)).astype(np.int64)
    return trips[np.argsort(qh, kind="stable")], float(far.mean())


def _chamfer_roofline(prof, P, N, samples):
    """Second roofline line: the a1 Chamfer kernel of the step (nng_query, one
    launch = both directions of all P pairs).  It is bound by the latency of its
    dependent cell walks (the grids are L2-resident), so the bound is a
    probe-latency model: per wave the longest lane's chain of dependent L2 round
    trips (grid_walk_replay on the sampled pairs, both directions) x the L2-hit
    latency, 8 waves per SIMD in flight on 1,024 SIMDs.  frac = model floor /
    measured time.  The algorithmic bytes (each query read once, its (dist, idx)
    written, each grid read once) are kept beside it as hbm_* for reference."""
    ms, n = prof
    if not n:
        return None
    per = ms / n
    S = 256
    while S < N:
        S <<= 1
    nbytes = 2 * P * N * (12 + 8) + 2 * P * (N * 16 + (S + 1) * 4)
    gbs = nbytes / (per * 1e-3) / 1e9
    wave_trips, mean_trips, far = [], [], []
    for qa, ca in samples:
        t, f = grid_walk_replay(qa, ca)
        nw = len(t) // 64
        wave_trips.append(t[:nw * 64].reshape(nw, 64).max(1).mean())
        mean_trips.append(t.mean())
        far.append(f)
    waves = 2 * P * (-(-N // 64))
    trips_w = float(np.mean(wave_trips))
    slots = 1024 * WAVES_PER_SIMD
    floor_ms = -(-waves // slots) * trips_w * L2_HIT_CYC / (CLOCK_GHZ_PEAK * 1e9) * 1e3
    floors = {"l2_latency_ms": floor_ms}
    sq, src = _pmc_sq("nng_query<1>", P)
    if sq and "SQ_INSTS_VALU" in sq:
        f64 = sum(sq.get(c, 0.0) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                             "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))
        floors["valu_issue_ms"] = (2.0 * sq["SQ_INSTS_VALU"] + 2.0 * f64) / 1024 / (CLOCK_GHZ_PEAK * 1e9) * 1e3
        floors["valu_insts_per_launch"] = sq["SQ_INSTS_VALU"]
        floors["sq_source"] = src
    top = max(floors.get("valu_issue_ms", 0.0), floor_ms)
    return {"bound": "l2-latency (dependent probe chain)" if top == floor_ms else "valu-issue",
            "kernel": "nng_query<1> (certified grid 1-NN)",
            "model_floor_ms": top, "floors": floors, "kernel_ms_per_launch": per, "launches": n,
            "frac": top / per,
            "model": {"round_trips_per_query_mean": float(np.mean(mean_trips)),
                      "round_trips_per_wave_max_lane": trips_w, "fallback_fraction": float(np.mean(far)),
                      "l2_hit_cycles": L2_HIT_CYC, "clock_ghz": CLOCK_GHZ_PEAK,
                      "waves_per_launch": waves, "waves_in_flight": slots,
                      "source": f"grid_walk_replay over {len(samples)} sampled (query cloud, grid) "
                                "directions of this step"},
            "hbm_achieved_gbs": gbs, "hbm_peak_gbs": PEAK_HBM_GBS, "hbm_frac": gbs / PEAK_HBM_GBS,
            "traffic": _pmc_traffic("nng_query"), "bytes_per_launch": nbytes}


def _slot_of(c, S):
    """grid.h cell_hash on integer cell coordinates c (..., 3): the low 10 bits of
    each packed, murmur3's 32-bit finaliser, & (S - 1)."""
    k = ((c[..., 0] & 1023) | ((c[..., 1] & 1023) << 10) | ((c[..., 2] & 1023) << 20)).astype(np.uint64)
    for sh, mul in ((16, 0x85ebca6b), (13, 0xc2b2ae35), (16, None)):
        k ^= k >> np.uint64(sh)
        if mul is not None:
            k = (k * np.uint64(mul)) & np.uint64(0xffffffff)
    return ((k * np.uint64(S)) >> np.uint64(32)).astype(np.int64)


def grid_candidates(src, tgt, T, d, slot_num=2):
    """Mean candidates c_bar examined per radius-d grid query of src (through T)
    against tgt: a host replay of grid.h's walk (cells 2.01 d, the <=2x2x2 cells
    of the 1.001 d box that the cell-gap test keeps, each kept cell's hash slot
    walked whole -- points of other cells in the same slot included)."""
    cell = 2.01 * d
    thr = float(np.float32(d * d))
    S = 256
    while S < len(tgt):
        S <<= 1
    S = S // 2 * slot_num  # grid.hip build_grids (RANSAC's grids: 3)
    kt = np.floor(tgt.astype(np.float64) / cell).astype(np.int64)
    slot_cnt = np.bincount(_slot_of(kt, S), minlength=S)
    p = src.astype(np.float64) @ T[:3, :3].T + T[:3, 3]
    lo = np.floor((p - 1.001 * d) / cell).astype(np.int64)
    hi = np.floor((p + 1.001 * d) / cell).astype(np.int64)
    total = np.zeros(p.shape[0])
    for dx in (0, 1):
        for dy in (0, 1):
            for dz in (0, 1):
                c = lo + np.array([dx, dy, dz])
                ok = np.all(c <= hi, axis=1)
                gap = np.maximum(np.maximum(c * cell - p, p - (c + 1) * cell), 0.0)
                ok &= (gap * gap).sum(1) <= thr
                total += np.where(ok, slot_cnt[_slot_of(c, S)], 0)
    return float(total.mean())


# Per 32 x 32 tile and wave, the inner loop of the shipped build's screens
# (tools/isa_loop_mix.py on the gfx950 ISA; one loop trip = 2 row tiles x 16
# column tiles = 32 tiles, D = 32 -> the 1-term screen executes S = 2 k-chunks
# of 16, the f16(x) segment, with the columns' |y|^2 + B as the MFMA's C):
#  featnn_row9<2,16,true> (pass 1): 2 v_mfma_f32_32x32x16_f16, 19.8 VALU per
#    tile (per 32 tiles: 240 v_min3_u32 + 48 v_min + 16 x (v_med3, v_cmp,
#    v_cndmask) + 256 v_mov_b32_dpp -- the C operand's row broadcasts -- + 41
#    other), 1.5 LDS reads, 0.3 s_nop;
#  featnn_row9<2,16,false> (pass 2): the same with the C operand as 4
#    ds_read_b128 per column tile: 11.8 VALU, 3 LDS reads, 0.25 s_nop.
# SIMD issue cycles (MI355X guide, 'vector-instruction ISSUE cost'): an MFMA holds
# vector issue 8 of its 32 cycles, VALU / LDS / s_nop 4 each; the waves of a SIMD
# share that port.  The MFMA pipe needs 2 x 32 = 64 cycles per tile.
SCREEN_TILE_ISSUE = {"mfma": 2 * 8, "valu": 633 / 32 * 4, "lds": 48 / 32 * 4, "s_nop": 10 / 32 * 4}
SCREEN_TILE_ISSUE2 = {"mfma": 2 * 8, "valu": 376 / 32 * 4, "lds": 96 / 32 * 4, "s_nop": 8 / 32 * 4}
SCREEN_TILE_MFMA = 2


def _screen_issue_model(tiles, ms, table, mfma=SCREEN_TILE_MFMA):
    """Floor of a feature screen launch: per tile the larger of its vector-issue
    cycles and the MFMA pipe's (32 cycles per MFMA), on 1,024 SIMDs at 2.4 GHz."""
    issue = sum(table.values())
    pipe = mfma * 32
    cyc = max(issue, pipe)
    floor_ms = tiles * cyc / 1024 / (CLOCK_GHZ_PEAK * 1e9) * 1e3
    return {"issue_cycles_per_tile": issue, "breakdown": table, "tiles_per_launch": tiles,
            "mfma_pipe_cycles_per_tile": pipe,
            "binding": "vector issue" if issue > pipe else "MFMA pipe",
            "floor_ms_at_2p4ghz": floor_ms, "model_frac": floor_ms / ms if ms else None}


def _newest(pattern):
    """Newest committed profiles/rNN/vMM_<pattern> file, or None."""
    import glob
    import re
    best, key = None, None
    for f in glob.glob(os.path.join(ROOT, TRAFFIC_DIR, "r*", "*" + pattern)):
        m = re.search(r"r(\d+)[/\\]v(\d+)_" + re.escape(pattern) + "$", f)
        if m:
            k = (int(m.group(1)), int(m.group(2)))
            if key is None or k > key:
                best, key = f, k
    return best


def _pmc_sq(kernel, pairs):
    """Per-launch SQ instruction counters of `kernel` for a launch over `pairs`
    pairs: tools/pmc_sq.sh on this bench at the same pair count (the newest
    profiles/rNN/vMM_sq_pmc_<P>pairs.json; vMM_sq_pmc.json is the 256-pair
    run), or else the newest counters of another pair count scaled by the
    pair ratio (the sweeps' work is per pair).  Returns (counters, source)."""
    best = None
    for pat, pp in ((f"sq_pmc_{pairs}pairs.json", pairs), ("sq_pmc.json", 256)):
        f = _newest(pat)
        if f is not None:
            best = (f, pp)
            break
    if best is None:
        return None, None
    f, pp = best
    try:
        with open(f) as fh:
            d = json.load(fh)
        ks = d["kernels"]
        pp = int(d.get("pairs", pp))
    except (OSError, ValueError, KeyError):
        return None, None
    for k, v in ks.items():
        if kernel in k:
            c = dict(v.get("counters", v))
            src = os.path.relpath(f, ROOT)
            if pp != pairs:
                c = {n: x * pairs / pp for n, x in c.items()}
                src += f" (scaled {pairs}/{pp} pairs)"
            return c, src
    return None, None


def _sweep_roofline(name, kernel, prof, sweeps, N, cbar, P):
    """Roofline line of a grid-sweep kernel (RANSAC verification a7 / ICP a8).
    Its candidate gathers are served from the pair's LDS copy of the target grid,
    so the bound is VALU issue: the kernel's own executed VALU instructions (PMC
    SQ_INSTS_VALU per launch, tools/pmc_sq.sh) at the SIMD's throughput -- a wave64
    f32 VALU instruction takes 2 cycles of a SIMD-32, an f64 one 4 (the f64 vector
    rate is half the f32 rate) -- on 1,024 SIMDs at 2.4 GHz.  frac = that floor /
    measured time.  SURVEY 8d's algorithmic bytes per sweep of N source points
    (N*12 points + N*c_bar*12 candidate targets + N/8 inlier mask bits) are kept
    beside it, labelled LDS-served."""
    ms, n = prof
    if not n:
        return None
    per = ms / n
    per_sweep = N * 12 + N * cbar * 12 + N / 8
    nbytes = sweeps * per_sweep
    gbs = nbytes / (per * 1e-3) / 1e9
    sq, src = _pmc_sq(kernel, P)
    out = {"bound": "valu-issue", "kernel": kernel, "kernel_ms_per_launch": per, "launches": n,
           "sweeps_per_launch": sweeps, "c_bar": cbar,
           "lds_served": {"algorithmic_bytes_per_launch": nbytes, "achieved_gbs": gbs,
                          "peak_gbs": PEAK_LDS_GBS, "frac": gbs / PEAK_LDS_GBS,
                          "note": f"{name}: candidate gathers read the pair's LDS copy of its "
                                  "target grid; HBM sees the points once per launch.  frac: "
                                  "SURVEY 8d's algorithmic bytes per sweep against the chip's LDS "
                                  "rate (256 CUs x 256 B/clk x 2.4 GHz, MI355X guide 'LDS')"},
           "algorithmic_frac": gbs / PEAK_LDS_GBS,
           "traffic": _pmc_traffic(kernel), "frac": None}
    if sq and "SQ_INSTS_VALU" in sq:
        # the largest launch's counts (`*_max`; RANSAC launches its sweep twice a
        # step, the gated second round nearly empty: the mean would halve the work)
        cnt = lambda c: sq.get(c + "_max", sq.get(c, 0.0))  # noqa: E731
        valu = cnt("SQ_INSTS_VALU")
        f64 = sum(cnt(c) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                     "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))
        cyc = 2.0 * (valu - f64) + 4.0 * f64
        floor_ms = cyc / 1024 / (CLOCK_GHZ_PEAK * 1e9) * 1e3
        lane_ops = valu * 64 + f64 * 64   # f32-equivalent lane operations (f64 = 2)
        out.update({"achieved": lane_ops / (per * 1e-3) / 1e12,
                    "peak": 1024 * 32 * CLOCK_GHZ_PEAK / 1e3, "unit": "T lane-op/s (f32-equivalent VALU)",
                    "frac": floor_ms / per, "model_floor_ms": floor_ms,
                    "valu_insts_per_launch": valu, "valu_f64_insts_per_launch": f64 if f64 else None,
                    "lds_insts_per_launch": cnt("SQ_INSTS_LDS"), "sq_source": src})
    return out


def run_timed(step, steps, warmup, world):
    """W untimed steps, then exactly K steps bracketed by barrier + synchronize;
    returns the max over ranks of the wall time (s) and the last step's result."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = None
    for _ in range(steps):
        out = step()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    return max_over_ranks(time.perf_counter() - t0, world), out


def measure_host_resident(batch, params, pair_ids, steps, warmup, world, total_pairs):
    """SURVEY 8d's end-to-end C4 definition: inputs resident on the HOST (pinned),
    each step = H2D of the rank's xyz + descriptors, the pipeline, the records
    all-gather and their D2H.  Double-buffered: the copy of batch k+1 runs on its
    own HIP stream while batch k computes, so the rate is that of a stream of
    batches (min of PCIe and compute throughput)."""
    from pointcloudregistration_amd.multigpu import gather_records
    from pointcloudregistration_amd.pipeline import PairPipeline
    host = [torch.from_numpy(np.ascontiguousarray(x)).pin_memory()
            for x in (batch.src, batch.tgt, batch.src_feat, batch.tgt_feat)]
    bufs = [[torch.empty(h.shape, dtype=h.dtype, device="cuda") for h in host] for _ in range(2)]
    pipes = [PairPipeline(*bufs[k], params, pair_ids=pair_ids) for k in range(2)]
    P = batch.src.shape[0]
    rows = -(-total_pairs // world)
    rec_host = torch.empty((rows * world, 40), dtype=torch.float64).pin_memory()
    copy_s = torch.cuda.Stream()
    comp = torch.cuda.current_stream()
    copied = [torch.cuda.Event() for _ in range(2)]
    freed = [torch.cuda.Event() for _ in range(2)]
    h2d_bytes = sum(h.numel() * h.element_size() for h in host)

    def issue_copy(k):
        b = k % 2
        with torch.cuda.stream(copy_s):
            if k >= 2:
                copy_s.wait_event(freed[b])
            for d, h in zip(bufs[b], host):
                d.copy_(h, non_blocking=True)
            copied[b].record(copy_s)

    def run(n):
        issue_copy(0)
        for k in range(n):
            if k + 1 < n:
                issue_copy(k + 1)
            b = k % 2
            comp.wait_event(copied[b])
            pipes[b].run()
            rec = gather_records(pipes[b].records(), world, rows)
            freed[b].record(comp)
            rec_host.copy_(rec, non_blocking=True)

    run(max(warmup, 1))
    torch.cuda.synchronize()
    # the copy alone, for the PCIe rate
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(copy_s):
        e0.record(copy_s)
        for d, h in zip(bufs[0], host):
            d.copy_(h, non_blocking=True)
        e1.record(copy_s)
    torch.cuda.synchronize()
    h2d_ms = e0.elapsed_time(e1)
    wall, _ = run_timed(lambda: run(steps), 1, 0, world)
    return {"value": total_pairs * steps / wall, "unit": "pairs/s",
            "ms_per_step": wall / steps * 1e3, "h2d_bytes_per_step_per_rank": h2d_bytes,
            "h2d_ms_per_step": h2d_ms, "h2d_gbs": h2d_bytes / (h2d_ms * 1e-3) / 1e9,
            "note": "pinned host inputs -> HBM on a copy stream overlapped with the previous "
                    "batch's pipeline; records all-gathered and copied back to the host"}


def measure_s8d_job(batch, params, pair_ids, world, total_pairs, warmup=3, runs=10, chunks=None,
                    lanes=None):
    """SURVEY 8d / BASELINE.md's C4 definition, literally: throughput = the job's
    pairs / the wall time of ONE job from "inputs resident on the host" to "all
    (R,t) gathered on rank 0" (H2D and the RCCL gather included, data generation
    excluded); 3 warm-up jobs, the median of 10.  Each job is a synchronous unit
    (nothing carried over from the previous one).  Inside it the rank's shard is
    split into C chunks copied in order (pinned host -> HBM, one copy stream);
    chunk c's pipeline runs as soon as its copy lands, on the current stream
    (lanes > 1: chunk c on lane c mod L, each lane its own stream and libpcr
    workspace context).  The job then costs about the whole copy (PCIe-bound:
    ~41 us per pair at 56 GB/s) plus the last chunk's pipeline."""
    from pointcloudregistration_amd import _lib
    from pointcloudregistration_amd.multigpu import gather_records
    from pointcloudregistration_amd.pipeline import PairPipeline
    P = batch.src.shape[0]
    # 5 chunks at 256 pairs: a chunk pipeline costs ~0.94 ms + ~17.5 us per pair
    # against ~41 us per pair of copy, so chunks of ~41+ pairs keep up with
    # their copies and the smaller last chunk shortens the tail (measured, one
    # box: C = 4 19,919-20,075, 5 20,224-20,496, 6 20,344-20,527, 7 19,485
    # pairs/s; gpurun_out/s8d)
    C = chunks or (5 if P >= 128 else (2 if P >= 32 else 1))
    C = max(1, min(C, P))
    L = max(1, min(lanes or 1, C, 4))
    bounds = [P * c // C for c in range(C + 1)]
    hosts, devs, pipes = [], [], []
    for c in range(C):
        a, b = bounds[c], bounds[c + 1]
        h = [torch.from_numpy(np.ascontiguousarray(x[a:b])).pin_memory()
             for x in (batch.src, batch.tgt, batch.src_feat, batch.tgt_feat)]
        d = [torch.empty(t.shape, dtype=t.dtype, device="cuda") for t in h]
        hosts.append(h)
        devs.append(d)
        pipes.append(PairPipeline(*d, params, pair_ids=pair_ids[a:b], context=c % L))
    rows = -(-total_pairs // world)
    rec_host = torch.empty((rows * world, 40), dtype=torch.float64).pin_memory()
    rec_dev = torch.empty((P, 40), dtype=torch.float64, device="cuda")
    # the copies on a high-priority stream (torch's pool of those): measured
    # (tools/s8d_probe.py) a copy stream that shares a hardware queue with the
    # pipeline's stream serialises the chunk pipelines behind every copy (25.6 vs
    # 13.7 ms per job); lane 0 is the current stream, more lanes measured slower
    # (two 32-pair pipelines in flight: 13.4-16.4 ms, box to box)
    copy_s = torch.cuda.Stream(priority=-1)
    comp = torch.cuda.current_stream()
    lane_s = [comp] + [torch.cuda.Stream() for _ in range(L - 1)]
    copied = [torch.cuda.Event() for _ in range(C)]
    if L > 1:
        _lib.call("pcr_set_concurrency", L)

    def job():
        for s_ in lane_s[1:]:
            s_.wait_stream(comp)
        with torch.cuda.stream(copy_s):
            for c in range(C):
                for d, h in zip(devs[c], hosts[c]):
                    d.copy_(h, non_blocking=True)
                copied[c].record(copy_s)
        for c in range(C):
            s_ = lane_s[c % L]
            s_.wait_event(copied[c])
            with torch.cuda.stream(s_):
                pipes[c].run()
                rec_dev[bounds[c]:bounds[c + 1]].copy_(pipes[c].records())
        for s_ in lane_s[1:]:
            comp.wait_stream(s_)
        rec = gather_records(rec_dev, world, rows)
        rec_host.copy_(rec, non_blocking=True)
        torch.cuda.synchronize()

    try:
        for _ in range(warmup):
            job()
        times = []
        for _ in range(runs):
            barrier(world)
            t0 = time.perf_counter()
            job()
            times.append(max_over_ranks(time.perf_counter() - t0, world))
    finally:
        if L > 1:
            _lib.call("pcr_set_concurrency", 1)
    med = float(np.median(times))
    return {"value": total_pairs / med, "unit": "pairs/s", "ms_per_job": med * 1e3,
            "ms_per_job_min": min(times) * 1e3, "ms_per_job_max": max(times) * 1e3,
            "warmup_jobs": warmup, "timed_jobs": runs, "chunks_per_rank": C, "pipelines_in_flight": L,
            "records": rec_host[:total_pairs].clone(),
            "note": "SURVEY 8d: one job of the whole C4 batch, pinned host inputs -> (R,t) records "
                    "all-gathered and on the host of rank 0; median of 10 after 3 warm-ups; the "
                    "contract's `value` is the HBM-resident rate (inputs already on the GPU)"}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}; launch with "
              f"torchrun --nproc-per-node {args.gpus} or without a launcher", file=sys.stderr)
        sys.exit(2)
    from pointcloudregistration_amd import synth
    from pointcloudregistration_amd.multigpu import gather_records, shard
    from pointcloudregistration_amd.pipeline import default_params

    # the job's `pairs` pairs split over the ranks (strong scaling);
    # every rank generates its own shard on the host
    first, P = shard(args.pairs, world, rank)
    _TRAFFIC_PAIRS["launch"] = P
    if P == 0:
        print(f"bench: rank {rank} has no pairs ({args.pairs} over {world})", file=sys.stderr)
        sys.exit(2)
    N, D = args.points, args.dim
    batch = synth.make_batch(P, n=N, m=N, d=D, base_seed=1000, first_pair=first,
                             feat_noise=args.feat_noise)
    params = default_params(seed=0)
    pair_ids = np.arange(first, first + P, dtype=np.int32)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(batch, params, args.cpu_budget, pair_ids)  # before any GPU call

    rank, world, local = dist_setup()
    from pointcloudregistration_amd import _lib
    from pointcloudregistration_amd.pipeline import PairPipeline
    # --graph: the headline replays the step as one captured HIP graph (eager if
    # the runtime refuses to record a launch); the profiled steps run eagerly
    pipe = PairPipeline(batch.src, batch.tgt, batch.src_feat, batch.tgt_feat, params,
                        pair_ids=pair_ids, graph=args.graph)

    rows = -(-args.pairs // world)   # equal-size record blocks for the all-gather
    S = max(1, min(args.streams, 4, P))
    if S > 1:
        # the shard as S sub-batches, each a pipeline with its own workspace
        # context on its own stream: one sub-batch's latency-bound stages (RANSAC
        # rounds, ICP iterations) overlap another's screens
        _lib.call("pcr_set_concurrency", S)
        cuts = [P * k // S for k in range(S + 1)]
        subs = [PairPipeline(batch.src[a:b], batch.tgt[a:b], batch.src_feat[a:b], batch.tgt_feat[a:b],
                             params, pair_ids=pair_ids[a:b], context=k)
                for k, (a, b) in enumerate(zip(cuts[:-1], cuts[1:]))]
        sub_streams = [torch.cuda.Stream() for _ in range(S)]
        rec_all = torch.empty((P, 40), dtype=torch.float64, device="cuda")

    def step():
        if S == 1:
            pipe.run()
            return gather_records(pipe.records(), world, rows)
        cur = torch.cuda.current_stream()
        for k in range(S):
            sub_streams[k].wait_stream(cur)
            with torch.cuda.stream(sub_streams[k]):
                subs[k].run()
                rec_all[cuts[k]:cuts[k + 1]].copy_(subs[k].records())
        for k in range(S):
            cur.wait_stream(sub_streams[k])
        return gather_records(rec_all, world, rows)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # the headline: K steps with nothing else in the stream
    wall, rec = run_timed(step, args.steps, 0, world)
    # the per-kernel split from K more steps with libpcr's HIP events around the
    # named kernels (the events add their own packets, so these steps are not
    # the headline's)
    graphed = pipe._graph is not None
    pipe.use_graph = False
    _lib.profile_enable(True)
    for pid in range(_lib.PROF_SLOTS):
        _lib.profile_read(pid, reset=True)
    _lib.featnn_rescan_rows(reset=True)
    _lib.featnn_fallback_rows(reset=True)
    pwall, _ = run_timed(step, args.steps, 0, world)
    if S > 1:
        _lib.call("pcr_set_concurrency", 1)
    prof = {name: _lib.profile_read(pid) for name, pid in
            (("feature_screen", _lib.PROF_FEAT_SCREEN), ("nnd_fwd", _lib.PROF_NND_FWD),
             ("ransac_validate", _lib.PROF_RANSAC_VALIDATE), ("ransac_hyp", _lib.PROF_RANSAC_HYP),
             ("icp", _lib.PROF_ICP), ("feat_rescan", _lib.PROF_FEAT_RESCAN),
             ("feat_pack", _lib.PROF_FEAT_PACK), ("nnd_grid_query", _lib.PROF_NND_GRID),
             ("feature_screen2", _lib.PROF_FEAT_SCREEN2), ("feature_screen1b", _lib.PROF_FEAT_SCREEN1B),
             ("feature_screen2b", _lib.PROF_FEAT_SCREEN2B), ("feat_regroup", _lib.PROF_FEAT_REGROUP))}
    _lib.profile_enable(False)
    rescan_rows = _lib.featnn_rescan_rows(reset=True)
    fallback_rows = _lib.featnn_fallback_rows(reset=True)

    # stage split of one extra (untimed) step
    pipe.run(time_stages=True)
    torch.cuda.synchronize()
    stages = dict(zip(("feature_match", "corres+ransac", "icp", "transform", "chamfer"),
                      pipe.stage_ms()))

    # dominant kernel: pass 1 of the feature screen, featnn_row9 (one launch = the
    # source->target row screen of all P pairs).  Algorithmic work:
    # the P*N*M*D MACs of the distance matrix = 2*P*N*M*D flops, which pass 1
    # computes in full; pass 2 re-screens only the target rows J that some
    # source chose (the mutual check), so the screen STAGE (pass 1 + pass 2 +
    # their regroups and 3-term fallbacks) is also reported against the same
    # algorithmic flops.  The 1-term screen executes 16*ceil(D/16) k-steps per
    # tile (the f16 values; the norms come in as the MFMA's C) instead of D.
    ms_tot, launches = prof["feature_screen"]
    per_launch_ms = ms_tot / max(launches, 1)
    ms2_tot, launches2 = prof["feature_screen2"]
    per2_ms = ms2_tot / max(launches2, 1)
    flops_launch = 2.0 * P * N * N * D
    kexec = 16 * (-(-D // 16))
    achieved = flops_launch / (per_launch_ms * 1e-3) / 1e12
    executed = achieved * kexec / D
    nn12 = torch.sort(pipe.nn12, dim=1).values
    jrows = ((nn12[:, 1:] != nn12[:, :-1]).sum(1) + 1).cpu().numpy().astype(np.int64)
    tiles1 = P * (-(-N // 32)) * (-(-N // 32))
    tiles2 = int(sum(-(-int(j) // 32) for j in jrows)) * (-(-N // 32))
    extra_ms = sum(prof[k][0] for k in ("feature_screen1b", "feature_screen2b", "feat_regroup")) / args.steps
    stage_ms = per_launch_ms + per2_ms + extra_ms
    stage_tf = flops_launch / (stage_ms * 1e-3) / 1e12

    recs = rec.cpu().numpy()
    mine = recs[rank * rows:rank * rows + P]
    T_icp = mine[:, 16:32].reshape(P, 4, 4)
    rre, rte = synth.rre_rte(T_icp[:, :3, :3], T_icp[:, :3, 3], batch.R, batch.t)

    # sweep rooflines (a7 RANSAC verification, a8 ICP): sweeps per launch from the
    # kernels' own counters, c_bar from a host replay on 4 sampled pairs
    rr, ir, _, _ = pipe.last
    validated = int(rr.stats[:, 1].sum().item())
    icp_sweeps = int((ir.stats[:, 0] + 1).sum().item())
    samp = list(range(min(4, P)))
    cb_r = float(np.mean([grid_candidates(batch.src[p], batch.tgt[p], mine[p, 0:16].reshape(4, 4),
                                          params.ransac.max_correspondence_distance, 3) for p in samp]))
    cb_i = float(np.mean([grid_candidates(batch.src[p], batch.tgt[p], T_icp[p],
                                          params.icp.max_correspondence_distance) for p in samp]))
    chamfer_samples = []
    for p in samp[:2]:
        al = (batch.src[p].astype(np.float64) @ T_icp[p, :3, :3].T + T_icp[p, :3, 3]).astype(np.float32)
        chamfer_samples += [(al, batch.tgt[p]), (batch.tgt[p], al)]

    total_pairs = args.pairs * args.steps   # every pair of the job, once per step
    out = {
        "metric": "TOF/PC pairs/sec (8192 pts)",
        "value": total_pairs / wall,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32 xyz/features; f64 RANSAC/ICP; 1-term f16 MFMA screen (certified bound), "
                 "f16x3-split MFMA screen for the rows it leaves, f64 exact re-rank",
        "data": f"synthetic: procedural surface pairs, ROPNet-style augmentation, D={D} "
                f"descriptors (noise {args.feat_noise}), generated per rank (seeds 1000+pair)",
        "config": {"workload": "C4: batch of augmented TOF/PC pairs (featNN+RANSAC+ICP+Chamfer)",
                   "pairs_total": args.pairs, "pairs_per_gpu": P, "points": N, "feature_dim": D,
                   "streams_per_gpu": S,
                   "ransac": "d=0.04 mutual n=3 edge0.9 dist0.04 (100000,0.999)",
                   "icp": "d=0.02 (1e-6,1e-6,30)", "parallelism": f"pair-sharded x{world}",
                   "inputs": "resident in HBM (see host_resident for the PCIe-inclusive rate)"},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_F16_MFMA_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / PEAK_F16_MFMA_TFLOPS,
                     "traffic": _pmc_traffic("featnn_row9<", "true>"),
                     "traffic_source": f"{_traffic_source()} (rocprofv3 --pmc FETCH_SIZE, "
                                       "WRITE_SIZE passes of this bench; FETCH_SIZE x2 per the "
                                       "gfx950 note)",
                     "kernel": "featnn_row9<2,16,true> (pass 1: 1-term f16 screen on "
                               "v_mfma_f32_32x32x16_f16 with the operands transposed -- a lane "
                               "holds one row --, the columns' |y|^2 + B as the MFMA's accumulator "
                               "input (2 MFMAs per tile) and a group-min sweep; featnn_regroup9 "
                               "recovers the winning group's column and second value)",
                     "kernel_ms_per_launch": per_launch_ms, "launches": launches,
                     "flops_per_launch": flops_launch,
                     "executed_mfma_tflops": executed,
                     "executed_frac": executed / PEAK_F16_MFMA_TFLOPS,
                     "vs_f32_mfma_peak": achieved / PEAK_F32_MFMA_TFLOPS,
                     "issue_model": _screen_issue_model(tiles1, per_launch_ms, SCREEN_TILE_ISSUE),
                     "pass2": {"kernel": "featnn_row9<2,16,false> (target rows J = unique(nn12), "
                                         "values only)",
                               "kernel_ms_per_launch": per2_ms, "launches": launches2,
                               "j_rows_mean": float(jrows.mean()),
                               "flops_per_launch": 2.0 * float(jrows.sum()) * N * D,
                               "traffic": _pmc_traffic("featnn_row9<", "false>"),
                               "issue_model": _screen_issue_model(tiles2, per2_ms, SCREEN_TILE_ISSUE2)},
                     "screen_stage": {"ms_per_launch": stage_ms, "achieved": stage_tf,
                                      "frac": stage_tf / PEAK_F16_MFMA_TFLOPS,
                                      "parts_ms_per_step": {k: prof[k][0] / args.steps for k in (
                                          "feature_screen", "feature_screen2", "feat_regroup",
                                          "feature_screen1b", "feature_screen2b")},
                                      "note": "pass 1 + pass 2 + their regroups + the 3-term "
                                              "fallback screens against the distance matrix's "
                                              "2*P*N*M*D algorithmic flops"}},
        "roofline_chamfer": _chamfer_roofline(prof["nnd_grid_query"], P, N, chamfer_samples),
        "roofline_ransac": _sweep_roofline("a7 RANSAC verification", "ransac_sweep_kernel",
                                           prof["ransac_validate"], validated, N, cb_r, P),
        "roofline_icp": _sweep_roofline("a8 ICP", "icp_kernel", prof["icp"], icp_sweeps, N, cb_i, P),
        "kernels_ms_per_step": {k: v[0] / args.steps for k, v in prof.items()},
        "profiled_ms_per_step": pwall / args.steps * 1e3,  # the steps kernels_ms_per_step came from
        "step_graph": graphed,  # the headline steps were replays of the captured step
        "featnn_rescan_rows_per_step": [r / args.steps for r in rescan_rows],
        "featnn_fallback_rows_per_step": [r / args.steps for r in fallback_rows],
        "stages_ms": stages,
        "accuracy": {"rre_deg_median": float(np.median(rre)), "rre_deg_max": float(np.max(rre)),
                     "rte_median": float(np.median(rte)), "rte_max": float(np.max(rte)),
                     "ransac_iters_mean": float(mine[:, 37].mean()),
                     "ransac_validations_mean": validated / P,
                     "mutual_corres_mean": float(mine[:, 39].mean())},
    }
    if not args.no_host_resident:
        del pipe
        torch.cuda.empty_cache()
        # the s8d job first: its copy stream must not share a hardware queue with
        # the pipeline's (measured: a job after the host_resident leg's streams
        # took 16.3 ms, first 13.8)
        job = measure_s8d_job(batch, params, pair_ids, world, args.pairs, chunks=args.s8d_chunks,
                              lanes=args.s8d_lanes)
        # the job's records are the headline step's, bit for bit
        job["records_equal_headline"] = bool(np.array_equal(job.pop("records").numpy(),
                                                            recs[:args.pairs]))
        torch.cuda.empty_cache()
        out["host_resident"] = measure_host_resident(batch, params, pair_ids, args.steps,
                                                     args.warmup, world, args.pairs)
        out["s8d_job"] = job
    if world > 1:
        # secondary: weak scaling, `pairs` pairs on EVERY rank
        wfirst = rank * args.pairs
        wb = synth.make_batch(args.pairs, n=N, m=N, d=D, base_seed=1000, first_pair=wfirst,
                              feat_noise=args.feat_noise)
        wpipe = PairPipeline(wb.src, wb.tgt, wb.src_feat, wb.tgt_feat, params,
                             pair_ids=np.arange(wfirst, wfirst + args.pairs, dtype=np.int32))

        def wstep():
            wpipe.run()
            return gather_records(wpipe.records(), world, args.pairs)
        wwall, _ = run_timed(wstep, args.steps, args.warmup, world)
        out["weak_scaling"] = {"value": args.pairs * world * args.steps / wwall,
                               "unit": "pairs/s", "pairs_per_gpu": args.pairs,
                               "ms_per_step": wwall / args.steps * 1e3}
    if cpu is not None:
        cb, Ts = cpu
        out["cpu_baseline"] = cb
        ks = sorted(Ts)
        k = len(ks)
        T_r = mine[ks, 0:16].reshape(k, 4, 4)
        same_r = all(np.array_equal(T_r[i], Ts[p][0]) for i, p in enumerate(ks))
        same_i = all(np.array_equal(T_icp[p], Ts[p][1]) for p in ks)
        d_rre, d_rte = synth.rre_rte(T_icp[ks, :3, :3], T_icp[ks, :3, 3],
                                     np.stack([Ts[p][1][:3, :3] for p in ks]),
                                     np.stack([Ts[p][1][:3, 3] for p in ks]))
        out["accuracy"]["vs_cpu_ref"] = {"pairs": k, "T_ransac_bitexact": bool(same_r),
                                         "T_icp_bitexact": bool(same_i),
                                         "rre_deg_max": float(np.max(d_rre)),
                                         "rte_max": float(np.max(d_rte))}
    if rank == 0 and world == 1 and not args.no_secondary:
        wc = not args.no_cpu_baseline
        out["secondary"] = {"c2_nnd": measure_c2(wc),
                            "a4_lrf": measure_lrf(wc),
                            "a10_ndp_warp": measure_ndp(wc),
                            "f1_fpfh": measure_fpfh(wc),
                            "f4_ndp_opt": measure_ndp_opt(wc),
                            "f2_voxel": measure_voxel(wc),
                            "c3_flow": measure_c3(wc),
                            "c5_flow": measure_c5(wc)}
    if rank == 0:
        print(json.dumps(out))
    if os.environ.get("PCR_DUMP_MAPS"):
        # diagnostics: the library map of this process, to symbolise a crash at exit
        with open("/proc/self/maps") as f, open(os.environ["PCR_DUMP_MAPS"], "w") as g:
            g.write(f.read())
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    _lib.shutdown()   # the library's device objects, before the runtime's teardown


if __name__ == "__main__":
    main()
