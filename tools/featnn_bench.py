"""Feature-NN (a5) microbenchmark: P pairs of N x D descriptors built like
synth.make_pair's (shared code pool + Gaussian noise), generated on the GPU.
Prints one JSON line with per-kernel times (library event profiler) and the
number of rows sent to the exact rescan."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloudregistration_amd import _lib, registration as reg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=256)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--noise", type=float, default=1.0)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--mode", choices=("full", "mutual"), default="full",
                    help="full: feature_match (dual screen); mutual: feature_correspondences")
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(7)
    pool = int(a.n * 1.45)
    code = torch.randn(a.pairs, pool, a.d, device="cuda", generator=g)
    pi = torch.argsort(torch.rand(a.pairs, pool, device="cuda", generator=g), dim=1)[:, :a.n]
    pj = torch.argsort(torch.rand(a.pairs, pool, device="cuda", generator=g), dim=1)[:, :a.n]
    F = torch.gather(code, 1, pi[..., None].expand(-1, -1, a.d)) + a.noise * torch.randn(
        a.pairs, a.n, a.d, device="cuda", generator=g)
    G = torch.gather(code, 1, pj[..., None].expand(-1, -1, a.d)) + a.noise * torch.randn(
        a.pairs, a.n, a.d, device="cuda", generator=g)
    F, G = F.contiguous(), G.contiguous()
    del code
    run = (lambda: reg.feature_match(F, G)) if a.mode == "full" else \
        (lambda: reg.feature_correspondences(F, G))
    run()
    torch.cuda.synchronize()
    _lib.profile_enable(True)
    for pid in range(_lib.PROF_SLOTS):
        _lib.profile_read(pid, reset=True)
    _lib.featnn_rescan_rows(reset=True)
    _lib.featnn_fallback_rows(reset=True)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(a.iters):
        run()
    ev1.record()
    torch.cuda.synchronize()
    prof = {name: _lib.profile_read(pid)[0] / a.iters for name, pid in
            (("screen", _lib.PROF_FEAT_SCREEN), ("rescan", _lib.PROF_FEAT_RESCAN),
             ("pack", _lib.PROF_FEAT_PACK), ("screen2", _lib.PROF_FEAT_SCREEN2),
             ("screen1b", _lib.PROF_FEAT_SCREEN1B), ("screen2b", _lib.PROF_FEAT_SCREEN2B),
             ("regroup", _lib.PROF_FEAT_REGROUP))}
    rows = _lib.featnn_rescan_rows(reset=True)
    fb = _lib.featnn_fallback_rows(reset=True)
    flops = 2.0 * a.pairs * a.n * a.n * a.d
    print(json.dumps({"pairs": a.pairs, "mode": a.mode,
                      "n": a.n, "d": a.d, "ms_total": ev0.elapsed_time(ev1) / a.iters,
                      "ms": prof, "screen_alg_tflops": flops / prof["screen"] / 1e9,
                      "rescan_rows": [r / a.iters for r in rows],
                      "fallback_rows": [r / a.iters for r in fb]}))


if __name__ == "__main__":
    main()
