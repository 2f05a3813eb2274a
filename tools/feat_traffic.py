"""Per-step HBM bytes of the feature stage from a tools/pmc_traffic.sh summary
(FETCH_SIZE already doubled for gfx950; bench.py --steps 2 --warmup 1 plus the
profiled pass = `steps` steps).  usage: python tools/feat_traffic.py SUMMARY.json [steps]"""
import json
import sys

d = json.load(open(sys.argv[1]))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 6.0
rows, tot = [], 0.0
for k, v in d["kernels"].items():
    if any(s in k for s in ("feat", "corres_build")):
        b = (v["fetch_size_bytes"] + v["write_size_bytes"]) * v["launches"] / steps / 1e6
        rows.append((b, k[:64], v["launches"] / steps))
        tot += b
for b, k, n in sorted(rows, reverse=True):
    print("%8.1f MB/step  %5.1f launches/step  %s" % (b, n, k))
print("feature stage: %.1f MB per step" % tot)
