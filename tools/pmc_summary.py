"""Per-kernel average FETCH_SIZE / WRITE_SIZE (bytes per launch) from the two
rocprofv3 --pmc passes of tools/pmc_traffic.sh.  FETCH_SIZE is doubled: on gfx950
it reports half the bytes of 16-B-per-lane streaming reads (MI355X_MICROARCH.md,
HBM section); WRITE_SIZE is taken as is.  Both counters are in KiB.  Also the
largest dispatch's bytes (`*_bytes_max`): a kernel launched more than once per
step with very different sizes (RANSAC's gated second round) is priced by its
big launch, not by the mean with the near-empty one."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = sys.argv[1]
res = defaultdict(dict)
for counter in ("FETCH_SIZE", "WRITE_SIZE"):
    files = glob.glob(os.path.join(out, counter, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        scale = 1024.0 * (2.0 if counter == "FETCH_SIZE" else 1.0)
        res[k][counter.lower() + "_bytes"] = sum(v) / len(v) * scale
        res[k][counter.lower() + "_bytes_max"] = max(v) * scale
        res[k]["launches"] = len(v)
short = {}
for k, v in res.items():
    name = k.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    short[name[:80]] = v
print(json.dumps({"note": "per-launch averages and the largest launch (*_max); FETCH_SIZE x2 "
                          "(gfx950 correction), KiB -> bytes",
                  "kernels": short}, indent=1))
