"""Per-kernel SQ counters (mean per launch, and `<counter>_max`: the largest
launch) from rocprofv3 --pmc pass directories.
Usage: python3 tools/sq_summary.py OUTDIR [kernel-substring ...]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = sys.argv[1]
keys = sys.argv[2:]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for k, cs in acc.items():
    if keys and not any(s in k for s in keys):
        continue
    res[k[:70]] = {c: sum(v) / len(v) for c, v in sorted(cs.items())}
    res[k[:70]].update({c + "_max": max(v) for c, v in sorted(cs.items())})
print(json.dumps(res, indent=1))
