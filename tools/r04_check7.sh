# Round 4 GPU check 7: the default bench line (all secondary legs: C2, f4, C5 ...)
# and the ICP workgroups-per-pair sweep at the 32 / 64-pair shards.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-r04c7}
mkdir -p $T
timeout -k 10 600 python bench.py > $T/bench.json 2> $T/bench.err || { tail -20 $T/bench.err; exit 10; }
python3 - <<PY
import json
d = json.loads(open("$T/bench.json").read().strip().splitlines()[-1])
print("value", round(d["value"]), "ms", round(d["ms_per_step"], 3))
for k, v in d.get("secondary", {}).items():
    print(k, json.dumps(v)[:600])
PY
GS="0 2 3 4 8" PAIRS="32 64" bash tools/coop_g_ab.sh > $T/coopg.txt 2>&1 || { cat $T/coopg.txt; exit 15; }
cat $T/coopg.txt
