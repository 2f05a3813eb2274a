#!/usr/bin/env bash
# SQ instruction counters per kernel over a short bench run (kernel trace only,
# one --pmc pass each): pass a = instruction mix, pass b = the f64 VALU split
# when this rocprofv3 lists those counters.  bench.py's sweep rooflines read the
# committed summary (profiles/rNN/vMM_sq_pmc.json).
# Usage on the GPU box: bash tools/pmc_sq.sh OUTDIR  -> OUTDIR/summary.json
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
# one ICP launch (the tail hand-off's cooperative launch faults at exit under
# the profiler)
export PCR_ICP_TAIL=0
OUT=${1:-gpurun_out/pmc_sq}
PAIRS=${PAIRS:-256}   # the bench's pair count (bench.py reads profiles/rNN/vMM_sq_pmc[_<P>pairs].json)
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv \
    -- python3 bench.py --pairs $PAIRS --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-host-resident > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  return $rc
}
run a SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAVES || exit 1
timeout -s KILL 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
if grep -q SQ_INSTS_VALU_FMA_F64 "$OUT/avail.txt"; then
  run b SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 || exit 1
fi
python3 - "$OUT" "$PAIRS" > "$OUT/summary.json" <<'PY'
import json, subprocess, sys
raw = json.loads(subprocess.check_output([sys.executable, "tools/sq_summary.py", sys.argv[1]]))
print(json.dumps({"note": "tools/pmc_sq.sh: per-launch averages of SQ counters over "
                  f"bench.py --pairs {sys.argv[2]} --steps 2 (wave-level instruction counts, whole chip)",
                  "pairs": int(sys.argv[2]),
                  "kernels": {k: {"counters": v} for k, v in raw.items()}}, indent=1))
PY
cat "$OUT/summary.json" | head -40
