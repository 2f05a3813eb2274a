#!/usr/bin/env bash
# HBM traffic per kernel from PMC counters, one counter per pass (FETCH_SIZE uses 3
# of the 4 TCC slots, WRITE_SIZE 2), kernel trace only, over a short bench run
# (HBM-resident legs only: the s8d leg's small-chunk cooperative ICP launches make
# the process fault at exit under the profiler).
# Usage on the GPU box: bash tools/pmc_traffic.sh OUTDIR  -> OUTDIR/{fetch,write}/
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
# one ICP launch (the tail hand-off's cooperative launch faults at exit under
# the profiler)
export PCR_ICP_TAIL=0
OUT=${1:-gpurun_out/pmc_traffic}
mkdir -p "$OUT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d "$OUT/$c" -o run --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-host-resident > "$OUT/$c.log" 2>&1
  rc=$?
  echo "pmc $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
