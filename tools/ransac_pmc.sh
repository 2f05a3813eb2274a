#!/usr/bin/env bash
# PMC passes over a short bench run, reported for the RANSAC / ICP kernels
# (separate --pmc runs, kernel trace only).  Usage: bash tools/ransac_pmc.sh OUT
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export PCR_ICP_TAIL=0  # the cooperative tail launch faults at exit under the profiler
OUT=${1:-gpurun_out/pmc_ransac}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv \
    -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-secondary > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU
run b SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM
