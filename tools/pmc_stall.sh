#!/usr/bin/env bash
# Where the waves of the dominant kernels spend their cycles (one --pmc pass each,
# kernel trace only): pass a = the disjoint wave-cycle buckets (parked / issue-
# stalled / issuing) and LDS bank conflicts; pass b = the instruction-active
# split.  Per-launch means -> OUTDIR/summary.json.
# Usage on the GPU box: bash tools/pmc_stall.sh OUTDIR [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_stall}
shift || true
ARGS=${*:-"--steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-host-resident"}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv \
    -- python3 bench.py $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  return $rc
}
run a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES || exit 1
run b SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES || exit 1
python3 tools/sq_summary.py "$OUT" featnn_row8 ransac_sweep icp_kernel nng_query featnn_rescan3 > "$OUT/summary.json"
cat "$OUT/summary.json"
