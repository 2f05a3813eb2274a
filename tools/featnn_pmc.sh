#!/usr/bin/env bash
# PMC passes over the feature-NN microbenchmark (separate --pmc runs, kernel
# trace only).  Usage on the GPU box: bash tools/featnn_pmc.sh [PAIRS]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=${1:-64}
MODE=${2:-full}
OUT=gpurun_out/pmc_featnn_$MODE
mkdir -p "$OUT"
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run \
    --output-format csv -- python3 tools/featnn_bench.py --pairs "$P" --iters 2 --mode "$MODE" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run b SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM
