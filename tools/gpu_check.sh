#!/usr/bin/env bash
# GPU-box session: tests -> smoke -> bench -> rocprof.  Each GPU step has its own
# time limit; a crash/abort/timeout (anything but a plain test failure) ends the run.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
R=$(pwd)
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py ${BENCH_ARGS:-}
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run \
       --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline ${BENCH_ARGS:-}
fi
echo done
