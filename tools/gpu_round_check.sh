# Round-end check on the GPU box: the GPU suite, smoke(), the default bench
# line, then (second call: STAGE=prof) the rocprof kernel stats, the PMC
# traffic passes and the small-shard bench lines.  Outputs: gpurun_out/<TAG>_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-rc}
if [ "${STAGE:-tests}" = tests ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/${T}_pytest_gpu.txt 2>&1 || { tail -20 gpurun_out/${T}_pytest_gpu.txt; exit 11; }
  tail -1 gpurun_out/${T}_pytest_gpu.txt
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { cat gpurun_out/${T}_smoke.txt; exit 12; }
  cat gpurun_out/${T}_smoke.txt | grep smoke
  timeout -k 10 420 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 13
  tail -c 300 gpurun_out/${T}_bench.json
else
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/${T}_prof.log 2>&1 || exit 14
  timeout -k 10 700 bash tools/pmc_traffic.sh gpurun_out/${T}_pmc > gpurun_out/${T}_pmc.log 2>&1 || exit 15
  timeout -k 10 700 bash tools/pmc_sq.sh gpurun_out/${T}_sq > gpurun_out/${T}_sq.log 2>&1 || exit 17
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c5prof -o run -- python3 tools/c5_run.py > gpurun_out/${T}_c5prof.log 2>&1 || exit 18
  for P in 32 64; do
    timeout -k 10 200 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > gpurun_out/${T}_bench_${P}pairs.json 2>/dev/null || exit 16
  done
  echo done
fi
