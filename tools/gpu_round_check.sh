set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/t12.log 2>&1 || exit 11
timeout -k 10 300 python bench.py > gpurun_out/bench12.json 2> gpurun_out/bench12.err || exit 12
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof12 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/prof12.log 2>&1 || exit 13
bash tools/pmc_traffic.sh gpurun_out/pmc12 > gpurun_out/pmc12.log 2>&1 || exit 14
echo done
