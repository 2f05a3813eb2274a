# Kernel trace + stats of the feature stage (mutual path, 256 pairs) and the SQ
# counters of its kernels (64 pairs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ftrace
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ftrace/kt -o run -- python3 tools/featnn_bench.py --pairs 256 --iters 3 --mode mutual > gpurun_out/ftrace/kt.log 2>&1 || exit 9
bash tools/featnn_pmc.sh 64 mutual || exit 8
python3 tools/sq_summary.py gpurun_out/pmc_featnn_mutual featnn_ > gpurun_out/pmc_featnn_mutual/summary.json || exit 7
