# SQ counters of the feature screens, dual (full) and mutual paths, 64 pairs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for M in full mutual; do
  timeout -k 10 120 python3 tools/featnn_bench.py --pairs 256 --iters 3 --mode $M || exit 9
  bash tools/featnn_pmc.sh 64 $M || exit 8
  python3 tools/sq_summary.py gpurun_out/pmc_featnn_$M featnn_ > gpurun_out/pmc_featnn_$M/summary.json || exit 7
done
