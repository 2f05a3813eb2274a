# Iterations per captured NDP graph (1 / 2 / 4): f4 replays, C5 wall; the NDP
# suites; a kernel profile of the f4 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c20
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_ndp_opt_gpu.py tests/test_ndp_train_gpu.py tests/test_c5_full_gpu.py tests/test_c2p_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $T/tests.txt
case $rc in 0) ;; *) grep -E "FAILED|Error|error" $T/tests.txt | head -20; exit 11;; esac
for S in 1 2 4; do
  PCR_NDP_GRAPH_STEPS=$S timeout -k 10 200 python tools/ndp_opt_bench.py > $T/f4_s$S.txt 2>&1 || { tail -20 $T/f4_s$S.txt; exit 12; }
  echo "f4 steps=$S"; tail -1 $T/f4_s$S.txt | cut -c1-130
  PCR_NDP_GRAPH_STEPS=$S timeout -k 10 200 python tools/c5_run.py > $T/c5_s$S.txt 2>&1 || { tail -20 $T/c5_s$S.txt; exit 13; }
  echo "c5 steps=$S"; grep "rep 1" $T/c5_s$S.txt | cut -c1-60
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/f4prof -o run -- python3 tools/ndp_opt_bench.py > $T/f4prof.log 2>&1 || exit 14
echo done
