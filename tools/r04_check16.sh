# Box-path level Chamfer: its tests, the NDP / C5 suites, f4 and C5 timings with
# the box path and the grid path, a kernel profile of the f4 bench (box path).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c16
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_ndp_chamfer_gpu.py tests/test_ndp_opt_gpu.py tests/test_ndp_train_gpu.py tests/test_c5_full_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 $T/tests.txt
case $rc in 0) ;; *) grep -E "FAILED|Error|error" $T/tests.txt | head -20; exit 11;; esac
for V in "1 4" "1 8" "1 2" "0 4"; do
  set -- $V
  PCR_NC_BOX=$1 PCR_NC_LPQ=$2 timeout -k 10 200 python tools/ndp_opt_bench.py > $T/f4_box$1_$2.txt 2>&1 || { tail -20 $T/f4_box$1_$2.txt; exit 12; }
  echo "f4 box=$1 lpq=$2"; tail -1 $T/f4_box$1_$2.txt | cut -c1-130
done
PCR_NDP_CHUNK=256 timeout -k 10 200 python tools/ndp_opt_bench.py > $T/f4_chunk256.txt 2>&1 || { tail -20 $T/f4_chunk256.txt; exit 12; }
echo "f4 box=1 lpq=4 chunk=256"; tail -1 $T/f4_chunk256.txt | cut -c1-130
for B in 1 0; do
  PCR_NC_BOX=$B timeout -k 10 200 python tools/c5_run.py > $T/c5_box$B.txt 2>&1 || { tail -20 $T/c5_box$B.txt; exit 13; }
  echo "c5 box=$B"; grep "rep 1" $T/c5_box$B.txt | cut -c1-300
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/f4prof -o run -- python3 tools/ndp_opt_bench.py > $T/f4prof.log 2>&1 || exit 14
echo done
