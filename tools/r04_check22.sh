# Register-direct weight gradients (ndp_wgrad2) vs the LDS-staged kernel, at
# 128 / 256-point chunks: the NDP suites, f4 replays, C5, a profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c22
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_ndp_opt_gpu.py tests/test_ndp_train_gpu.py tests/test_c5_full_gpu.py tests/test_c2p_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $T/tests.txt
case $rc in 0) ;; *) grep -E "FAILED|Error|error|assert" $T/tests.txt | head -20; exit 11;; esac
for V in "0 128" "0 256" "1 128"; do
  set -- $V
  PCR_NDP_WGRAD=$1 PCR_NDP_CHUNK=$2 timeout -k 10 200 python tools/ndp_opt_bench.py > $T/f4_$1_$2.txt 2>&1 || { tail -20 $T/f4_$1_$2.txt; exit 12; }
  echo "f4 lds=$1 chunk=$2"; tail -1 $T/f4_$1_$2.txt | cut -c1-130
done
timeout -k 10 200 python tools/c5_run.py > $T/c5.txt 2>&1 || { tail -20 $T/c5.txt; exit 13; }
grep "rep 1" $T/c5.txt | cut -c1-60
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/f4prof -o run -- python3 tools/ndp_opt_bench.py > $T/f4prof.log 2>&1 || exit 14
echo done
