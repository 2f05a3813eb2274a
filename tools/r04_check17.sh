# Box-path level Chamfer v3 (query-uniform leaf lists): tests, f4 at LPQ 8 / 16 / 4,
# the scan statistics, C5, a kernel profile of the f4 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c17
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_ndp_chamfer_gpu.py tests/test_ndp_opt_gpu.py tests/test_ndp_train_gpu.py tests/test_c5_full_gpu.py tests/test_nnd_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 $T/tests.txt
case $rc in 0) ;; *) grep -E "FAILED|Error|error" $T/tests.txt | head -20; exit 11;; esac
for L in 8 16 4; do
  PCR_NC_LPQ=$L timeout -k 10 200 python tools/ndp_opt_bench.py > $T/f4_lpq$L.txt 2>&1 || { tail -20 $T/f4_lpq$L.txt; exit 12; }
  echo "f4 lpq=$L"; tail -1 $T/f4_lpq$L.txt | cut -c1-130
done
PCR_NC_STATS=1 LEVELS=3 timeout -k 10 200 python tools/ndp_opt_bench.py > $T/f4_stats.txt 2>&1 || { tail -20 $T/f4_stats.txt; exit 12; }
tail -1 $T/f4_stats.txt | cut -c1-600
timeout -k 10 200 python tools/c5_run.py > $T/c5.txt 2>&1 || { tail -20 $T/c5.txt; exit 13; }
grep "rep 1" $T/c5.txt | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/f4prof -o run -- python3 tools/ndp_opt_bench.py > $T/f4prof.log 2>&1 || exit 14
PCR_ROW1_RT=1 PCR_ROW2_RT=1 timeout -k 10 300 python -u -m pytest tests/test_featcorres_gpu.py tests/test_c4_full_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests_rt1.txt 2>&1 || { tail -5 $T/tests_rt1.txt; exit 15; }
tail -1 $T/tests_rt1.txt
for R in "2 2" "2 1" "1 2"; do
  set -- $R
  PCR_ROW1_RT=$1 PCR_ROW2_RT=$2 timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --no-host-resident > $T/bench_rt$1$2.json 2> $T/bench_rt$1$2.err || { tail -5 $T/bench_rt$1$2.err; exit 16; }
  python3 -c "import json;d=json.loads(open('$T/bench_rt$1$2.json').read().strip().splitlines()[-1]);k=d['kernels_ms_per_step'];print('rt $1 $2',round(d['ms_per_step'],3),round(k['feature_screen'],3),round(k['feature_screen2'],3))"
done
echo done
