# Pass-1 / pass-2 row tiles per wave A/B (PCR_ROW1_RT / PCR_ROW2_RT), and SQ
# counters of the f4 kernels (one level) for the box query's issue / wait mix.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c18
mkdir -p $T
PCR_ROW1_RT=1 PCR_ROW2_RT=1 timeout -k 10 300 python -u -m pytest tests/test_featcorres_gpu.py tests/test_c4_full_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests_rt1.txt 2>&1
rc=$?; tail -1 $T/tests_rt1.txt; case $rc in 0) ;; *) tail -20 $T/tests_rt1.txt; exit 15;; esac
for R in "2 2" "2 1" "1 2" "2 2"; do
  set -- $R
  PCR_ROW1_RT=$1 PCR_ROW2_RT=$2 timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --no-host-resident > $T/bench_rt$1$2.json 2> $T/bench_rt$1$2.err || { tail -5 $T/bench_rt$1$2.err; exit 16; }
  python3 -c "import json;d=json.loads(open('$T/bench_rt$1$2.json').read().strip().splitlines()[-1]);k=d['kernels_ms_per_step'];print('rt $1 $2',round(d['ms_per_step'],3),round(k['feature_screen'],3),round(k['feature_screen2'],3))"
done
LEVELS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $T/f4sq -o run --output-format csv -- python3 tools/ndp_opt_bench.py > $T/f4sq.log 2>&1
echo "f4 sq rc $?"
echo done
