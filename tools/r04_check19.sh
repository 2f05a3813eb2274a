# LDS-staged box tree for the level Chamfer query; pass 2 at one row tile per
# wave by default: the affected suites, f4 at LPQ 8 / 16, C5, one bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c19
mkdir -p $T
timeout -k 10 500 python -u -m pytest tests/test_ndp_chamfer_gpu.py tests/test_ndp_opt_gpu.py tests/test_ndp_train_gpu.py tests/test_c5_full_gpu.py tests/test_featcorres_gpu.py tests/test_c4_full_gpu.py tests/test_registration_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $T/tests.txt
case $rc in 0) ;; *) grep -E "FAILED|Error|error" $T/tests.txt | head -20; exit 11;; esac
for L in 8 16; do
  PCR_NC_LPQ=$L timeout -k 10 200 python tools/ndp_opt_bench.py > $T/f4_lpq$L.txt 2>&1 || { tail -20 $T/f4_lpq$L.txt; exit 12; }
  echo "f4 lpq=$L"; tail -1 $T/f4_lpq$L.txt | cut -c1-130
done
timeout -k 10 200 python tools/c5_run.py > $T/c5.txt 2>&1 || { tail -20 $T/c5.txt; exit 13; }
grep "rep 1" $T/c5.txt | cut -c1-300
timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-resident > $T/bench.json 2> $T/bench.err || { tail -5 $T/bench.err; exit 16; }
python3 -c "import json;d=json.loads(open('$T/bench.json').read().strip().splitlines()[-1]);k=d['kernels_ms_per_step'];s=d['secondary'];print('bench',round(d['value']),round(d['ms_per_step'],3),round(k['feature_screen2'],3),'c2',s['c2_nnd']['gpu_ms_brute'],'f4',s['f4_ndp_opt']['roofline']['frac'],s['f4_ndp_opt']['roofline']['replay_ms'],'c5',s['c5_flow']['ndp_ms'])"
echo done
