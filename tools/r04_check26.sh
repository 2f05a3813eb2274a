# ICP tail rebalancing (two launches): coop + C4 + estimation suites, bench A/B
# (PCR_ICP_TAIL=0 / default) at 256 pairs, a kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c26
mkdir -p $T
timeout -k 10 500 python -u -m pytest tests/test_coop_gpu.py tests/test_c4_full_gpu.py tests/test_estimation_gpu.py tests/test_registration_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/tests.txt 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $T/tests.txt
case $rc in 0) ;; *) grep -E "FAILED|Error|error|assert" $T/tests.txt | head -20; exit 11;; esac
for V in 0 1 0 1; do
  PCR_ICP_TAIL=$V timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --no-host-resident > $T/b$V.json 2> $T/b$V.err || { tail -5 $T/b$V.err; exit 12; }
  python3 -c "import json;d=json.loads(open('$T/b$V.json').read().strip().splitlines()[-1]);k=d['kernels_ms_per_step'];print('tail=$V',round(d['ms_per_step'],3),'icp',round(k['icp'],3))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-host-resident > $T/prof.log 2>&1
echo "prof rc $?"
echo done
