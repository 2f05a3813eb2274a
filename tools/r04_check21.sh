# Backward's branch gradients once per workgroup; box query without the
# last-block counter: the NDP suites, f4, C5, the full bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c21
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_ndp_chamfer_gpu.py tests/test_ndp_opt_gpu.py tests/test_ndp_train_gpu.py tests/test_c5_full_gpu.py tests/test_c2p_gpu.py tests/test_ndp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $T/tests.txt
case $rc in 0) ;; *) grep -E "FAILED|Error|error" $T/tests.txt | head -20; exit 11;; esac
timeout -k 10 200 python tools/ndp_opt_bench.py > $T/f4.txt 2>&1 || { tail -20 $T/f4.txt; exit 12; }
tail -1 $T/f4.txt | cut -c1-130
timeout -k 10 200 python tools/c5_run.py > $T/c5.txt 2>&1 || { tail -20 $T/c5.txt; exit 13; }
grep "rep 1" $T/c5.txt | cut -c1-60
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/f4prof -o run -- python3 tools/ndp_opt_bench.py > $T/f4prof.log 2>&1 || exit 14
timeout -k 10 400 python bench.py > $T/bench.json 2> $T/bench.err || { tail -5 $T/bench.err; exit 16; }
python3 -c "import json;d=json.loads(open('$T/bench.json').read().strip().splitlines()[-1]);s=d['secondary'];print('bench',round(d['value']),round(d['ms_per_step'],3),'c2',s['c2_nnd']['gpu_ms_brute'],'f4',s['f4_ndp_opt']['roofline']['frac'],s['f4_ndp_opt']['roofline']['replay_ms'],'c5',s['c5_flow']['ndp_ms'])"
echo done
