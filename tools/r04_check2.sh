# Round 4 GPU check 2: the C5 gradient-path A/B, the whole -m gpu suite
# (no -x: every failure listed), then the C4 bench at 256 and 32 pairs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-r04c2}
mkdir -p $T
timeout -k 10 300 python tools/c5_grad_ab.py > $T/c5ab.json 2> $T/c5ab.err || { tail -20 $T/c5ab.err; exit 10; }
python3 -c "
import json;d=json.load(open('$T/c5ab.json'))
for k,v in d.items(): print(k, [round(l['max_rel'],5) for l in v['levels']], round(v['warped_max_abs'],6))"
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
echo "pytest rc $?"
grep -E "passed|failed|FAILED|Error" $T/tests.txt | tail -15
for P in 256 32; do
  timeout -k 10 300 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > $T/bench_${P}.json 2> $T/bench_${P}.err || { tail -5 $T/bench_${P}.err; exit 12; }
  python3 -c "import json;d=json.load(open('$T/bench_${P}.json'));print($P, round(d['value']), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()}, d['featnn_rescan_rows_per_step'])"
done
for P in 256 32; do for SS in 2 4; do
  timeout -k 10 300 python bench.py --pairs $P --streams $SS --no-secondary --no-cpu-baseline --no-host-resident > $T/bench_${P}_s$SS.json 2> $T/bench_${P}_s$SS.err || { tail -5 $T/bench_${P}_s$SS.err; exit 16; }
  python3 -c "import json;d=json.load(open('$T/bench_${P}_s$SS.json'));print('streams $SS', $P, round(d['value']), round(d['ms_per_step'],3))"
done; done
if [ -n "$STALL" ]; then
  bash tools/pmc_stall.sh $T/stall > $T/stall.txt 2>&1 || { tail -5 $T/stall.txt; exit 13; }
  tail -3 $T/stall.txt
fi
if [ -f ab/libpcr_gqxy.so ]; then
  TAG=${TAG:-r04c2}/ab LIBS="pointcloudregistration_amd/libpcr.so ab/libpcr_gqxy.so" TESTS="tests/test_coop_gpu.py tests/test_registration_gpu.py" KEYS="ransac_validate icp" bash tools/r04_ab.sh || exit 14
fi
GS="0 2 4 8" bash tools/coop_g_ab.sh > $T/coopg.txt 2>&1 || { cat $T/coopg.txt; exit 15; }
cat $T/coopg.txt
PCR_DUMP_MAPS=$T/maps.txt timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $T/t32 -o run -- python3 bench.py --pairs 32 --steps 3 --warmup 2 --no-secondary --no-cpu-baseline --no-host-resident > $T/t32.log 2>&1
echo "rocprof t32 exit $?"
tail -3 $T/t32.log
