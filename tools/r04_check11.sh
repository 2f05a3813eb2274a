# Round 4 GPU check 11: fewer fill launches per step (feature max partials, RANSAC
# headers cleared in-kernel, nng per-set flags) -- suite, C4 step, host probe.

set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-r04c11}
mkdir -p $T
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
rc=$?
echo "pytest rc $rc"
grep -E "passed|failed|FAILED|Error" $T/tests.txt | tail -15
[ $rc -eq 0 ] || exit 11
for i in 1 2; do for P in 256 32; do
  timeout -k 10 200 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > $T/b_$P.json 2>$T/b.err || { tail -5 $T/b.err; exit 13; }
  python3 -c "
import json; d=json.load(open('$T/b_$P.json')); k=d['kernels_ms_per_step']
print($P, round(d['ms_per_step'],3), {x: round(k[x],3) for x in 'ransac_validate icp nnd_grid_query feature_screen'.split()})"
done; done
for P in 32 256; do
  PCR_HOST_TIMING=1 timeout -k 10 200 python tools/host_overhead.py $P > $T/host_$P.txt 2>&1 || { tail -5 $T/host_$P.txt; exit 14; }
  cat $T/host_$P.txt
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $T/t32 -o run --output-format csv -- python3 bench.py --pairs 32 --steps 3 --warmup 2 --no-secondary --no-cpu-baseline --no-host-resident > $T/t32.log 2>&1
echo "rocprof t32 exit $? (139 = the cooperative-launch teardown fault, DESIGN 7)"
