# Round evidence for profiles/rNN/ (ROUND=r05 TAG=vN): the -m gpu suite, smoke,
# the default bench line (all legs), the 32 / 64-pair shards, the kernel stats of
# the 256-pair bench, PMC traffic and SQ counters, the C5 / f4 kernel stats.  The
# profiled and PMC runs here use one ICP launch (PCR_ICP_TAIL=0) because the tail
# hand-off's cooperative launch makes the process fault at exit under the profiler
# (the HIP runtime) and nothing may run after a fault in the same
# call; tools/final_profile_tail.sh profiles the shipped path in a call of its own.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
V=${TAG:-v1}; R=${ROUND:-r05}
T=gpurun_out/${R}final_$V
mkdir -p $T
if [ "${PART:-all}" != b ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $T/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $T/pytest_gpu.txt
case $rc in 124|134|137|139) exit 11;; esac
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.txt 2>&1 || { tail -20 $T/smoke.txt; exit 12; }
tail -2 $T/smoke.txt
timeout -k 10 600 python bench.py > $T/bench.json 2> $T/bench.err || { tail -20 $T/bench.err; exit 13; }
python3 -c "import json;d=json.loads(open('$T/bench.json').read().strip().splitlines()[-1]);print('value',round(d['value']),'ms',round(d['ms_per_step'],3))"
for P in 32 64; do
  timeout -k 10 300 python bench.py --pairs $P --no-secondary --no-cpu-baseline > $T/bench_${P}pairs.json 2> $T/bench_$P.err || { tail -5 $T/bench_$P.err; exit 14; }
  python3 -c "import json;d=json.loads(open('$T/bench_${P}pairs.json').read().strip().splitlines()[-1]);print($P,'pairs ms',round(d['ms_per_step'],3))"
done
fi
[ "${PART:-all}" = a ] && exit 0
PCR_ICP_TAIL=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline --no-host-resident > $T/prof.log 2>&1
rc=$?; echo "rocprof stats rc $rc"
case $rc in 124|134|137) exit 15;; esac
bash tools/pmc_traffic.sh $T/traffic > $T/traffic.txt 2>&1; echo "traffic rc $?"
bash tools/pmc_sq.sh $T/sq > $T/sq.txt 2>&1; echo "sq rc $?"
[ "${F4:-1}" = 0 ] && exit 0
TAG=${R}final_${V}_f4 bash tools/gpu_f4_prof.sh > $T/f4.txt 2>&1; echo "f4 prof rc $?"
tail -3 $T/f4.txt
