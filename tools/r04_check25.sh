# The step as a captured HIP graph: C4 tests (incl. graph == eager), bench A/B
# at 256 / 32 / 64 pairs with and without the graph.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c25
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_c4_full_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $T/tests.txt 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "PASS|FAIL|ERROR" $T/tests.txt | tail -12
case $rc in 0) ;; *) tail -30 $T/tests.txt; exit 11;; esac
for P in 256 32 64; do
  for G in "" "--no-graph"; do
    timeout -k 10 300 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident $G > $T/b$P$G.json 2> $T/b$P$G.err || { tail -5 $T/b$P$G.err; exit 12; }
    python3 -c "import json;d=json.loads(open('$T/b$P$G.json').read().strip().splitlines()[-1]);print('$P','$G',round(d['ms_per_step'],3),'graph',d.get('step_graph'),'prof',round(d['profiled_ms_per_step'],3))"
  done
done
echo done
