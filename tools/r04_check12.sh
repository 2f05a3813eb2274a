# Round 4 GPU check 12: the Chamfer query with the candidate grid in LDS -- the
# -m gpu suite, then the C4 step at 256 / 32 pairs with it on / off (x2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-r04c12}
mkdir -p $T
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
rc=$?
echo "pytest rc $rc"
grep -E "passed|failed|FAILED|Error" $T/tests.txt | tail -15
[ $rc -eq 0 ] || exit 11
for i in 1 2; do for L in on off; do for P in 256 32; do
  if [ $L = off ]; then export PCR_NND_LDSQ=0; else unset PCR_NND_LDSQ; fi
  timeout -k 10 200 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > $T/b_$P.json 2>$T/b.err || { tail -5 $T/b.err; exit 13; }
  python3 -c "
import json; d=json.load(open('$T/b_$P.json')); k=d['kernels_ms_per_step']
print('ldsq $L', $P, round(d['ms_per_step'],3), round(d['profiled_ms_per_step'],3), {x: round(k[x],3) for x in 'ransac_validate icp nnd_grid_query feature_screen'.split()})"
done; done; done
unset PCR_NND_LDSQ
