# Round 4 GPU check 8: champion-first RANSAC -- the whole -m gpu suite (bit-exact
# scheduling variants included), its task statistics, the C4 step with the
# champion on / off; f4 with the level Chamfer's ring bounds on / off; the
# Chamfer grid cell factor now that the ring walk skips cells.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-r04c8}
mkdir -p $T
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
rc=$?
echo "pytest rc $rc"
grep -E "passed|failed|FAILED|Error" $T/tests.txt | tail -15
[ $rc -eq 0 ] || exit 11
for P in 256 32; do
  PCR_RANSAC_STATS=1 timeout -k 10 200 python bench.py --pairs $P --steps 1 --warmup 0 --no-secondary --no-cpu-baseline --no-host-resident > $T/rs_$P.json 2> $T/rs_$P.err || { tail -5 $T/rs_$P.err; exit 12; }
  grep "ransac gated" $T/rs_$P.err | tail -2
done
for i in 1 2; do for C in 1 0; do for P in 256 32; do
  PCR_RANSAC_CHAMP=$C timeout -k 10 200 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > $T/b.json 2>$T/b.err || { tail -5 $T/b.err; exit 13; }
  python3 -c "
import json; d=json.load(open('$T/b.json')); k=d['kernels_ms_per_step']
print('champ $C', $P, round(d['ms_per_step'],3), {x: round(k[x],3) for x in 'ransac_validate icp nnd_grid_query feature_screen'.split()})"
done; done; done
for L in pointcloudregistration_amd/libpcr.so ab/libpcr_ncskip.so pointcloudregistration_amd/libpcr.so ab/libpcr_ncskip.so; do
  PCR_LIB=$L timeout -k 10 200 python tools/ndp_opt_bench.py > $T/f4.txt 2>&1 || { tail -5 $T/f4.txt; exit 14; }
  echo "$L $(tail -1 $T/f4.txt | cut -c1-160)"
done
bash tools/nnd_cell_ab.sh > $T/cell.txt 2>&1 || { tail -5 $T/cell.txt; exit 15; }
cat $T/cell.txt
