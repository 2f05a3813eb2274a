# Round 4 GPU check 14: two point tiles per workgroup in the NDP MLP kernels
# (PCR_NDP_PT=2 default vs 1) and the branch-free grid-query update
# (ab/libpcr_old.so = the branchy one): the -m gpu suite, f4 and C4 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-r04c14}
mkdir -p $T
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
rc=$?
echo "pytest rc $rc"
grep -E "passed|failed|FAILED|Error" $T/tests.txt | tail -15
[ $rc -eq 0 ] || exit 11
PCR_NDP_PT=1 timeout -k 10 300 python -u -m pytest tests/test_ndp_train_gpu.py tests/test_ndp_opt_gpu.py tests/test_c5_full_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > $T/tests_pt1.txt 2>&1 || { tail -20 $T/tests_pt1.txt; exit 12; }
tail -1 $T/tests_pt1.txt
for i in 1 2; do for PT in 2 1; do
  PCR_NDP_PT=$PT timeout -k 10 200 python tools/ndp_opt_bench.py > $T/f4.txt 2>&1 || { tail -5 $T/f4.txt; exit 14; }
  echo "PT $PT $(tail -1 $T/f4.txt | cut -c1-120)"
done; done
for i in 1 2; do for L in pointcloudregistration_amd/libpcr.so ab/libpcr_old.so; do for P in 256 32; do
  PCR_LIB=$L timeout -k 10 200 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > $T/b.json 2>$T/b.err || { tail -5 $T/b.err; exit 13; }
  python3 -c "
import json; d=json.load(open('$T/b.json')); k=d['kernels_ms_per_step']
print('$(basename $L)', $P, round(d['ms_per_step'],3), {x: round(k[x],3) for x in 'ransac_validate icp nnd_grid_query'.split()})"
done; done; done
