# A/B of library variants: parity tests of the affected path under each, then the
# C4 bench at 256 and 32 pairs (step and the named kernels), twice, interleaved.
# LIBS="pointcloudregistration_amd/libpcr.so ab/libpcr_X.so" TESTS="tests/..." KEYS="ransac_validate icp"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-ab}
mkdir -p $T
for L in $LIBS; do
  PCR_LIB=$L timeout -k 10 300 python -u -m pytest ${TESTS} -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests_$(basename $L).txt 2>&1 || { echo "tests FAILED under $L"; tail -20 $T/tests_$(basename $L).txt; exit 11; }
  echo "$L: $(tail -1 $T/tests_$(basename $L).txt)"
done
for i in 1 2; do for L in $LIBS; do for P in ${PAIRS:-256 32}; do
  PCR_LIB=$L timeout -k 10 200 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > $T/b.json 2>$T/b.err || { tail -5 $T/b.err; exit 12; }
  python3 -c "
import json; d=json.load(open('$T/b.json')); k=d['kernels_ms_per_step']
print('$(basename $L)', $P, round(d['ms_per_step'],3), {x: round(k[x],3) for x in '${KEYS:-ransac_validate icp}'.split()})"
done; done; done
