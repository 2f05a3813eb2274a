# Round 4 GPU check 15: triple-buffered column stream in the row screens
# (PCR_ROW_NBUF=3 default vs ab/libpcr_nbuf2.so) -- suite, C4 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-r04c15}
mkdir -p $T
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
rc=$?
echo "pytest rc $rc"
grep -E "passed|failed|FAILED|Error" $T/tests.txt | tail -15
[ $rc -eq 0 ] || exit 11
for i in 1 2; do for L in pointcloudregistration_amd/libpcr.so ab/libpcr_nbuf2.so; do for P in 256 32; do
  PCR_LIB=$L timeout -k 10 200 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > $T/b.json 2>$T/b.err || { tail -5 $T/b.err; exit 13; }
  python3 -c "
import json; d=json.load(open('$T/b.json')); k=d['kernels_ms_per_step']
print('$(basename $L)', $P, round(d['ms_per_step'],3), {x: round(k[x],3) for x in 'feature_screen feature_screen2 feat_rescan'.split()})"
done; done; done
