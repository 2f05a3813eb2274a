# RANSAC candidates per grid-walk step (PCR_RANSAC_KW 2 / 4 (library) / 6 / 8).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c31
mkdir -p $T
for L in pointcloudregistration_amd/libpcr.so ab/libpcr_rkw2.so ab/libpcr_rkw6.so ab/libpcr_rkw8.so pointcloudregistration_amd/libpcr.so; do
  n=$(basename $L .so)
  PCR_LIB=$L timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --no-host-resident > $T/$n.json 2> $T/$n.err || { tail -5 $T/$n.err; exit 12; }
  python3 -c "import json;d=json.loads(open('$T/$n.json').read().strip().splitlines()[-1]);k=d['kernels_ms_per_step'];print('$n',round(d['ms_per_step'],3),'ransac',round(k['ransac_validate'],3))"
done
echo done
