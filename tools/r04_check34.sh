# Pass-2 MFMA/VALU interleave (PCR_ROW_KV2 variants; default 5) A/B: feature screen time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c34
mkdir -p $T
for L in pointcloudregistration_amd/libpcr.so ab/libpcr_kv2_3.so ab/libpcr_kv2_8.so ab/libpcr_kv2_12.so pointcloudregistration_amd/libpcr.so; do
  n=$(basename $L .so)
  PCR_LIB=$L timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --no-host-resident > $T/$n.json 2> $T/$n.err || { tail -5 $T/$n.err; exit 12; }
  python3 -c "import json;d=json.loads(open('$T/$n.json').read().strip().splitlines()[-1]);k=d['kernels_ms_per_step'];print('$n',round(d['ms_per_step'],3),'p1',round(k['feature_screen'],3),'p2',round(k['feature_screen2'],3))"
done
echo done
