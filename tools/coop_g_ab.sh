# ICP workgroups per pair (PCR_COOP_G) at the 32 / 64-pair shards
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for P in ${PAIRS:-32 64}; do for G in ${GS:-0 4 8 16}; do
  if [ "$G" = 0 ]; then unset PCR_COOP_G; else export PCR_COOP_G=$G; fi
  timeout -k 10 200 python bench.py --pairs $P --steps 10 --warmup 3 --no-secondary --no-cpu-baseline --no-host-resident > gpurun_out/coopg.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/coopg.json').read().strip().splitlines()[-1]);print('pairs $P G $G', round(d['ms_per_step'],3), round(d['kernels_ms_per_step']['icp'],3))"
done; done
