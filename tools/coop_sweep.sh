# workgroups per pair (PCR_COOP_G) for the RANSAC / ICP kernels at a small shard:
# bench lines at --pairs P for each G given (default 2 4 8 and the built-in rule)
set -o pipefail
mkdir -p gpurun_out
P=${PAIRS:-32}
for g in "${@:-auto 2 4 8}"; do
  ( [ "$g" = auto ] || export PCR_COOP_G=$g
    timeout -k 10 200 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > gpurun_out/coop_$g.json 2> gpurun_out/coop_$g.err ) || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/coop_$g.json'))
print('G=$g', round(d['value']), 'pairs/s', round(d['ms_per_step'], 3), 'ms; ransac', round(d['roofline_ransac']['kernel_ms_per_launch'], 3), 'icp', round(d['roofline_icp']['kernel_ms_per_launch'], 3))"
done
