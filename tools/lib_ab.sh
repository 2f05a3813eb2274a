# A/B of library variants on the C4 bench (one kernel's time, $KEY, and the step time)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do for L in ${LIBS}; do for P in 256 32; do
  PCR_LIB=$L timeout -k 10 120 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > gpurun_out/ab_$P.json 2>/dev/null || exit 3
  python -c "import json; d=json.load(open('gpurun_out/ab_$P.json')); print('$L', $P, round(d['ms_per_step'],3), round(d['kernels_ms_per_step']['${KEY:-feat_rescan}'],3))"
done; done; done
