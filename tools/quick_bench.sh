# Quick A/B on the GPU box: featcorres parity, then the C4 bench at 256 and 32
# pairs without the secondary legs.  Outputs gpurun_out/${TAG}_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-qb}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread ${QB_TESTS:-tests/test_featcorres_gpu.py} > gpurun_out/${T}_tests.txt 2>&1 || { tail -20 gpurun_out/${T}_tests.txt; exit 11; }
tail -1 gpurun_out/${T}_tests.txt
for P in 256 32; do
  timeout -k 10 300 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > gpurun_out/${T}_bench_${P}.json 2> gpurun_out/${T}_bench_${P}.err || { tail -5 gpurun_out/${T}_bench_${P}.err; exit 12; }
  python3 -c "import json;d=json.load(open('gpurun_out/${T}_bench_${P}.json'));print($P, round(d['value']), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()}, {k:round(v,3) for k,v in d['stages_ms'].items()})"
done
