set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_coop_gpu.py tests/test_registration_gpu.py tests/test_c4_full_gpu.py tests/test_quality_gpu.py tests/test_c2p_gpu.py tests/test_dip_gpu.py tests/test_fpfh_gpu.py > gpurun_out/rs_test.txt 2>&1 || { tail -30 gpurun_out/rs_test.txt; exit 11; }
tail -2 gpurun_out/rs_test.txt
for P in 256 32; do
timeout -k 10 200 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > gpurun_out/rs_bench_$P.json 2>gpurun_out/rs_bench_$P.err || { tail gpurun_out/rs_bench_$P.err; exit 13; }
python -c "
import json; d=json.load(open('gpurun_out/rs_bench_$P.json')); print($P, d['value'], d['ms_per_step']); print(d['kernels_ms_per_step'])"
done
