# A/B check of a kernel change: the parity tests named in $AB_TESTS (default: the
# registration + nnd + coop suites) and one short bench run's per-kernel times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest ${AB_TESTS:-tests/test_registration_gpu.py tests/test_coop_gpu.py tests/test_c4_full_gpu.py tests/test_nnd_gpu.py tests/test_chamfer_gpu.py tests/test_quality_gpu.py} -q --timeout 200 --timeout-method thread > gpurun_out/ab_test.txt 2>&1; tail -2 gpurun_out/ab_test.txt
timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --no-host-resident > gpurun_out/ab_bench.json 2>gpurun_out/ab_bench.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/ab_bench.json')); print(d['value'], d['ms_per_step']); print('ransac', d['roofline_ransac']['kernel_ms_per_launch'], 'icp', d['roofline_icp']['kernel_ms_per_launch'], 'screen', d['roofline']['kernel_ms_per_launch'], 'chamfer', d['roofline_chamfer'])"
