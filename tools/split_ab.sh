# A/B of the RANSAC split factor on the small shards (bench stage times)
set -o pipefail
mkdir -p gpurun_out
for P in 32 64; do for S in 1 2 4; do
  PCR_RANSAC_SPLIT=$S timeout -k 10 120 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > gpurun_out/split_${P}_${S}.json 2>/dev/null || exit 3
  python -c "import json; d=json.load(open('gpurun_out/split_${P}_${S}.json')); print($P, $S, round(d['ms_per_step'],3), round(d['kernels_ms_per_step']['ransac_validate'],3))"
done; done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_coop_gpu.py tests/test_c2p_gpu.py tests/test_dip_gpu.py tests/test_fpfh_gpu.py tests/test_registration_gpu.py > gpurun_out/split_tests.txt 2>&1 || { tail -20 gpurun_out/split_tests.txt; exit 4; }
tail -1 gpurun_out/split_tests.txt
