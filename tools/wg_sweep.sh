# featnn screen variants: timing (256 and 32 pairs) + the feature-NN parity tests,
# once per environment setting given as an argument (NAME=VALUE or "default")
set -o pipefail
mkdir -p gpurun_out
for env in "${@:-default}"; do
  tag=${env//[^A-Za-z0-9]/_}
  ( [ "$env" = default ] || export "$env"
    timeout -k 10 120 python tools/featnn_bench.py --pairs 256 --iters 5 > gpurun_out/wg_$tag.json 2>&1 &&
    timeout -k 10 120 python tools/featnn_bench.py --pairs 32 --iters 10 > gpurun_out/wg32_$tag.json 2>&1 &&
    timeout -k 10 300 python -m pytest tests/test_registration_gpu.py tests/test_c4_full_gpu.py -q -k "feature_match or c4" --timeout 200 --timeout-method thread > gpurun_out/wgtest_$tag.txt 2>&1 ) || { tail -5 gpurun_out/wgtest_$tag.txt; exit 1; }
  echo "$env $(tail -1 gpurun_out/wgtest_$tag.txt)"
  grep pairs gpurun_out/wg_$tag.json gpurun_out/wg32_$tag.json
done
