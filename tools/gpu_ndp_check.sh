# NDP Chamfer path on the GPU box: its parity tests, the NDP / C5 / nnd suites,
# the C5 flow timings and a kernel profile of it.  Outputs: gpurun_out/<TAG>_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-ndp}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_ndp_chamfer_gpu.py tests/test_ndp_train_gpu.py tests/test_ndp_opt_gpu.py \
  tests/test_c5_full_gpu.py tests/test_nnd_gpu.py tests/test_chamfer_gpu.py tests/test_c2p_gpu.py \
  > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 11; }
tail -3 gpurun_out/${T}_tests.txt
timeout -k 10 200 python tools/c5_run.py > gpurun_out/${T}_c5.txt 2>&1 || { tail -20 gpurun_out/${T}_c5.txt; exit 12; }
grep rep gpurun_out/${T}_c5.txt
timeout -k 10 200 python tools/ndp_opt_bench.py > gpurun_out/${T}_f4.txt 2>&1 || { tail -20 gpurun_out/${T}_f4.txt; exit 14; }
tail -3 gpurun_out/${T}_f4.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c5prof -o run -- python3 tools/c5_run.py > gpurun_out/${T}_c5prof.log 2>&1 || exit 13
echo done
