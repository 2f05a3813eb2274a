# one-workgroup subset grid build: NDP Chamfer parity under both builds, then
# C5 / f4 replay times per library (PCR_LIB=each of $LIBS)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ndp_chamfer_gpu.py \
  tests/test_ndp_opt_gpu.py tests/test_c5_full_gpu.py tests/test_ndp_train_gpu.py \
  > gpurun_out/b1_tests.txt 2>&1 || { tail -30 gpurun_out/b1_tests.txt; exit 2; }
tail -1 gpurun_out/b1_tests.txt
PCR_NDP_BUILD3=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_ndp_chamfer_gpu.py > gpurun_out/b1_tests3.txt 2>&1 || { tail -30 gpurun_out/b1_tests3.txt; exit 5; }
tail -1 gpurun_out/b1_tests3.txt
LIBS="$LIBS" bash tools/c5_ab.sh || exit 3
