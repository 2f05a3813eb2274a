cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_featcorres_gpu.py tests/test_coop_gpu.py -k "featcorres or feature_corres or icp" > gpurun_out/r03v2_new.txt 2>&1; rc=$?
tail -5 gpurun_out/r03v2_new.txt
[ $rc -eq 0 ] || exit $rc
TAG=r03v2 bash tools/gpu_round_check.sh
