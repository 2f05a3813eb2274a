# ring-walk variants: parity suites on the new library, then C5 / f4 replay
# times and the C4 nng_query time per library (PCR_LIB=each of $LIBS)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ndp_chamfer_gpu.py \
  tests/test_nnd_gpu.py tests/test_chamfer_gpu.py tests/test_ndp_opt_gpu.py tests/test_c5_full_gpu.py \
  > gpurun_out/ringab_tests.txt 2>&1 || { tail -30 gpurun_out/ringab_tests.txt; exit 2; }
tail -1 gpurun_out/ringab_tests.txt
LIBS="$LIBS" bash tools/c5_ab.sh || exit 3
for L in ${LIBS}; do
  PCR_LIB=$L timeout -k 10 200 python bench.py --pairs 256 --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-host-resident > gpurun_out/ringab.json 2>/dev/null || exit 4
  python3 -c "import json;d=json.load(open('gpurun_out/ringab.json'));print('$L c4', d['value'], d['kernels_ms_per_step']['nnd_grid_query'], d['stages_ms']['chamfer'])"
done
