# C4 Chamfer (nng_query) time under lanes per query x grid cell factor on the bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in ${LPQS:-1 2}; do for C in ${CELLS:-0.6}; do
  PCR_NND_LPQ=$L PCR_NND_CELL=$C timeout -k 10 200 python bench.py --pairs 256 --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-host-resident > gpurun_out/lpq_$L_$C.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/lpq_$L_$C.json'));print('lpq $L cell $C', d['value'], d['kernels_ms_per_step']['nnd_grid_query'], d['stages_ms']['chamfer'])"
done; done
