# C4 Chamfer (nng_query) time under grid cell factors (PCR_NND_CELL) on the bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in 0.6 0.4 0.5 0.8 1.0; do
  PCR_NND_CELL=$C timeout -k 10 200 python bench.py --pairs 256 --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-host-resident > gpurun_out/cell_$C.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/cell_$C.json'));print('cell $C', d['kernels_ms_per_step']['nnd_grid_query'], d['stages_ms']['chamfer'])"
done
