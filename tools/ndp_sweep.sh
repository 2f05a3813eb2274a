# C5 / f4 NDP replay times under ring caps / lanes per query (tuning of ndp_chamfer.hip)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for R in ${RINGS:-0 1 2 3}; do for L in ${LPQS:-4 8}; do
  PCR_NDP_CHAMFER_RINGS=$R PCR_NND_LPQ=$L REPS=1 timeout -k 10 120 python tools/c5_run.py > gpurun_out/sweep_r${R}_l${L}.txt 2>&1 || exit 1
  echo "rings $R lpq $L c5: $(grep -o 'replay_ms \[[^]]*\]' gpurun_out/sweep_r${R}_l${L}.txt)"
  PCR_NDP_CHAMFER_RINGS=$R PCR_NND_LPQ=$L timeout -k 10 120 python tools/ndp_opt_bench.py > gpurun_out/sweepf4_r${R}_l${L}.txt 2>&1 || exit 2
  echo "rings $R lpq $L f4: $(grep '^1 ' gpurun_out/sweepf4_r${R}_l${L}.txt | grep -o 'sum [0-9.]*')"
done; done
