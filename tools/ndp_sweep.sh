# C5 NDP replay time under ring caps / lanes per query (tuning of ndp_chamfer.hip)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for R in 0 1 2 3; do for L in 4 8; do
  PCR_NDP_CHAMFER_RINGS=$R PCR_NND_LPQ=$L REPS=1 timeout -k 10 120 python tools/c5_run.py > gpurun_out/sweep_r${R}_l${L}.txt 2>&1 || exit 1
  echo "rings $R lpq $L: $(grep -o 'replay_ms \[[^]]*\]' gpurun_out/sweep_r${R}_l${L}.txt)"
done; done
