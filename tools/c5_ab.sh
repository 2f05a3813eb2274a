# A/B of library variants on the C5 / f4 NDP replay times (PCR_LIB=each of $LIBS)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do for L in ${LIBS}; do
  PCR_LIB=$L REPS=2 timeout -k 10 120 python tools/c5_run.py > gpurun_out/c5ab.txt 2>&1 || exit 3
  echo "$L c5: $(grep 'rep 1' gpurun_out/c5ab.txt | grep -o 'replay_ms \[[^]]*\]')"
  PCR_LIB=$L timeout -k 10 120 python tools/ndp_opt_bench.py > gpurun_out/f4ab.txt 2>&1 || exit 4
  echo "$L f4: $(grep '^1 ' gpurun_out/f4ab.txt | grep -o 'sum.*')"
done; done
