# ICP phase split (PCR_ICP_TIMING: shader clocks per phase, mean over pairs) at
# 256 and 32 pairs, and the per-pair ICP iteration counts of one step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c24
mkdir -p $T
for P in 256 32; do
  PCR_ICP_TIMING=1 timeout -k 10 300 python bench.py --pairs $P --steps 3 --warmup 1 --no-secondary --no-cpu-baseline --no-host-resident > $T/b$P.json 2> $T/b$P.err || { tail -5 $T/b$P.err; exit 12; }
  grep "icp timing" $T/b$P.err | tail -2
done
timeout -k 10 300 python tools/icp_iters.py > $T/iters.txt 2>&1 || { tail -5 $T/iters.txt; exit 13; }
cat $T/iters.txt
echo done
