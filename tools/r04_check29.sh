# ICP phase split (PCR_ICP_PHASES build, PCR_ICP_TIMING): 32 / 64 / 256 pairs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c29
mkdir -p $T
for P in 32 64 256; do
  PCR_LIB=ab/libpcr_phases.so PCR_ICP_TIMING=1 timeout -k 10 300 python bench.py --pairs $P --steps 2 --warmup 1 --no-secondary --no-cpu-baseline --no-host-resident > $T/b$P.json 2> $T/b$P.err || { tail -5 $T/b$P.err; exit 12; }
  echo "P=$P"; grep "icp timing" $T/b$P.err | tail -2
done
echo done
