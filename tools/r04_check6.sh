# Round 4 GPU check 6: which part of the bench makes the process fault at exit
# under rocprofv3 (torch alone did not, check 5), and RANSAC's task statistics.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-r04c6}
mkdir -p $T
prof() {  # name, program args...
  local n=$1; shift
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $T/$n -o run --output-format csv -- "$@" > $T/$n.log 2>&1
  echo "$n exit $?"
}
prof load python3 tools/exit_probe.py load
prof nnd python3 tools/exit_probe.py nnd
prof icp32 python3 tools/icp_bench.py 32
PCR_COOP_G=1 prof icp32g1 python3 tools/icp_bench.py 32
prof icp256 python3 tools/icp_bench.py 256
prof b256 python3 bench.py --pairs 256 --steps 2 --warmup 1 --no-secondary --no-cpu-baseline --no-host-resident
for P in 256 32; do
  PCR_RANSAC_STATS=1 timeout -k 10 200 python bench.py --pairs $P --steps 1 --warmup 0 --no-secondary --no-cpu-baseline --no-host-resident > $T/rs_$P.json 2> $T/rs_$P.err || { tail -5 $T/rs_$P.err; exit 12; }
  grep "ransac gated" $T/rs_$P.err | tail -4
done
