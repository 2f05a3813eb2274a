# Round-6 profiles (TAG=vN): the 256-pair bench's kernel stats, PMC traffic and
# SQ counters (one ICP launch: PCR_ICP_TAIL=0).  The 32-pair
# shipped path's kernel stats run in a call of their own (tools/r06_profile32.sh:
# its cooperative ICP launches fault at exit under the profiler).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
V=${TAG:-v1}; T=gpurun_out/r06prof_$V
mkdir -p $T
PCR_ICP_TAIL=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline --no-host-resident > $T/prof.log 2>&1
rc=$?; echo "rocprof stats rc $rc"
case $rc in 0) ;; *) exit 15;; esac
cp $(find $T/prof -name '*kernel_stats.csv' | head -1) $T/kernel_stats.csv
bash tools/pmc_traffic.sh $T/traffic > $T/traffic.txt 2>&1; echo "traffic rc $?"
PAIRS=256 bash tools/pmc_sq.sh $T/sq > $T/sq.txt 2>&1; echo "sq rc $?"
python3 tools/feat_traffic.py $T/traffic/summary.json > $T/feature_traffic.txt 2>&1; echo "feat traffic rc $?"
