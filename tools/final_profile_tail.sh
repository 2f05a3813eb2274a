# The shipped path under the profiler: kernel trace + stats of the default
# bench (ICP tail hand-off on).  The process faults at exit after the
# profiler's finalisation (the HIP runtime's teardown of a process that made a
# cooperative launch): the CSVs are complete before that, so
# rc 139 is recorded and accepted here.  Run it as the LAST GPU step of its
# gpurun call (nothing may follow a fault in the same call).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
V=${TAG:-v1}; R=${ROUND:-r05}
T=gpurun_out/${R}final_${V}_tail
mkdir -p $T
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline --no-host-resident > $T/prof.log 2>&1
rc=$?; echo "rocprof stats (tail on) rc $rc"
find $T/prof -name "*kernel_stats.csv" | head -1 | xargs -r head -12
exit 0
