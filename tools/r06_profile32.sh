# the shipped 32-pair path (the 8-GPU shard; tail hand-off on) under
# rocprofv3 --kernel-trace --stats; its cooperative ICP launches make the
# process fault at exit after the profile is written: last
# step of its call
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
V=${TAG:-v1}; T=gpurun_out/r06prof32_$V
mkdir -p $T
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof -o run --output-format csv -- python3 bench.py --pairs 32 --steps 20 --warmup 3 --no-secondary --no-cpu-baseline --no-host-resident > $T/prof.log 2>&1
echo "rocprof 32 rc $?"
f=$(find $T/prof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp $f $T/kernel_stats.csv
exit 0
