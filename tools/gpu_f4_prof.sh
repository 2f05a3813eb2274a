# f4 / C5 timings with the fallback list counts, and a kernel profile of the f4
# bench (tools/ndp_opt_bench.py).  Outputs: gpurun_out/<TAG>_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-f4}
timeout -k 10 200 python tools/c5_run.py > gpurun_out/${T}_c5.txt 2>&1 || { tail -20 gpurun_out/${T}_c5.txt; exit 12; }
grep rep gpurun_out/${T}_c5.txt
timeout -k 10 200 python tools/ndp_opt_bench.py > gpurun_out/${T}_f4.txt 2>&1 || { tail -20 gpurun_out/${T}_f4.txt; exit 14; }
tail -2 gpurun_out/${T}_f4.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_f4prof -o run -- python3 tools/ndp_opt_bench.py > gpurun_out/${T}_f4prof.log 2>&1 || exit 13
echo done
