# Round 4 GPU check: the whole -m gpu suite and smoke, the ICP
# workgroups-per-pair sweep at the 32/64-pair shards (tools/coop_g_ab.sh), and
# the rocprofv3 command whose process crashed at exit in round 3 (bench.py
# --pairs 32 under --kernel-trace), with the library map dumped so any frames
# can be symbolised.  Outputs gpurun_out/${TAG:-r04e}/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-r04e}
mkdir -p $T
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests.txt 2>&1 || { tail -30 $T/tests.txt; exit 11; }
tail -2 $T/tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.txt 2>&1 || { tail -20 $T/smoke.txt; exit 12; }
tail -1 $T/smoke.txt
if [ -n "$COOPG" ]; then
  GS="0 2 4 8" bash tools/coop_g_ab.sh > $T/coopg.txt 2>&1 || { cat $T/coopg.txt; exit 13; }
  cat $T/coopg.txt
fi
PCR_DUMP_MAPS=$T/maps.txt timeout -k 10 240 rocprofv3 --kernel-trace -d $T/t32 -o run -- python3 bench.py --pairs 32 --steps 3 --warmup 2 --no-secondary --no-cpu-baseline --no-host-resident > $T/t32.log 2>&1
echo "rocprof exit $?"
tail -5 $T/t32.log
