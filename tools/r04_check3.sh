# Round 4 GPU check 3: full -m gpu suite, featnn pass-1 A/B (group code vs the
# per-tile code), grid-query A/B (xy prefilter), ICP G sweep, 32-pair kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-r04c3}
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
echo "pytest rc $?"
grep -E "passed|failed|FAILED" $T/tests.txt | tail -8
TAG=${TAG:-r04c3}/abf LIBS="pointcloudregistration_amd/libpcr.so ab/libpcr_tilecode.so" TESTS="tests/test_featcorres_gpu.py tests/test_c4_full_gpu.py" KEYS="feature_screen feature_screen2 feat_rescan" bash tools/r04_ab.sh || exit 14
TAG=${TAG:-r04c3}/abg LIBS="pointcloudregistration_amd/libpcr.so ab/libpcr_gqxy.so" TESTS="tests/test_coop_gpu.py tests/test_registration_gpu.py" KEYS="ransac_validate icp" bash tools/r04_ab.sh || exit 15
GS="0 2 4 8" bash tools/coop_g_ab.sh > $T/coopg.txt 2>&1 || { cat $T/coopg.txt; exit 16; }
cat $T/coopg.txt
PCR_DUMP_MAPS=$T/maps.txt timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $T/t32 -o run -- python3 bench.py --pairs 32 --steps 3 --warmup 2 --no-secondary --no-cpu-baseline --no-host-resident > $T/t32.log 2>&1
echo "rocprof t32 exit $?"
tail -3 $T/t32.log
