# Round 4 GPU check 4: f32-screened grid query A/B (parity + timing), ICP phase
# split at 32 / 256 pairs, the 32-pair kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-r04c4}
mkdir -p $T
TAG=${TAG:-r04c4}/abg LIBS="pointcloudregistration_amd/libpcr.so ab/libpcr_gq32.so" TESTS="tests/test_coop_gpu.py tests/test_registration_gpu.py tests/test_c4_full_gpu.py tests/test_fpfh_gpu.py tests/test_dip_gpu.py" KEYS="ransac_validate icp" bash tools/r04_ab.sh || exit 14
for P in 32 256; do
  PCR_LIB=ab/libpcr_icpph.so PCR_ICP_TIMING=1 timeout -k 10 120 python tools/icp_bench.py $P > $T/icpph_$P.txt 2>&1 || { tail -5 $T/icpph_$P.txt; exit 15; }
  grep -E "ms/launch|icp timing" $T/icpph_$P.txt
done
PCR_DUMP_MAPS=$T/maps.txt timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $T/t32 -o run -- python3 bench.py --pairs 32 --steps 3 --warmup 2 --no-secondary --no-cpu-baseline --no-host-resident > $T/t32.log 2>&1
echo "rocprof t32 exit $?"
tail -3 $T/t32.log
