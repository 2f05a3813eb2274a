# Round 4 GPU check 13: what bounds the RANSAC / ICP sweeps -- the C4 step with
# the candidate distance in f32 (ab/libpcr_probe.so, a timing probe, NOT exact)
# against the exact build, interleaved, plus SQ counters of the exact build with
# the GPU's busy cycles (GRBM) for the units.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-r04c13}
mkdir -p $T
for i in 1 2; do for L in pointcloudregistration_amd/libpcr.so ab/libpcr_probe.so; do for P in 256 32; do
  PCR_LIB=$L timeout -k 10 200 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > $T/b.json 2>$T/b.err || { tail -5 $T/b.err; exit 13; }
  python3 -c "
import json; d=json.load(open('$T/b.json')); k=d['kernels_ms_per_step']
print('$(basename $L)', $P, round(d['ms_per_step'],3), {x: round(k[x],3) for x in 'ransac_validate icp nnd_grid_query'.split()})"
done; done; done
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-host-resident"
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$T/$name" -o run --output-format csv -- python3 bench.py $ARGS > "$T/$name.log" 2>&1
  echo "pmc $name rc=$?"
}
run a GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS
timeout -s KILL 60 rocprofv3 --list-avail > "$T/avail.txt" 2>&1 || true
B=""
for c in SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_CVT SQ_LDS_BANK_CONFLICT; do
  grep -qw "$c" "$T/avail.txt" && B="$B $c"
done
echo "pass b counters:$B"
[ -n "$B" ] && run b $B
python3 tools/sq_summary.py "$T" ransac_sweep icp_kernel nng_query featnn_row7 > $T/summary.json
cat $T/summary.json
