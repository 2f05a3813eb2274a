#!/usr/bin/env bash
# One parameterised A/B driver for library variants (replaces round 4's
# single-use r04_check*.sh scripts).  Build variants first on the CPU side:
#   tools/build_variant.sh NAME "-DMACRO=..."   -> ab/libpcr_NAME.so
# then on the GPU box:
#   LIBS="pointcloudregistration_amd/libpcr.so ab/libpcr_NAME.so" REPS=2 \
#     bash tools/ab.sh featnn|bench|bench32|custom ["extra args"]
# featnn : tools/featnn_bench.py (mutual path, 256 pairs) per-kernel ms
# bench  : bench.py at 256 pairs (step ms + the kernel slots)
# bench32: bench.py --pairs 32
# custom : CMD="python3 ..." run with PCR_LIB set (output appended)
# Every run has its own time limit; the script stops at the first failure.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
MODE=${1:-featnn}; EXTRA=${2:-}
LIBS=${LIBS:-pointcloudregistration_amd/libpcr.so}
REPS=${REPS:-2}
OUT=gpurun_out/ab_${MODE}
mkdir -p "$OUT"
for i in $(seq 1 "$REPS"); do
  for L in $LIBS; do
    tag=$(basename "$L" .so)
    case $MODE in
      featnn) PCR_LIB=$L timeout -k 10 120 python3 tools/featnn_bench.py --pairs 256 --iters 10 --mode mutual $EXTRA \
                > "$OUT/$tag.$i.json" 2> "$OUT/$tag.$i.err" || exit 3
              python3 -c "import json,sys; d=json.load(open('$OUT/$tag.$i.json')); print('$tag', $i, json.dumps(d['ms']), d['rescan_rows'])" ;;
      bench|bench32)
              P=256; [ "$MODE" = bench32 ] && P=32
              PCR_LIB=$L timeout -k 10 180 python3 bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident $EXTRA \
                > "$OUT/$tag.$i.json" 2> "$OUT/$tag.$i.err" || exit 3
              python3 -c "import json; d=json.load(open('$OUT/$tag.$i.json')); print('$tag', $i, $P, round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()})" ;;
      custom) PCR_LIB=$L timeout -k 10 300 $CMD >> "$OUT/$tag.log" 2>&1 || exit 3
              echo "$tag $i ok" ;;
    esac
  done
done
