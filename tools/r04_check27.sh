# Rescan slices per (pair, direction) at 256 pairs: 4 (library) / 8 / 16 / 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c27
mkdir -p $T
PCR_RESCAN_DEBUG=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-secondary --no-cpu-baseline --no-host-resident > $T/dbg.json 2> $T/dbg.err || { tail -5 $T/dbg.err; exit 11; }
grep "rescan dir" $T/dbg.err | head -4
for S in 4 8 16 2 4; do
  PCR_RESCAN_S=$S timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --no-host-resident > $T/b$S.json 2> $T/b$S.err || { tail -5 $T/b$S.err; exit 12; }
  python3 -c "import json;d=json.loads(open('$T/b$S.json').read().strip().splitlines()[-1]);k=d['kernels_ms_per_step'];print('S=$S',round(d['ms_per_step'],3),'rescan',round(k['feat_rescan'],3))"
done
PCR_RESCAN_S=16 timeout -k 10 300 python -u -m pytest tests/test_featcorres_gpu.py tests/test_c4_full_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/tests.txt 2>&1
rc=$?; echo "pytest S=16 rc $rc"; tail -1 $T/tests.txt
echo done
