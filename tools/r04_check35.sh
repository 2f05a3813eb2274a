# Side-stream prep start (PCR_PREP_AT 0: with the step, 1: after pass 1,
# 2: at pass 1's launch) A/B at 256 and 32 pairs, plus the pipeline tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c35
mkdir -p $T
for A in 1 2; do
  PCR_PREP_AT=$A timeout -k 10 300 python -u -m pytest tests/test_c4_full_gpu.py -x -q --timeout 120 --timeout-method thread > $T/tests_$A.txt 2>&1 || { tail -20 $T/tests_$A.txt; exit 11; }
  tail -1 $T/tests_$A.txt
done
for i in 1 2; do
for A in 0 1 2; do
  PCR_PREP_AT=$A timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --no-host-resident > $T/b256_$A_$i.json 2> $T/b256_${A}_$i.err || { tail -5 $T/b256_${A}_$i.err; exit 12; }
  PCR_PREP_AT=$A timeout -k 10 300 python bench.py --pairs 32 --no-secondary --no-cpu-baseline --no-host-resident > $T/b32_$A_$i.json 2> $T/b32_${A}_$i.err || { tail -5 $T/b32_${A}_$i.err; exit 13; }
  python3 -c "import json;a=json.loads(open('$T/b256_$A_$i.json').read().strip().splitlines()[-1]);b=json.loads(open('$T/b32_$A_$i.json').read().strip().splitlines()[-1]);print('at $A 256p',round(a['ms_per_step'],3),'32p',round(b['ms_per_step'],3))"
done
done
echo done
