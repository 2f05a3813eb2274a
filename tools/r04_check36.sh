# Side-stream prep start at the 64- and 128-pair shards (PCR_PREP_AT 0/1/2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c36
mkdir -p $T
for i in 1 2; do
for P in 64 128; do
for A in 0 1 2; do
  f=$T/b${P}_${A}_$i
  PCR_PREP_AT=$A timeout -k 10 300 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > $f.json 2> $f.err || { tail -5 $f.err; exit 12; }
  python3 -c "import json;a=json.loads(open('$f.json').read().strip().splitlines()[-1]);print('pairs $P at $A',round(a['ms_per_step'],3))"
done
done
done
echo done
