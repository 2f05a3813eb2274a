# The whole -m gpu suite and smoke at HEAD (prep start by batch size), and the
# 64-pair shard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c37
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $T/tests.txt
case $rc in 0) ;; *) grep -E "FAILED|Error|error|assert" $T/tests.txt | head -20; exit 11;; esac
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.txt 2>&1 || { tail -20 $T/smoke.txt; exit 12; }
tail -2 $T/smoke.txt
timeout -k 10 300 python bench.py --pairs 64 --no-secondary --no-cpu-baseline --no-host-resident > $T/b64.json 2> $T/b64.err || { tail -5 $T/b64.err; exit 13; }
python3 -c "import json;a=json.loads(open('$T/b64.json').read().strip().splitlines()[-1]);print('64 pairs',round(a['ms_per_step'],3))"
echo done
