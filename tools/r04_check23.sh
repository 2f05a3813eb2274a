# The whole -m gpu suite at HEAD (incl. the level Chamfer's small / ragged sizes)
# and smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c23
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $T/tests.txt
case $rc in 0) ;; *) grep -E "FAILED|Error|error|assert" $T/tests.txt | head -20; exit 11;; esac
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.txt 2>&1 || { tail -20 $T/smoke.txt; exit 12; }
tail -2 $T/smoke.txt
echo done
