# Launch trims (nng_bbox + nng_build + the aligned transform in one launch;
# no per-call ICP barrier memset): the whole -m gpu suite, smoke, then the
# bench at 256 and 32 pairs, head vs new.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/r04c33
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $T/tests.txt
case $rc in 0) ;; *) grep -E "FAILED|Error|error|assert" $T/tests.txt | head -20; exit 11;; esac
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.txt 2>&1 || { tail -20 $T/smoke.txt; exit 12; }
tail -2 $T/smoke.txt
for i in 1 2; do
for v in head new; do
L=""; [ $v = head ] && L=ab/libpcr_head.so
PCR_LIB=${L:-pointcloudregistration_amd/libpcr.so} timeout -k 10 240 python bench.py --pairs 32 --no-host-resident > $T/b32_${v}_$i.json 2> $T/b32_${v}_$i.err || { tail -20 $T/b32_${v}_$i.err; exit 14; }
PCR_LIB=${L:-pointcloudregistration_amd/libpcr.so} timeout -k 10 300 python bench.py --no-host-resident > $T/b256_${v}_$i.json 2> $T/b256_${v}_$i.err || { tail -20 $T/b256_${v}_$i.err; exit 15; }
python -c "import json;a=json.load(open('$T/b32_${v}_$i.json'));b=json.load(open('$T/b256_${v}_$i.json'));print('$v 32p ms',a['ms_per_step'],' 256p ms',b['ms_per_step'],b['value'])"
done
done
echo done
