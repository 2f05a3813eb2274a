# Round 4 GPU check 5: the whole -m gpu suite on the new default library (cheaper
# grid-query setup, ICP sums in quanta, Horn's relative stop), A/B timing against
# the committed code (ab/libpcr_base.so), the ICP phase split, the 32-pair trace
# (csv stats), and whether a torch-only program also faults at exit under rocprofv3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-r04c5}
mkdir -p $T
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $T/tests.txt 2>&1
echo "pytest rc $?"
grep -E "passed|failed|FAILED|Error" $T/tests.txt | tail -15
for i in 1 2; do for L in pointcloudregistration_amd/libpcr.so ab/libpcr_base.so; do for P in 256 32; do
  PCR_LIB=$L timeout -k 10 200 python bench.py --pairs $P --no-secondary --no-cpu-baseline --no-host-resident > $T/b.json 2>$T/b.err || { tail -5 $T/b.err; exit 12; }
  python3 -c "
import json; d=json.load(open('$T/b.json')); k=d['kernels_ms_per_step']
print('$(basename $L)', $P, round(d['ms_per_step'],3), {x: round(k[x],3) for x in 'ransac_validate icp nnd_grid_query feature_screen'.split()})"
done; done; done
for P in 32 256; do
  PCR_LIB=ab/libpcr_icpph.so PCR_ICP_TIMING=1 timeout -k 10 120 python tools/icp_bench.py $P > $T/icpph_$P.txt 2>&1 || { tail -5 $T/icpph_$P.txt; exit 15; }
  grep -E "ms/launch|icp timing" $T/icpph_$P.txt
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $T/t32 -o run --output-format csv -- python3 bench.py --pairs 32 --steps 3 --warmup 2 --no-secondary --no-cpu-baseline --no-host-resident > $T/t32.log 2>&1
echo "rocprof t32 exit $?"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $T/torch_only -o run --output-format csv -- python3 -c "import torch; x = torch.ones(1024, device='cuda'); print(float(x.sum()))" > $T/torch_only.log 2>&1
echo "rocprof torch-only exit $?"
tail -4 $T/torch_only.log
