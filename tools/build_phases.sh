#!/usr/bin/env bash
# Debug build of libpcr with the ICP phase clocks compiled in (-DPCR_ICP_PHASES):
# pointcloudregistration_amd/libpcr_phases.so.  Use with PCR_LIB=<that path>
# PCR_ICP_TIMING=1 python tools/icp_bench.py ...  (never the product library).
set -euo pipefail
cd "$(dirname "$0")/../pointcloudregistration_amd/csrc"
make -s -j8 >/dev/null
mkdir -p build/phases
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include \
  -DPCR_ICP_PHASES -c icp.hip -o build/phases/icp.hip.o
objs=$(ls build/*.o | grep -v '/icp.hip.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build/phases/icp.hip.o -o ../libpcr_phases.so
echo "built pointcloudregistration_amd/libpcr_phases.so"
