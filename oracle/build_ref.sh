#!/usr/bin/env bash
# Build recipe for oracle/_ref: compiles the REFERENCE's own CPU nndistance source
# (dip/torch-nndistance/src/my_lib.cpp, read in place under /root/reference, never
# copied) into a Python extension module `torch_nndistance_ref` with plain g++.
#
# TEST INFRASTRUCTURE ONLY: the product never loads anything under oracle/.
# The module is used (a) to generate tests/golden/nnd_*.npz and (b) as the
# "reference" CPU baseline for the nndistance leg of bench.py.
#
# The reference file needs only torch/pybind11 headers + libtorch, which ship in
# this image; no reference build system, no stand-ins.  Output only into oracle/_ref/.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
SRC=/root/reference/dip/torch-nndistance/src/my_lib.cpp
OUT="$HERE/_ref/torch_nndistance_ref$(python3 -c 'import sysconfig;print(sysconfig.get_config_var("EXT_SUFFIX"))')"
mkdir -p "$HERE/_ref"
build_nnd() {
if [ ! -f "$SRC" ]; then
  echo "reference source $SRC absent (expected on the GPU box); keeping prebuilt $OUT" >&2
  return 0
fi
if [ -f "$OUT" ] && [ "$OUT" -nt "$SRC" ] && [ "$OUT" -nt "$0" ]; then return 0; fi
TORCH_DIR=$(python3 -c 'import torch,os;print(os.path.dirname(torch.__file__))')
PYINC=$(python3 -c 'import sysconfig;print(sysconfig.get_paths()["include"])')
PYBIND=$(python3 -c 'import pybind11;print(pybind11.get_include())')
# -O2, default x86-64 ISA (SSE2: no FMA contraction possible), exactly as a
# setuptools CppExtension build of the reference would compile it.
g++ -O2 -std=c++17 -fPIC -shared -w \
  -DTORCH_EXTENSION_NAME=torch_nndistance_ref -DTORCH_API_INCLUDE_EXTENSION_H \
  -D_GLIBCXX_USE_CXX11_ABI=1 \
  -I"$TORCH_DIR/include" -I"$TORCH_DIR/include/torch/csrc/api/include" \
  -I"$PYINC" -I"$PYBIND" \
  "$SRC" -o "$OUT" \
  -L"$TORCH_DIR/lib" -lc10 -ltorch -ltorch_cpu -ltorch_python \
  -Wl,-rpath,"$TORCH_DIR/lib"
echo "built $OUT"
}
build_nnd

# --- KPConv helpers (c2p-net/ngenet/cpp_wrappers), SURVEY 8(f) row f2 -------------
# The reference's grid_subsampling.cpp / neighbors.cpp / cloud.cpp compiled in place
# with its own setup.py flags; oracle/ref_kpconv.cpp (ours) is the C-ABI marshalling
# that replaces the CPython wrapper.cpp files (they do not compile against numpy 2).
KP=/root/reference/c2p-net/ngenet/cpp_wrappers
KPOUT="$HERE/_ref/libref_kpconv.so"
if [ -d "$KP" ]; then
  if [ ! -f "$KPOUT" ] || [ "$HERE/ref_kpconv.cpp" -nt "$KPOUT" ] || [ "$0" -nt "$KPOUT" ]; then
    g++ -O2 -std=c++11 -D_GLIBCXX_USE_CXX11_ABI=0 -fPIC -shared -w \
      -I"$KP/cpp_utils" -I"$KP/cpp_subsampling" -I"$KP/cpp_neighbors" \
      "$HERE/ref_kpconv.cpp" "$KP/cpp_subsampling/grid_subsampling/grid_subsampling.cpp" \
      "$KP/cpp_neighbors/neighbors/neighbors.cpp" "$KP/cpp_utils/cloud/cloud.cpp" \
      -o "$KPOUT"
    echo "built $KPOUT"
  fi
else
  echo "reference KPConv sources absent; keeping prebuilt $KPOUT" >&2
fi

