#!/usr/bin/env bash
# Build a libpcr variant with extra compile flags into ab/libpcr_NAME.so (its own
# copy of the sources under /tmp, the in-tree build untouched).  bench.py / tests
# load it with PCR_LIB=ab/libpcr_NAME.so.   Usage: tools/build_variant.sh NAME "-DFLAG=1 ..."
# OLDREV=<git rev> OLDFILES="a.hip b.h": those csrc files as of that revision (A/B
# against the committed code).
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=/tmp/pcr_variant/$NAME
rm -rf "$B"; mkdir -p "$B/pkg/csrc" "$B/include" "$ROOT/ab"
cp -r "$ROOT/pointcloudregistration_amd/csrc/." "$B/pkg/csrc/"
cp "$ROOT/include/"*.h "$B/include/"
for f in ${OLDFILES:-}; do git -C "$ROOT" show "$OLDREV:pointcloudregistration_amd/csrc/$f" > "$B/pkg/csrc/$f"; done
rm -rf "$B/pkg/csrc/build"
make -s -j8 -C "$B/pkg/csrc" OUT="$ROOT/ab/libpcr_$NAME.so" CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-variable -I$B/include $FLAGS"
ls -la "$ROOT/ab/libpcr_$NAME.so"
