#!/bin/bash
# Build a variant of libsccg.so for A/B runs: sccg-genome-compression_amd/tools/ab/build_variant.sh <name> [walk.hip source] [extra hipcc flags...]
# (objects other than walk.hip are the in-tree ones; output abvar/<name>/libsccg.so)
set -eo pipefail
NAME=$1; SRC=${2:-sccg-genome-compression_amd/csrc/walk.hip}; shift 2 || shift $#
PKG=sccg-genome-compression_amd
OUT=abvar/$NAME
mkdir -p $OUT
cp "$SRC" $PKG/csrc/_variant_walk.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -c $PKG/csrc/_variant_walk.hip -o $OUT/walk.o
rm -f $PKG/csrc/_variant_walk.hip
objs=$(ls $PKG/build/*.o | grep -v walk.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/libsccg.so $objs $OUT/walk.o
rm -f $OUT/walk.o
echo built $OUT/libsccg.so
