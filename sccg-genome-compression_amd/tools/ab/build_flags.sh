#!/bin/bash
# Build a variant of libsccg.so with extra compiler flags on every source:
#   sccg-genome-compression_amd/tools/ab/build_flags.sh <name> <flags...>   -> abvar/<name>/libsccg.so
set -eo pipefail
NAME=$1; shift
PKG=sccg-genome-compression_amd
OUT=abvar/$NAME
mkdir -p $OUT/obj
for f in $PKG/csrc/*.hip $PKG/csrc/*.cpp; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -c $f -o $OUT/obj/$(basename $f).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/libsccg.so $OUT/obj/*.o
rm -rf $OUT/obj
echo built $OUT/libsccg.so
