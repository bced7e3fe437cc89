#!/bin/bash
# Single-block kernel widths: the tree (256-thread round tail / scans / strip scans) vs variants
# with each back at 1024 threads, interleaved: genome bench and the chr1 pair.
set -o pipefail
OUT=gpurun_out/r03blk
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
run() { local lib=$1; shift; [ "$lib" = "-" ] && lib=""; env SCCG_LIB_PATH=$lib timeout -k 10 180 python3 "$@" 2>/dev/null | tail -n 1; }
for pass in 1 2 3; do
  for name in head all1024 rt1024 sb1024 scan1024 prev2; do
    lib=variants/$name/libsccg.so; [ $name = head ] && lib=-
    echo "[$(date +%T)] $pass $name"
    echo "$name genome $(run $lib bench.py --no-cpu-baseline --no-decomp --no-e2e --no-check --steps 10)" >> $OUT/res.txt || exit 1
    echo "$name chr1 $(run $lib $T/bench_pair.py hg 247249719 249250621 1 --steps 10)" >> $OUT/res.txt || exit 1
  done
done
echo done
