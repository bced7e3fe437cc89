#!/bin/bash
# T2T-like pairs at walk chunk sizes 8 / 12 / 16 Ki (16 Ki = the size rule's pick), interleaved.
set -o pipefail
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
OUT=gpurun_out/r03t2tchunk
mkdir -p $OUT
for rep in 1 2; do
  for c in 16384 8192 12288; do
    for pr in "100000000 100000000 7" "20000000 20000000 5"; do
      echo -n "chunk $c rep $rep: " >> $OUT/ab.txt
      SCCG_WALK_CHUNK=$c timeout -k 10 120 python3 $T/bench_pair.py t2t $pr --steps 3 --sha >> $OUT/ab.txt 2>> $OUT/err.txt || exit 1
    done
  done
done
cat $OUT/ab.txt
