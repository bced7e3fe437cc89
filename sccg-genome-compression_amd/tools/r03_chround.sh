#!/bin/bash
# Chain start round (SCCG_CHAIN_ROUND 3 / 5 / 10) on the T2T-like 100 Mb pair and a 20 Mb T2T-like pair.
set -o pipefail
OUT=gpurun_out/r03chround
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
for pass in 1 2; do
  for r in 10 3 5 7; do
    echo "cr$r $(SCCG_CHAIN_ROUND=$r timeout -k 10 120 python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 5 --sha 2>/dev/null)" >> $OUT/res.txt || exit 1
    echo "cr$r $(SCCG_CHAIN_ROUND=$r timeout -k 10 120 python3 $T/bench_pair.py t2t 20000000 20000000 5 --steps 5 --sha 2>/dev/null)" >> $OUT/res.txt || exit 1
  done
done
cut -c1-250 $OUT/res.txt
echo done
