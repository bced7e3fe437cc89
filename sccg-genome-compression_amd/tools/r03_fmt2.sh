#!/bin/bash
# Formatter grid (persistent blocks) A/B on the chr1 reconstruction.
set -o pipefail
OUT=gpurun_out/r03fmt2
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "reconstruct or roundtrip or run_line or golden" > $OUT/tests.out 2>&1 || { tail -30 $OUT/tests.out; exit 1; }
tail -n 1 $OUT/tests.out
for pass in 1 2; do
  for e in X=1 SCCG_FMT_GRID=1024 SCCG_FMT_GRID=2048 SCCG_FMT_GRID=4096 SCCG_FMT_GRID=8192; do
    echo "$e $(env $e timeout -k 10 120 python3 $T/bench_decomp.py hg 247249719 249250621 1 --steps 10 --prof 2>/dev/null)" >> $OUT/res.txt || exit 1
  done
done
echo done
