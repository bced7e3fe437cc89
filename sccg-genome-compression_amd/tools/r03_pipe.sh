#!/bin/bash
# Pipelined formatter: reconstruction tests, then chr1 reconstruction A/B: pipe (default) vs one
# block per tile (SCCG_FMT_NOPIPE=1), and pipe with 2 / 4 blocks per CU.
set -o pipefail
OUT=gpurun_out/r03pipe
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "reconstruct or roundtrip or golden or fuzz or paren or token or dense or run_line or synth" > $OUT/tests.out 2>&1 || { tail -30 $OUT/tests.out; exit 1; }
tail -n 1 $OUT/tests.out
for pass in 1 2 3; do
  for v in pipe:X=1 nopipe:SCCG_FMT_NOPIPE=1 bpc2:SCCG_FMT_PIPE_BPC=2 bpc3:SCCG_FMT_PIPE_BPC=3; do
    IFS=: read name e <<< "$v"
    echo "$name $(env $e timeout -k 10 120 python3 $T/bench_decomp.py hg 247249719 249250621 1 --steps 10 --prof 2>/dev/null)" >> $OUT/res.txt || exit 1
  done
done
cut -c1-300 $OUT/res.txt
echo done
