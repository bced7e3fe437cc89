#!/bin/bash
# Frozen-first start: walk/chain/T2T GPU tests, then the T2T-like 100 Mb pair and chr22 A/B
# (default vs SCCG_NO_FROZEN_FIRST=1), phase clocks of the default on the T2T pair.
set -o pipefail
OUT=gpurun_out/r03ff
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "t2t or chain or trapped or frozen or chr21 or synth or fuzz or seam or genome or params or poor" > $OUT/tests.out 2>&1 || { tail -30 $OUT/tests.out; exit 1; }
tail -n 1 $OUT/tests.out
for pass in 1 2 3; do
  for v in ff:X=1 noff:SCCG_NO_FROZEN_FIRST=1; do
    IFS=: read name e <<< "$v"
    echo "$name $(env $e timeout -k 10 120 python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 5 --sha 2>/dev/null)" >> $OUT/res.txt || exit 1
  done
done
for seed in 3 5; do
  for v in ff:X=1 noff:SCCG_NO_FROZEN_FIRST=1; do
    IFS=: read name e <<< "$v"
    echo "$name $(env $e timeout -k 10 120 python3 $T/bench_pair.py t2t 20000000 20000000 $seed --steps 5 --sha 2>/dev/null)" >> $OUT/res.txt || exit 1
  done
done
cut -c1-300 $OUT/res.txt
SCCG_DEBUG=1 timeout -k 10 120 python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 1 > $OUT/t2t_dbg.json 2> $OUT/t2t_dbg.err || exit 1
echo done
