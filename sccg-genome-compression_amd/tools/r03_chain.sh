#!/bin/bash
# Chain generations: windowed find-first scans + step skip-ahead.  Walk/chain GPU tests, then the
# T2T-like 100 Mb pair and the synthetic chr22 (trapped chain) A/B vs the previous walk
# (variants/prev), record sha256 checked against the genome manifest by the caller.
set -o pipefail
OUT=gpurun_out/r03chain
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "t2t or chain or trapped or frozen or chr21 or synth or fuzz or seam or genome" > $OUT/tests.out 2>&1 || { tail -30 $OUT/tests.out; exit 1; }
tail -n 1 $OUT/tests.out
for pass in 1 2; do
  for v in head:- prev:variants/prev/libsccg.so; do
    IFS=: read name lib <<< "$v"; [ "$lib" = "-" ] && lib=""
    echo "$name $(SCCG_LIB_PATH=$lib timeout -k 10 120 python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 5 --sha --prof 2>/dev/null)" >> $OUT/res.txt || exit 1
    echo "$name $(SCCG_LIB_PATH=$lib timeout -k 10 120 python3 $T/bench_pair.py hg 49691432 51304566 22 --steps 5 --sha 2>/dev/null)" >> $OUT/res.txt || exit 1
  done
done
cut -c1-400 $OUT/res.txt
echo done
