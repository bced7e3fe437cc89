#!/bin/bash
# Batched token copies: reconstruction tests, chr1 reconstruction A/B vs the previous commit
# (variants/prev2), then the chr1 compress timeline head (single-block header search) vs the
# library before it (variants/prev).
set -o pipefail
OUT=gpurun_out/r03fill
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "reconstruct or roundtrip or golden or fuzz or paren or token or dense or synth" > $OUT/tests.out 2>&1 || { tail -30 $OUT/tests.out; exit 1; }
tail -n 1 $OUT/tests.out
for pass in 1 2; do
  for v in head:- prev2:variants/prev2/libsccg.so; do
    IFS=: read name lib <<< "$v"; [ "$lib" = "-" ] && lib=""
    echo "$name $(SCCG_LIB_PATH=$lib timeout -k 10 120 python3 $T/bench_decomp.py hg 247249719 249250621 1 --steps 10 --prof 2>/dev/null)" >> $OUT/res.txt || exit 1
  done
done
for v in head:- prev:variants/prev/libsccg.so; do
  IFS=: read name lib <<< "$v"; [ "$lib" = "-" ] && lib=""
  SCCG_LIB_PATH=$lib timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/t_$name -o run -- python3 $T/bench_pair.py hg 247249719 249250621 1 --steps 5 > $OUT/pair_$name.json 2> $OUT/pair_$name.err || exit 1
  TR=$(find $OUT/t_$name -name '*kernel_trace.csv' | head -n 1)
  python3 $T/trace_streams.py "$TR" --start-kernel $([ $name = head ] && echo k_find_header || echo k_first_match) --n 30 > $OUT/timeline_$name.txt
  rm -rf $OUT/t_$name
done
echo done
