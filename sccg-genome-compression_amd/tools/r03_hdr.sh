#!/bin/bash
# chr1 compress timeline head (the single-block header search), tree vs previous library.
set -o pipefail
OUT=gpurun_out/r03hdr
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
for v in head:- prev:variants/prev/libsccg.so; do
  IFS=: read name lib <<< "$v"; [ "$lib" = "-" ] && lib=""
  SCCG_LIB_PATH=$lib timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/t_$name -o run -- python3 $T/bench_pair.py hg 247249719 249250621 1 --steps 5 > $OUT/$name.json 2> $OUT/$name.err || exit 1
  TR=$(find $OUT/t_$name -name '*kernel_trace.csv' | head -n 1)
  python3 $T/trace_streams.py "$TR" --start-kernel $([ $name = head ] && echo k_find_header || echo k_first_match) --n 30 > $OUT/timeline_$name.txt
  rm -rf $OUT/t_$name
done
echo done
