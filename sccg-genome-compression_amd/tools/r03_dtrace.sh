#!/bin/bash
# Per-stream kernel timeline of the chr1 reconstruction (tiled decoders on / off).
set -o pipefail
OUT=gpurun_out/r03dtr
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
for e in X=1 SCCG_RL_SCAN=1,SCCG_TOK_SCAN=1; do
  tag=${e//[=,]/_}
  env ${e//,/ } timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/t_$tag -o run -- python3 $T/bench_decomp.py hg 247249719 249250621 1 --steps 3 > $OUT/$tag.json 2> $OUT/$tag.err || exit 1
  TR=$(find $OUT/t_$tag -name '*kernel_trace.csv' | head -n 1)
  python3 $T/trace_streams.py "$TR" --start-kernel k_newlines --n 60 > $OUT/timeline_$tag.txt
  rm -rf $OUT/t_$tag
done
echo done
