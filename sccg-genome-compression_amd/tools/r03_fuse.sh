#!/bin/bash
# Fused reconstruction (token table expanded inside the formatter): reconstruction tests, chr1
# reconstruction A/B fused vs SCCG_DC_UNFUSED=1 (same library), decompression kernel trace; then the
# T2T-like 100 Mb pair's kernel stats.
set -o pipefail
OUT=gpurun_out/r03fuse
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "reconstruct or roundtrip or golden or fuzz or paren or token or dense or run_line or synth" > $OUT/tests.out 2>&1 || { tail -30 $OUT/tests.out; exit 1; }
tail -n 1 $OUT/tests.out
for pass in 1 2 3; do
  for v in fused:X=1 unfused:SCCG_DC_UNFUSED=1; do
    IFS=: read name e <<< "$v"
    echo "$name $(env $e timeout -k 10 120 python3 $T/bench_decomp.py hg 247249719 249250621 1 --steps 10 --prof 2>/dev/null)" >> $OUT/res.txt || exit 1
  done
done
cat $OUT/res.txt | cut -c1-300
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/dtrace -o run -- python3 $T/bench_decomp.py hg 247249719 249250621 1 --steps 5 > $OUT/dtrace.json 2> $OUT/dtrace.err || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t2t -o run -- python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 3 > $OUT/t2t.json 2> $OUT/t2t.err || exit 1
find $OUT/t2t -name '*kernel_trace.csv' -exec mv {} $OUT/t2t_trace.csv \;
echo done
