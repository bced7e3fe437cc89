#!/bin/bash
# Output-centric formatter + early size readback: reconstruction tests, chr1 A/B against the
# position-centric formatter, and a trace of the new default.
set -o pipefail
OUT=gpurun_out/r03fmt
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "reconstruct or roundtrip or run_line or golden or fuzz or paren or token or dense or cli or synth" > $OUT/tests.out 2>&1 || { tail -30 $OUT/tests.out; exit 1; }
tail -n 1 $OUT/tests.out
for pass in 1 2; do
  for e in X=1 SCCG_FMT_SPAN=1; do
    echo "$e $(env $e timeout -k 10 120 python3 $T/bench_decomp.py hg 247249719 249250621 1 --steps 10 --prof 2>/dev/null)" >> $OUT/res.txt || exit 1
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o run -- python3 $T/bench_decomp.py hg 247249719 249250621 1 --steps 3 > $OUT/trace.json 2> $OUT/trace.err || exit 1
TR=$(find $OUT/t -name '*kernel_trace.csv' | head -n 1)
python3 $T/trace_streams.py "$TR" --start-kernel k_newlines --n 40 > $OUT/timeline.txt
rm -rf $OUT/t
echo done
