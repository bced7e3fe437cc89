#!/bin/bash
# Kernel trace of the genome bench (2 contexts) and of the chr21 pair: GPU busy fraction,
# concurrency, per-kernel sums (trace_busy.py) and the chr21 per-stream timeline.
set -o pipefail
OUT=gpurun_out/r03b
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/tg -o run -- python3 bench.py --no-cpu-baseline --no-decomp --no-e2e --no-check --no-prof --steps 3 --warmup 1 > $OUT/genome_trace.json 2> $OUT/genome_trace.err || exit 1
TR=$(find $OUT/tg -name '*kernel_trace.csv' | head -n 1)
MS=$(python3 -c "import json;print(3*json.loads(open('$OUT/genome_trace.json').read().strip().splitlines()[-1])['ms_per_step'])")
python3 $T/trace_busy.py "$TR" --window-ms $MS > $OUT/genome_busy.txt
rm -rf $OUT/tg
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/tp -o run -- python3 $T/bench_pair.py hg 46944323 48129895 21 --steps 3 > $OUT/chr21_trace.json 2> $OUT/chr21_trace.err || exit 1
TR=$(find $OUT/tp -name '*kernel_trace.csv' | head -n 1)
python3 $T/trace_streams.py "$TR" --n 150 > $OUT/chr21_timeline.txt
python3 $T/trace_busy.py "$TR" --window-ms 0.75 > $OUT/chr21_busy.txt
rm -rf $OUT/tp
echo done
