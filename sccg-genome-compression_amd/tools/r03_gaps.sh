#!/bin/bash
# Genome bench kernel trace: idle gaps (with the kernels around them) and concurrency.
set -o pipefail
OUT=gpurun_out/r03gaps
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/tg -o run -- python3 bench.py --no-cpu-baseline --no-decomp --no-e2e --no-check --no-prof --steps 3 --warmup 1 > $OUT/genome_trace.json 2> $OUT/genome_trace.err || exit 1
TR=$(find $OUT/tg -name '*kernel_trace.csv' | head -n 1)
MS=$(python3 -c "import json;print(json.loads(open('$OUT/genome_trace.json').read().strip().splitlines()[-1])['ms_per_step'])")
python3 $T/trace_busy.py "$TR" --window-ms $MS > $OUT/busy.txt
python3 $T/trace_gaps.py "$TR" --last-ms $MS --top 25 > $OUT/gaps.txt
python3 $T/trace_streams.py "$TR" --n 400 > $OUT/last_pair_timeline.txt
rm -rf $OUT/tg
echo done
