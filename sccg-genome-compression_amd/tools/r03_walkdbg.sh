#!/bin/bash
# Walk diagnostics: round-1 per-chunk statistics (host first step, so round 1 is reported), phase
# clocks, and the T2T-like 100 Mb pair's rounds.
set -eo pipefail
OUT=gpurun_out/r03w
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
echo "[$(date +%T)] chr21 r1"
SCCG_HOST_FIRST_STEP=1 SCCG_DEBUG=1 SCCG_DEBUG_PHASES=1 timeout -k 10 120 python3 $T/bench_pair.py hg 46944323 48129895 21 --steps 1 > $OUT/chr21_r1.json 2> $OUT/chr21_r1.err
echo "[$(date +%T)] chr1 r1"
SCCG_HOST_FIRST_STEP=1 SCCG_DEBUG=1 SCCG_DEBUG_PHASES=1 timeout -k 10 120 python3 $T/bench_pair.py hg 247249719 249250621 1 --steps 1 > $OUT/chr1_r1.json 2> $OUT/chr1_r1.err
echo "[$(date +%T)] t2t"
timeout -k 10 120 python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 3 > $OUT/t2t.json 2> $OUT/t2t.err
SCCG_DEBUG=1 SCCG_DEBUG_ROUNDS=30 timeout -k 10 180 python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 1 > $OUT/t2t_dbg.json 2> $OUT/t2t_dbg.err
echo "[$(date +%T)] trace t2t"
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 1 > $OUT/trace_t2t.json 2> $OUT/trace.err
TR=$(find $OUT/trace -name '*kernel_trace.csv' | head -n 1)
python3 $T/trace_streams.py "$TR" --n 400 > $OUT/t2t_timeline.txt
rm -rf $OUT/trace
echo done
