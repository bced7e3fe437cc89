#!/bin/bash
# The per-pair floor on a small chromosome (chr21-sized pair): phase clocks, a kernel timeline per
# stream, and the end-to-end (files) path on the chr1 pair.
set -eo pipefail
OUT=gpurun_out/r03f
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
echo "[$(date +%T)] gpu tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.out 2>&1
echo "[$(date +%T)] cli tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_cli.py -x -q --timeout 120 --timeout-method thread > $OUT/cli_tests.out 2>&1
echo "[$(date +%T)] pair"
timeout -k 10 120 python3 $T/bench_pair.py hg 46944323 48129895 21 --steps 10 > $OUT/chr21_pair.json 2> $OUT/chr21_pair.err
SCCG_DEBUG=1 timeout -k 10 120 python3 $T/bench_pair.py hg 46944323 48129895 21 --steps 2 > $OUT/chr21_dbg.json 2> $OUT/chr21_dbg.err
echo "[$(date +%T)] trace"
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $T/bench_pair.py hg 46944323 48129895 21 --steps 3 > $OUT/trace_pair.json 2> $OUT/trace.err
TR=$(find $OUT/trace -name '*kernel_trace.csv' | head -n 1)
python3 $T/trace_streams.py "$TR" --n 120 > $OUT/chr21_timeline.txt
rm -rf $OUT/trace
echo "[$(date +%T)] e2e"
timeout -k 10 240 python3 bench.py --workload chr1 --contexts 1 --no-cpu-baseline --steps 10 > $OUT/chr1_bench.json 2> $OUT/chr1_bench.err
echo done
