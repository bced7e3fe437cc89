#!/bin/bash
# Session-3 check at HEAD: smoke, full GPU suite, default bench line.
set -o pipefail
OUT=gpurun_out/r03s3
mkdir -p $OUT
export TMPDIR=/tmp
echo "[$(date +%T)] smoke"
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.out 2>&1 || { cat $OUT/smoke.out; exit 1; }
echo "[$(date +%T)] bench"
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
echo "[$(date +%T)] tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.out 2>&1 || { tail -30 $OUT/gpu_tests.out; exit 1; }
tail -n 1 $OUT/gpu_tests.out
echo done
