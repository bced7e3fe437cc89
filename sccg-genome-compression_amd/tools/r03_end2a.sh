#!/bin/bash
# Session-2 evidence, part 1: smoke, the full GPU suite, genome bench contexts A/B (2 / 3 per GPU).
set -o pipefail
OUT=gpurun_out/r03end2
mkdir -p $OUT
export TMPDIR=/tmp
echo "[$(date +%T)] smoke"
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.out 2>&1 || { cat $OUT/smoke.out; exit 1; }
echo "[$(date +%T)] tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.out 2>&1 || { tail -30 $OUT/gpu_tests.out; exit 1; }
tail -n 1 $OUT/gpu_tests.out
for pass in 1 2; do
  for c in 2 3; do
    echo "[$(date +%T)] contexts $c"
    timeout -k 10 300 python3 bench.py --contexts $c --steps 5 --no-cpu-baseline --no-decomp --no-e2e --no-prof > $OUT/ctx${c}_$pass.json 2> $OUT/ctx${c}_$pass.err || exit 1
    tail -n 1 $OUT/ctx${c}_$pass.json | cut -c1-200
  done
done
echo done
