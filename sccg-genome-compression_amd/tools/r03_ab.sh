#!/bin/bash
# Whole-genome bench A/B: contexts per GPU x hardware queues, interleaved, two passes.
set -eo pipefail
OUT=gpurun_out/r03ab
mkdir -p $OUT
export TMPDIR=/tmp
CFGS=${CFGS:-"1:4 2:4 2:8 3:8 3:12 4:16"}
for pass in 1 2; do
  for cfg in $CFGS; do
    c=${cfg%%:*}; q=${cfg##*:}
    echo "[$(date +%T)] pass $pass c$c q$q"
    timeout -k 10 240 python3 bench.py --contexts $c --hw-queues $q --no-cpu-baseline --no-decomp --no-e2e --no-check --steps 20 --warmup 2 \
        > $OUT/p${pass}_c${c}_q${q}.json 2> $OUT/p${pass}_c${c}_q${q}.err
  done
done
echo done
