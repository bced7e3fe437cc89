#!/bin/bash
# Genome bench: contexts per GPU (2/3/4) and HIP-event profiling on/off in the timed region, interleaved.
set -o pipefail
OUT=gpurun_out/r03x
mkdir -p $OUT
export TMPDIR=/tmp
for pass in 1 2; do
  for v in "c2_prof:--contexts 2" "c2:--contexts 2 --no-prof" "c3:--contexts 3 --no-prof" "c4:--contexts 4 --no-prof" "c3_prof:--contexts 3"; do
    name=${v%%:*}; args=${v#*:}
    echo "[$(date +%T)] pass $pass $name"
    echo "$name $(timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-decomp --no-e2e --no-check --steps 10 $args 2>/dev/null | tail -n 1)" >> $OUT/res.txt || exit 1
  done
done
echo done
