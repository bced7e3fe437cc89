#!/bin/bash
# Genome bench pair order over the two contexts: lpt (largest first) vs twoend, interleaved.
set -o pipefail
OUT=gpurun_out/r03queue
mkdir -p $OUT
export TMPDIR=/tmp
for pass in 1 2 3; do
  for q in lpt twoend; do
    timeout -k 10 300 python3 bench.py --queue $q --steps 10 --no-cpu-baseline --no-decomp --no-e2e --no-prof > $OUT/${q}_$pass.json 2> $OUT/${q}_$pass.err || exit 1
    echo "$q $(tail -n 1 $OUT/${q}_$pass.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), round(d["value"]/1e9,1), d["parity"]["pinned_checked"])')"
  done
done
echo done
