#!/bin/bash
# Genome bench: local-pass blocks per CU (SCCG_LOCAL_BPC 2 / 3 / 4) with two contexts, interleaved.
set -o pipefail
OUT=gpurun_out/r03lbpc${TAG:-}
mkdir -p $OUT
export TMPDIR=/tmp
for pass in 1 2 3 4 5; do
  for b in 3 2; do
    SCCG_LOCAL_BPC=$b timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --no-decomp --no-e2e --no-prof > $OUT/b${b}_$pass.json 2> $OUT/b${b}_$pass.err || exit 1
    echo "bpc$b $(tail -n 1 $OUT/b${b}_$pass.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), round(d["value"]/1e9,1), d["parity"]["pinned_checked"])')"
  done
done
echo done
