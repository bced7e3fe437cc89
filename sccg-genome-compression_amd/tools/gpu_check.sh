#!/bin/bash
# GPU box: full GPU test suite, then short benches (env variants in $VARIANTS, e.g.
# "SCCG_STALE_BUDGET=2048 SCCG_WALK_CHUNK=8192"; "-" = defaults) and an optional SCCG_DEBUG trace.
set -eo pipefail
mkdir -p gpurun_out/check
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/check/pytest.log 2>&1
i=0
for v in ${VARIANTS:--}; do
  if [ "$v" = "-" ]; then v=""; fi
  env $v timeout -k 10 150 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/check/bench_$i.json 2> gpurun_out/check/bench_$i.err
  echo "$v" > gpurun_out/check/bench_$i.env
  i=$((i+1))
done
if [ -n "$WALKDBG" ]; then
  SCCG_DEBUG=1 timeout -k 10 200 python -u sccg-genome-compression_amd/tools/dbg_walk.py hg 247249719 249250621 1 > gpurun_out/check/dbg_walk.log 2>&1
fi
