#!/bin/bash
# Queue-scheduled walk: GPU tests, then chunk-size sweep (SCCG_WALK_CHUNK) on chr21 / chr1 pairs,
# the genome bench and the T2T pair.
set -eo pipefail
OUT=gpurun_out/r03c
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  echo "[$(date +%T)] tests"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.out 2>&1
fi
for c in ${CHUNKS:-default 4096 8192 12288 16384}; do
  e=""; [ "$c" != default ] && e="SCCG_WALK_CHUNK=$c"
  echo "[$(date +%T)] chunk $c"
  env $e timeout -k 10 120 python3 $T/bench_pair.py hg 46944323 48129895 21 --steps 10 > $OUT/chr21_$c.json 2>/dev/null
  env $e timeout -k 10 120 python3 $T/bench_pair.py hg 247249719 249250621 1 --steps 10 > $OUT/chr1_$c.json 2>/dev/null
  env $e timeout -k 10 120 python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 3 > $OUT/t2t_$c.json 2>/dev/null
  env $e timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-decomp --no-e2e --no-check --steps 10 > $OUT/genome_$c.json 2>/dev/null
done
echo done
