#!/bin/bash
# A/B timing on the GPU box: alternates the default build/environment and an alternative --
# $ALT (a libsccg.so path) and/or $ALT_ENV ("VAR=value ...") -- for $REPS rounds of
# bench.py --steps $STEPS; one JSON line per run in gpurun_out/ab/.
set -eo pipefail
mkdir -p gpurun_out/ab
for r in $(seq 1 ${REPS:-3}); do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-check --steps ${STEPS:-30} > gpurun_out/ab/new_$r.json 2>/dev/null
  env ${ALT:+SCCG_LIB_PATH=$ALT} $ALT_ENV timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-check --steps ${STEPS:-30} > gpurun_out/ab/alt_$r.json 2>/dev/null
done
