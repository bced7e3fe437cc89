#!/bin/bash
# Interleaved timing of several build/environment variants on the GPU box.  $VARIANTS holds
# space-separated "name:lib:VAR=value,VAR=value" entries (lib "-" = in-tree libsccg.so, env may be
# empty); $REPS rounds of bench.py --steps $STEPS; one JSON line per run in gpurun_out/abm/.
set -eo pipefail
mkdir -p gpurun_out/abm
for r in $(seq 1 ${REPS:-3}); do
  for v in $VARIANTS; do
    name=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; envs=${rest#*:}
    args=()
    if [ "$lib" != "-" ]; then args+=("SCCG_LIB_PATH=$lib"); fi
    if [ -n "$envs" ]; then IFS=',' read -ra kv <<< "$envs"; args+=("${kv[@]}"); fi
    env "${args[@]}" timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-check --steps ${STEPS:-30} \
        > gpurun_out/abm/${name}_$r.json 2>/dev/null
  done
done
