#!/bin/bash
# GPU box: interleaved A/B of library variants on the chr1 bench and (optionally) one bench_configs
# workload.  VARIANTS="name:lib[:VAR=v,VAR=v] ..." (lib "-" = in-tree), REPS, STEPS, CONFIG
# (bench_configs --only).
set -eo pipefail
mkdir -p gpurun_out/ab
for r in $(seq 1 ${REPS:-3}); do
  for v in $VARIANTS; do
    name=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; envs=""
    if [ "$rest" != "$lib" ]; then envs=${rest#*:}; fi
    if [ "$lib" = "-" ]; then lib=""; fi
    args=("SCCG_LIB_PATH=$lib")
    if [ -n "$envs" ]; then IFS=',' read -ra kv <<< "$envs"; args+=("${kv[@]}"); fi
    env "${args[@]}" timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-check --steps ${STEPS:-20} \
        > gpurun_out/ab/${name}_$r.json 2>/dev/null
    if [ -n "$CONFIG" ]; then
      env "${args[@]}" timeout -k 10 120 python -u sccg-genome-compression_amd/tools/bench_configs.py --only $CONFIG --steps 2 \
          > gpurun_out/ab/${name}_${CONFIG}_$r.json 2>/dev/null
    fi
  done
done
python3 - <<'PY'
import glob, json, os, collections
res = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/ab/*.json")):
    b = os.path.basename(f)[:-5]
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    key = b.rsplit("_", 1)[0]
    res[key].append(d.get("ms_per_step") or d.get("seconds", 0) * 1e3)
for k, v in sorted(res.items()):
    print(f"{k:30s} " + " ".join(f"{x:8.3f}" for x in v) + f"   min {min(v):.3f} ms")
PY
