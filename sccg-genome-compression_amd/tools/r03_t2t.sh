#!/bin/bash
# T2T-like 100 Mb pair: library variants (VARIANTS="name:lib ...") x walk knobs (KNOBS), record
# sha256 printed for the parity check against tests/golden/genome_manifest.json (t2t100).
set -o pipefail
OUT=gpurun_out/r03t
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
for v in ${VARIANTS:-base:-}; do
  name=${v%%:*}; lib=${v#*:}; [ "$lib" = "-" ] && lib=""
  for e in ${KNOBS:-X=1}; do
    echo "[$(date +%T)] $name $e"
    env SCCG_LIB_PATH=$lib ${e//,/ } timeout -k 10 100 python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 3 --sha > $OUT/${name}_${e//[=,]/_}.json 2>/dev/null
    echo "rc=$?"
  done
done
echo done
