#!/bin/bash
# Session-2 evidence, part 2: the default bench line (genome headline, cpu_baseline on chr21,
# decompress, end-to-end, per-chromosome parity), then rocprofv3 kernel stats + FETCH/WRITE passes.
set -o pipefail
OUT=gpurun_out/r03end2
mkdir -p $OUT
export TMPDIR=/tmp
echo "[$(date +%T)] bench"
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -n 1 $OUT/bench.json | cut -c1-300
echo "[$(date +%T)] profile"
bash sccg-genome-compression_amd/tools/profile_bench.sh r03end2/prof || exit 1
echo done
