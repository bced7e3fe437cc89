#!/bin/bash
# Round 3: A/B of contexts x queues on the genome bench, then rocprof summaries (kernel stats +
# FETCH_SIZE / WRITE_SIZE passes) of the chr1 and genome workloads, and round-1 walk statistics
# without per-phase clocks.
set -eo pipefail
T=sccg-genome-compression_amd/tools
export TMPDIR=/tmp
bash $T/r03_ab.sh
bash $T/profile_bench.sh r03_chr1 --workload chr1 --contexts 1 --no-decomp --no-e2e
bash $T/profile_bench.sh r03_genome --no-decomp --no-e2e
OUT=gpurun_out/r03w2
mkdir -p $OUT
SCCG_HOST_FIRST_STEP=1 SCCG_DEBUG=1 timeout -k 10 120 python3 $T/bench_pair.py hg 46944323 48129895 21 --steps 1 > $OUT/chr21_r1.json 2> $OUT/chr21_r1.err
SCCG_HOST_FIRST_STEP=1 SCCG_DEBUG=1 timeout -k 10 120 python3 $T/bench_pair.py hg 247249719 249250621 1 --steps 1 > $OUT/chr1_r1.json 2> $OUT/chr1_r1.err
for c in 8192 12288; do
  SCCG_WALK_CHUNK=$c timeout -k 10 120 python3 $T/bench_pair.py hg 46944323 48129895 21 --steps 10 > $OUT/chr21_chunk$c.json 2>/dev/null
done
timeout -k 10 120 python3 $T/bench_pair.py hg 46944323 48129895 21 --steps 10 > $OUT/chr21_default.json 2>/dev/null
echo done
