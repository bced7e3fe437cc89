#!/bin/bash
# Round-1 per-chunk cost profile (SCCG_DEBUG with the host-side first step, so round 1 is read back
# before round 2 overwrites its counters) on the chr21 and chr1 pairs.
set -o pipefail
OUT=gpurun_out/r03d1
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
for p in "46944323 48129895 21" "247249719 249250621 1"; do
  set -- $p
  SCCG_DEBUG=1 SCCG_HOST_FIRST_STEP=1 timeout -k 10 120 python3 $T/bench_pair.py hg $p --steps 1 > $OUT/chr$3.json 2> $OUT/chr$3.err || exit 1
  SCCG_DEBUG=1 SCCG_DEBUG_PHASES=1 SCCG_HOST_FIRST_STEP=1 timeout -k 10 120 python3 $T/bench_pair.py hg $p --steps 1 > $OUT/chr$3_ph.json 2> $OUT/chr$3_ph.err || exit 1
done
echo done
