#!/bin/bash
# SQ counters of the genome bench's kernels (k_walk first), two rocprofv3 --pmc passes of at most
# 8 SQ counters each, summarised per kernel family by sq_summary.py:
#   tools/walk_sq.sh <tag> [extra bench.py args]        -> gpurun_out/<tag>/sq_{a,b}.txt
set -eo pipefail
TAG=${1:-sq}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
BENCH="bench.py --no-cpu-baseline --no-check --no-decomp --no-e2e --no-t2t --steps 2 --warmup 1 $*"
pass() {   # name, counters
  timeout -s KILL 90 rocprofv3 --pmc $2 --output-format csv -d "$OUT/$1" -o run -- python3 $BENCH > /dev/null 2> "$OUT/$1.err"
  F=$(find "$OUT/$1" -name '*counter_collection.csv' | head -n 1)
  python3 $T/sq_summary.py "$F" > "$OUT/sq_$1.txt"
  rm -rf "$OUT/$1"
}
pass a "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
pass b "SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES"
echo "sq done: $OUT"
