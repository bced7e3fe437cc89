#!/bin/bash
# One rocprofv3 --pmc pass over a short chr1 bench (GPU box), summarised per kernel family:
#   tools/pmc_pass.sh <tag> "<counters (one pass's worth)>" [extra bench.py args]
set -eo pipefail
TAG=$1; CTRS=$2; shift 2
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmc/$TAG -o run -- \
    python3 bench.py --no-cpu-baseline --no-check --steps 2 --warmup 1 "$@" > /dev/null 2> gpurun_out/pmc/$TAG.err
F=$(find gpurun_out/pmc/$TAG -name '*counter_collection.csv' | head -n 1)
python3 sccg-genome-compression_amd/tools/sq_summary.py "$F" > gpurun_out/pmc/$TAG.txt
rm -rf gpurun_out/pmc/$TAG
