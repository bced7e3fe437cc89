#!/bin/bash
# One rocprofv3 --pmc pass over one bench_configs workload (GPU box), summarised per kernel family:
#   tools/pmc_config.sh <tag> <workload> "<counters (one pass's worth)>"
set -eo pipefail
TAG=$1; WL=$2; CTRS=$3
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmc/$TAG -o run -- \
    python3 sccg-genome-compression_amd/tools/bench_configs.py --only $WL --steps 1 > /dev/null 2> gpurun_out/pmc/$TAG.err
F=$(find gpurun_out/pmc/$TAG -name '*counter_collection.csv' | head -n 1)
python3 sccg-genome-compression_amd/tools/sq_summary.py "$F" > gpurun_out/pmc/$TAG.txt
rm -rf gpurun_out/pmc/$TAG
