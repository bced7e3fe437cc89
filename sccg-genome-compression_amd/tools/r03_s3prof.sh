#!/bin/bash
# Session-3 profiles at HEAD: rocprofv3 kernel stats + FETCH/WRITE passes of the genome bench,
# then the T2T-like 100 Mb pair with phase clocks and per-round walk statistics.
set -o pipefail
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
OUT=gpurun_out/r03s3p
mkdir -p $OUT
echo "[$(date +%T)] profile"
bash $T/profile_bench.sh r03s3p || exit 1
echo "[$(date +%T)] t2t"
timeout -k 10 120 python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 3 --sha > $OUT/t2t.json 2> $OUT/t2t.err || exit 1
cat $OUT/t2t.json
SCCG_DEBUG=1 SCCG_DEBUG_ROUNDS=0 timeout -k 10 120 python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 1 > $OUT/t2t_dbg.json 2> $OUT/t2t_dbg.err || exit 1
echo done
