#!/bin/bash
# Session-2 check at HEAD: smoke, GPU tests, T2T-like 100 Mb pair with phase clocks.
set -o pipefail
OUT=gpurun_out/r03s2
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
echo "[$(date +%T)] smoke"
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.out 2>&1 || { cat $OUT/smoke.out; exit 1; }
echo "[$(date +%T)] t2t"
timeout -k 10 120 python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 3 --sha --prof > $OUT/t2t.json 2> $OUT/t2t.err || exit 1
SCCG_DEBUG=1 timeout -k 10 120 python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 1 > $OUT/t2t_dbg.json 2> $OUT/t2t_dbg.err || exit 1
echo "[$(date +%T)] tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.out 2>&1
echo "tests rc=$?"
tail -3 $OUT/gpu_tests.out
echo done
