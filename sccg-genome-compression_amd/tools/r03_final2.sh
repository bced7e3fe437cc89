#!/bin/bash
# Session-2 final check at HEAD: smoke, full GPU suite, T2T-like 100 Mb pair with kernel stats.
set -o pipefail
OUT=gpurun_out/r03final2
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.out 2>&1 || { cat $OUT/smoke.out; exit 1; }
cat $OUT/smoke.out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.out 2>&1 || { tail -30 $OUT/gpu_tests.out; exit 1; }
tail -n 1 $OUT/gpu_tests.out
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t2t -o run -- python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 3 --sha > $OUT/t2t.json 2> $OUT/t2t.err || exit 1
rm -f $OUT/t2t/*kernel_trace.csv
cut -c1-300 $OUT/t2t.json
echo done
