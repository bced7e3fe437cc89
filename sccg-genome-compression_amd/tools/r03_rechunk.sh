#!/bin/bash
# Frozen-first re-chunk (FF_CHUNK) A/B on T2T-like pairs, then the genome bench and the full GPU suite.
set -o pipefail
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
OUT=gpurun_out/r03rechunk
mkdir -p $OUT
for rep in 1 2; do
  for e in "" "SCCG_NO_RECHUNK=1"; do
    for pr in "100000000 100000000 7" "20000000 20000000 5" "20000000 20000000 3"; do
      echo -n "[$e] rep $rep: " >> $OUT/ab.txt
      env $e timeout -k 10 120 python3 $T/bench_pair.py t2t $pr --steps 3 --sha >> $OUT/ab.txt 2>> $OUT/err.txt || { cat $OUT/ab.txt; tail $OUT/err.txt; exit 1; }
    done
  done
done
cat $OUT/ab.txt
echo "[$(date +%T)] bench"
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
echo "[$(date +%T)] tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.out 2>&1 || { tail -30 $OUT/gpu_tests.out; exit 1; }
tail -n 1 $OUT/gpu_tests.out
echo done
