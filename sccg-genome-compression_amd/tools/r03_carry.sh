#!/bin/bash
# Carry-over fix-ups: full GPU suite, then head vs the previous commit (variants/prev3) on chr21,
# chr1, the T2T 100 Mb pair, the genome bench, and poor speculation (SCCG_ANCHOR_SHIFT=-2) on chr1.
set -o pipefail
OUT=gpurun_out/r03carry
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.out 2>&1 || { tail -30 $OUT/gpu_tests.out; exit 1; }
tail -n 1 $OUT/gpu_tests.out
run() { local lib=$1 ee=$2; shift 2; [ "$lib" = "-" ] && lib=""; env SCCG_LIB_PATH=$lib $ee timeout -k 10 180 python3 "$@" 2>/dev/null | tail -n 1; }
for pass in 1 2; do
  for v in head:- prev:variants/prev3/libsccg.so; do
    IFS=: read name lib <<< "$v"
    echo "[$(date +%T)] $pass $name"
    echo "$name chr21 $(run $lib X=1 $T/bench_pair.py hg 46944323 48129895 21 --steps 10)" >> $OUT/res.txt || exit 1
    echo "$name chr1 $(run $lib X=1 $T/bench_pair.py hg 247249719 249250621 1 --steps 10)" >> $OUT/res.txt || exit 1
    echo "$name t2t $(run $lib X=1 $T/bench_pair.py t2t 100000000 100000000 7 --steps 3 --sha)" >> $OUT/res.txt || exit 1
    echo "$name genome $(run $lib X=1 bench.py --no-cpu-baseline --no-decomp --no-e2e --no-check --steps 10)" >> $OUT/res.txt || exit 1
  done
done
for v in head:- prev:variants/prev3/libsccg.so; do
  IFS=: read name lib <<< "$v"
  echo "[$(date +%T)] shift $name"
  echo "$name chr1_shift2 $(run $lib SCCG_ANCHOR_SHIFT=-2 $T/bench_pair.py hg 247249719 249250621 1 --steps 2 --sha)" >> $OUT/res.txt || exit 1
done
echo done
