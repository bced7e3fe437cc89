#!/bin/bash
# Full GPU suite on the tree, then the genome bench A/B against the previous commit's library
# (variants/prev) and the pair timings, interleaved.
set -o pipefail
OUT=gpurun_out/r03full
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.out 2>&1 || { tail -30 $OUT/gpu_tests.out; exit 1; }
tail -n 1 $OUT/gpu_tests.out
run() { local lib=$1; shift; [ "$lib" = "-" ] && lib=""; env SCCG_LIB_PATH=$lib timeout -k 10 180 python3 "$@" 2>/dev/null | tail -n 1; }
for pass in 1 2; do
  for v in head:- prev:variants/prev2/libsccg.so; do
    IFS=: read name lib <<< "$v"
    echo "[$(date +%T)] $pass $name"
    echo "$name genome $(run $lib bench.py --no-cpu-baseline --no-decomp --no-e2e --no-check --steps 10)" >> $OUT/res.txt || exit 1
    echo "$name chr21 $(run $lib $T/bench_pair.py hg 46944323 48129895 21 --steps 10)" >> $OUT/res.txt || exit 1
    echo "$name chr1 $(run $lib $T/bench_pair.py hg 247249719 249250621 1 --steps 10)" >> $OUT/res.txt || exit 1
    echo "$name dchr1 $(run $lib $T/bench_decomp.py hg 247249719 249250621 1 --steps 10)" >> $OUT/res.txt || exit 1
  done
done
echo done
