#!/bin/bash
# k_walk waves per block (variants/wpb1, wpb2 vs the tree's 4) on chr21 / chr1 / the genome bench,
# interleaved; then walk chunk sizes with one wave per block.
set -o pipefail
OUT=gpurun_out/r03p
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
run() {   # tool lib env args...
  local tool=$1 lib=$2 ee=$3; shift 3
  [ "$lib" = "-" ] && lib=""
  env SCCG_LIB_PATH=$lib ${ee//,/ } timeout -k 10 180 python3 $tool "$@" 2>/dev/null
}
for pass in 1 2; do
  for v in wpb4:- wpb1:variants/wpb1/libsccg.so wpb2:variants/wpb2/libsccg.so; do
    IFS=: read name lib <<< "$v"
    echo "[$(date +%T)] pass $pass $name"
    echo "$name chr21 $(run $T/bench_pair.py $lib X=1 hg 46944323 48129895 21 --steps 10)" >> $OUT/res.txt || exit 1
    echo "$name chr1 $(run $T/bench_pair.py $lib X=1 hg 247249719 249250621 1 --steps 10)" >> $OUT/res.txt || exit 1
    echo "$name genome $(run bench.py $lib X=1 --no-cpu-baseline --no-decomp --no-e2e --no-check --no-prof --steps 10)" >> $OUT/res.txt || exit 1
  done
done
for c in 8192 12288 20480 24576; do
  echo "[$(date +%T)] wpb1 chunk $c"
  echo "wpb1_c$c chr21 $(run $T/bench_pair.py variants/wpb1/libsccg.so SCCG_WALK_CHUNK=$c hg 46944323 48129895 21 --steps 10)" >> $OUT/res.txt || exit 1
  echo "wpb1_c$c chr1 $(run $T/bench_pair.py variants/wpb1/libsccg.so SCCG_WALK_CHUNK=$c hg 247249719 249250621 1 --steps 10)" >> $OUT/res.txt || exit 1
done
echo done
