#!/bin/bash
# Round-3 regression hunt: the libraries of earlier commits (variants/r_<commit>) against the tree,
# interleaved, on the chr1 and chr21 pairs (bench_pair: device-resident compress time), then one
# pass with per-kernel HIP events on chr1.
set -o pipefail
OUT=gpurun_out/r03r
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
LIBS="head:- r02:variants/r_c9930e8/libsccg.so g2e5:variants/r_2e58f56/libsccg.so p67a:variants/r_67a3e1f/libsccg.so s668:variants/r_6688041/libsccg.so"
run() {   # name lib extra-env args...
  local name=$1 lib=$2 ee=$3; shift 3
  [ "$lib" = "-" ] && lib=""
  env SCCG_LIB_PATH=$lib $ee timeout -k 10 120 python3 $T/bench_pair.py "$@" 2>/dev/null
}
for pass in 1 2; do
  for v in $LIBS headrs:-:SCCG_RPACK_SWEEP=1; do
    IFS=: read name lib ee <<< "$v"; [ -z "$ee" ] && ee=X=1
    echo "[$(date +%T)] pass $pass $name"
    echo "$name chr1 $(run $name $lib $ee hg 247249719 249250621 1 --steps 10)" >> $OUT/res.txt || exit 1
    echo "$name chr21 $(run $name $lib $ee hg 46944323 48129895 21 --steps 10)" >> $OUT/res.txt || exit 1
  done
done
for v in $LIBS; do
  IFS=: read name lib ee <<< "$v"; [ -z "$ee" ] && ee=X=1
  echo "[$(date +%T)] prof $name"
  echo "$name chr1prof $(run $name $lib $ee hg 247249719 249250621 1 --steps 10 --prof)" >> $OUT/res.txt || exit 1
done
echo done
