#!/bin/bash
# After the packed-walk revert: chr1 / chr21 compress (tree vs round-2 end vs 2e58f56) and the chr1
# reconstruction (tree with the tiled decoders, with the scan-based ones, round-2 end), interleaved.
set -o pipefail
OUT=gpurun_out/r03r2
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
run() {   # tool lib env args...
  local tool=$1 lib=$2 ee=$3; shift 3
  [ "$lib" = "-" ] && lib=""
  env SCCG_LIB_PATH=$lib ${ee//,/ } timeout -k 10 120 python3 $T/$tool "$@" 2>/dev/null
}
for pass in 1 2; do
  for v in head:-:X=1 r02:variants/r_c9930e8/libsccg.so:X=1 g2e5:variants/r_2e58f56/libsccg.so:X=1; do
    IFS=: read name lib ee <<< "$v"
    echo "[$(date +%T)] pass $pass $name"
    echo "$name chr1 $(run bench_pair.py $lib $ee hg 247249719 249250621 1 --steps 10)" >> $OUT/res.txt || exit 1
    echo "$name chr21 $(run bench_pair.py $lib $ee hg 46944323 48129895 21 --steps 10)" >> $OUT/res.txt || exit 1
  done
  for v in head:-:X=1 headold:-:SCCG_RL_SCAN=1,SCCG_TOK_SCAN=1 headrl:-:SCCG_RL_SCAN=1 r02:variants/r_c9930e8/libsccg.so:X=1; do
    IFS=: read name lib ee <<< "$v"
    echo "[$(date +%T)] pass $pass decomp $name"
    echo "$name dchr1 $(run bench_decomp.py $lib $ee hg 247249719 249250621 1 --steps 10)" >> $OUT/res.txt || exit 1
  done
done
echo "head dchr1prof $(run bench_decomp.py - X=1 hg 247249719 249250621 1 --steps 10 --prof)" >> $OUT/res.txt
echo "head chr1prof $(run bench_pair.py - X=1 hg 247249719 249250621 1 --steps 10 --prof)" >> $OUT/res.txt
echo done
