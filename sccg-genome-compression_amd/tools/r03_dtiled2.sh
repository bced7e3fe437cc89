#!/bin/bash
# Tiled decoders (16-byte lanes, LDS-staged) x the reconstruction's reference-strip grid cap.
set -o pipefail
OUT=gpurun_out/r03dt2
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
SCCG_RL_TILED=1 SCCG_TOK_TILED=1 SCCG_DC_STRIP_GRID=512 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "reconstruct or roundtrip or run_line or golden or fuzz or paren or token or dense or cli" > $OUT/tests.out 2>&1 || { tail -30 $OUT/tests.out; exit 1; }
tail -1 $OUT/tests.out
B="SCCG_RL_TILED=1,SCCG_TOK_TILED=1"
for pass in 1 2; do
  for e in X=1 $B $B,SCCG_DC_STRIP_GRID=256 $B,SCCG_DC_STRIP_GRID=512 $B,SCCG_DC_STRIP_GRID=1024 SCCG_DC_STRIP_GRID=512; do
    echo "$e $(env ${e//,/ } timeout -k 10 120 python3 $T/bench_decomp.py hg 247249719 249250621 1 --steps 10 2>/dev/null)" >> $OUT/res.txt || exit 1
  done
done
echo done
