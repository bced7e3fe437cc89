#!/bin/bash
# LDS-staged tiled decoders: reconstruction tests with both switched on, then the chr1
# reconstruction A/B (scan-based / tiled run lines / tiled record line / both), interleaved.
set -o pipefail
OUT=gpurun_out/r03dt
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
SCCG_RL_TILED=1 SCCG_TOK_TILED=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "reconstruct or roundtrip or run_line or golden or fuzz or paren or token or dense or cli" > $OUT/tests.out 2>&1 || { tail -30 $OUT/tests.out; exit 1; }
tail -1 $OUT/tests.out
for pass in 1 2; do
  for e in X=1 SCCG_RL_TILED=1 SCCG_TOK_TILED=1 SCCG_RL_TILED=1,SCCG_TOK_TILED=1; do
    echo "$e $(env ${e//,/ } timeout -k 10 120 python3 $T/bench_decomp.py hg 247249719 249250621 1 --steps 10 2>/dev/null)" >> $OUT/res.txt || exit 1
  done
done
echo "prof $(SCCG_RL_TILED=1 SCCG_TOK_TILED=1 timeout -k 10 120 python3 $T/bench_decomp.py hg 247249719 249250621 1 --steps 10 --prof 2>/dev/null)" >> $OUT/res.txt
echo done
