#!/bin/bash
# Token-copy batch (k_tok_fill2): reconstruction tests, then chr1 reconstruction A/B over batch
# 1 / 2 (tree) / 3 and the previous commit's per-token copies, interleaved.
set -o pipefail
OUT=gpurun_out/r03tb2
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "reconstruct or roundtrip or golden or fuzz or paren or token or dense or synth" > $OUT/tests.out 2>&1 || { tail -30 $OUT/tests.out; exit 1; }
tail -n 1 $OUT/tests.out
for pass in 1 2 3; do
  for name in head prev3; do
    lib=variants/$name/libsccg.so; [ $name = head ] && lib=""
    echo "$name $(SCCG_LIB_PATH=$lib timeout -k 10 120 python3 $T/bench_decomp.py hg 247249719 249250621 1 --steps 10 2>/dev/null)" >> $OUT/res.txt || exit 1
  done
done
echo "headprof $(timeout -k 10 120 python3 $T/bench_decomp.py hg 247249719 249250621 1 --steps 10 --prof 2>/dev/null)" >> $OUT/res.txt
echo "prev3prof $(SCCG_LIB_PATH=variants/prev3/libsccg.so timeout -k 10 120 python3 $T/bench_decomp.py hg 247249719 249250621 1 --steps 10 --prof 2>/dev/null)" >> $OUT/res.txt
echo done
