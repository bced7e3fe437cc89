#!/bin/bash
# Chain knobs on the T2T-like 100 Mb pair: find-first window per block, generations per host sync,
# scan grid; then a kernel-stats profile and a phase-clock run of the default build.
set -o pipefail
OUT=gpurun_out/r03chain2
mkdir -p $OUT
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
for pass in 1 2; do
  for v in head:- ff16k:variants/ff16k/libsccg.so ff64k:variants/ff64k/libsccg.so gps8:variants/gps8/libsccg.so grid256:variants/grid256/libsccg.so; do
    IFS=: read name lib <<< "$v"; [ "$lib" = "-" ] && lib=""
    echo "$name $(SCCG_LIB_PATH=$lib timeout -k 10 120 python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 5 --sha 2>/dev/null)" >> $OUT/res.txt || exit 1
  done
done
cut -c1-300 $OUT/res.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t2t -o run -- python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 3 > $OUT/t2t.json 2> $OUT/t2t.err || exit 1
rm -f $OUT/t2t/*kernel_trace.csv
SCCG_DEBUG=1 timeout -k 10 120 python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 1 > $OUT/t2t_dbg.json 2> $OUT/t2t_dbg.err || exit 1
echo done
