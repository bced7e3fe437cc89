#!/bin/bash
# Walk chunk 8 Ki vs the size rule on the genome bench, the chr1 pair and chr21; T2T-like at 4 / 6 Ki.
set -o pipefail
export TMPDIR=/tmp
T=sccg-genome-compression_amd/tools
OUT=gpurun_out/r03chunk8
mkdir -p $OUT
for rep in 1 2; do
  for c in rule 8192; do
    if [ $c = rule ]; then E=""; else E="SCCG_WALK_CHUNK=$c"; fi
    echo "[$(date +%T)] genome $c rep $rep"
    env $E timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $OUT/genome_${c}_$rep.json 2>> $OUT/err.txt || exit 1
    python3 -c "import json,sys;d=json.load(open('$OUT/genome_${c}_$rep.json'));print('genome $c', round(d['ms_per_step'],2), d['parity']['pinned_mismatch'])" | tee -a $OUT/ab.txt
    echo -n "chr1 $c rep $rep: " >> $OUT/ab.txt
    env $E timeout -k 10 120 python3 $T/bench_pair.py hg 247249719 249250621 1 --steps 5 --sha >> $OUT/ab.txt 2>> $OUT/err.txt || exit 1
  done
done
for c in 4096 6144; do
  echo -n "t2t100 $c: " >> $OUT/ab.txt
  SCCG_WALK_CHUNK=$c timeout -k 10 120 python3 $T/bench_pair.py t2t 100000000 100000000 7 --steps 3 --sha >> $OUT/ab.txt 2>> $OUT/err.txt || exit 1
done
cat $OUT/ab.txt
