#!/bin/bash
# GPU tests (strip-fused packing check, tiled decompression parsers, compress_files), the genome
# bench with R' packed by its strip vs by the sweep, the chr1 bench (decompression leg), then the
# T2T variant sweep (r03_t2t.sh).
set -o pipefail
OUT=gpurun_out/r03g
mkdir -p $OUT
export TMPDIR=/tmp
echo "[$(date +%T)] tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.out 2>&1 || { tail -40 $OUT/gpu_tests.out; exit 1; }
tail -2 $OUT/gpu_tests.out
echo "[$(date +%T)] genome"
timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-decomp --no-e2e --no-check --steps 10 > $OUT/genome.json 2> $OUT/genome.err || exit 1
echo "[$(date +%T)] genome rsweep"
SCCG_RPACK_SWEEP=1 timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-decomp --no-e2e --no-check --steps 10 > $OUT/genome_rsweep.json 2> $OUT/genome_rsweep.err || exit 1
echo "[$(date +%T)] chr1"
timeout -k 10 240 python3 bench.py --workload chr1 --contexts 1 --no-cpu-baseline --steps 10 > $OUT/chr1.json 2> $OUT/chr1.err || exit 1
echo "[$(date +%T)] t2t"
bash sccg-genome-compression_amd/tools/r03_t2t.sh
