#!/bin/bash
# GPU box: decompression tests (optional, $DTESTS = pytest -k expression), then a rocprofv3
# kernel trace of the chr1 reconstruction (bench_configs chr1_decompress) -> per-kernel stats and
# the per-stream timeline of the last reconstruction.
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/dprof
mkdir -p $OUT
if [ -n "$DTESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$DTESTS" > $OUT/pytest.log 2>&1
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o run -- python3 sccg-genome-compression_amd/tools/bench_configs.py --only chr1_decompress --steps 5 > $OUT/out_prof.json 2> $OUT/err.log
T=$(find $OUT/tr -name '*kernel_trace.csv' | head -n 1)
S=$(find $OUT/tr -name '*kernel_stats.csv' | head -n 1)
cp "$S" $OUT/kernel_stats.csv
python3 sccg-genome-compression_amd/tools/trace_streams.py "$T" --start-kernel k_newlines --n 120 > $OUT/timeline.txt
rm -rf $OUT/tr
timeout -k 10 200 python3 sccg-genome-compression_amd/tools/bench_configs.py --only chr1_decompress --steps 20 > $OUT/out.json
