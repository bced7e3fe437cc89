set -eo pipefail
mkdir -p gpurun_out/sq
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/sq/a -o run -- python3 bench.py --no-cpu-baseline --no-check --steps 2 --warmup 1 > /dev/null 2> gpurun_out/sq/a.err
F=$(find gpurun_out/sq/a -name '*counter_collection.csv' | head -n 1)
python3 sccg-genome-compression_amd/tools/sq_summary.py "$F" > gpurun_out/sq/summary.txt
rm -rf gpurun_out/sq/a
