set -e
mkdir -p gpurun_out/sweep
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep/pytest.log 2>&1
for c in 16384 8192 4096; do
  SCCG_WALK_CHUNK=$c timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/sweep/bench_$c.json 2> gpurun_out/sweep/bench_$c.err
done
