#!/bin/bash
# Round-3 exploration on the GPU box: GPU tests, then the whole-genome bench under several
# context / hardware-queue settings.  Every GPU step has its own time limit; the first failure ends
# the script (no GPU work after a fault).
set -eo pipefail
OUT=gpurun_out/r03
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "[$(date +%T)] $name"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    step gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
fi
step bench_default 400 python3 bench.py
for cfg in "1 4" "2 4" "1 12" "3 16" "4 16"; do
    set -- $cfg
    step "bench_c$1_q$2" 240 python3 bench.py --contexts $1 --hw-queues $2 --no-cpu-baseline --no-decomp --steps 5
done
step bench_chr1 240 python3 bench.py --workload chr1 --contexts 1 --no-cpu-baseline --steps 10
echo done
