#!/bin/bash
# Profile the chr1 bench on the GPU box (run from the repo root, e.g. through gpurun):
#   1. rocprofv3 --kernel-trace --stats           -> per-kernel average durations
#   2. rocprofv3 --pmc FETCH_SIZE  (its own pass)  -> HBM read bytes per dispatch
#   3. rocprofv3 --pmc WRITE_SIZE  (its own pass)  -> HBM write bytes per dispatch
# then summarises 2+3 with pmc_summary.py (gfx950 FETCH_SIZE x2 correction, MI355X_MICROARCH.md).
# Usage: tools/profile_bench.sh <tag> [extra bench.py args]
set -eo pipefail
TAG=${1:-prof}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
TOOLS=sccg-genome-compression_amd/tools
BENCH="bench.py --no-cpu-baseline --no-check $*"

timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run \
    -- python3 $BENCH --steps 5 --warmup 1 > "$OUT/bench_under_rocprof.json" 2> "$OUT/stats.err"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
    -- python3 $BENCH --steps 2 --warmup 1 > /dev/null 2> "$OUT/fetch.err"
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
    -- python3 $BENCH --steps 2 --warmup 1 > /dev/null 2> "$OUT/write.err"

STATS=$(find "$OUT/stats" -name '*kernel_stats.csv' | head -n 1)
FETCH=$(find "$OUT/fetch" -name '*counter_collection.csv' | head -n 1)
WRITE=$(find "$OUT/write" -name '*counter_collection.csv' | head -n 1)
cp "$STATS" "$OUT/kernel_stats.csv"
python3 $TOOLS/pmc_summary.py "$FETCH" "$WRITE" "$OUT/pmc_summary.json" > "$OUT/pmc_summary.txt"
# keep only the small per-kernel summaries of the large per-dispatch CSVs
python3 - "$FETCH" "$WRITE" "$OUT" <<'EOF'
import csv, sys, collections
for path, name in ((sys.argv[1], "pmc_fetch_size.csv"), (sys.argv[2], "pmc_write_size.csv")):
    acc = collections.defaultdict(lambda: [0, 0.0])
    with open(path) as f:
        for row in csv.DictReader(f):
            a = acc[(row["Kernel_Name"], row["Counter_Name"])]
            a[0] += 1
            a[1] += float(row["Counter_Value"])
    with open(f"{sys.argv[3]}/{name}", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Counter_Name", "Dispatches", "Total_KiB", "Avg_KiB_per_dispatch"])
        for (k, c), (n, v) in sorted(acc.items(), key=lambda x: -x[1][1]):
            w.writerow([k, c, n, f"{v:.1f}", f"{v / n:.1f}"])
EOF
rm -rf "$OUT/fetch" "$OUT/write"
echo "profile done: $OUT"
