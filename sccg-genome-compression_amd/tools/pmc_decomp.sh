#!/bin/bash
# GPU box: one SQ counter pass over the chr1 reconstruction (bench_configs chr1_decompress) ->
# per-kernel sums in gpurun_out/dpmc/summary.txt (diagnostics).  Optional: $1 = output tag, then the
# counters of the pass (at most 8 SQ counters).
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/dpmc${1:+_$1}
shift || true
CTRS="$*"
[ -z "$CTRS" ] && CTRS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES"
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc $CTRS \
    --output-format csv -d $OUT/raw -o run -- python3 sccg-genome-compression_amd/tools/bench_configs.py --only chr1_decompress --steps 2 > $OUT/out.json 2> $OUT/err.log
F=$(find $OUT/raw -name '*counter_collection.csv' | head -n 1)
python3 - "$F" > $OUT/summary.txt <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:60]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    if any(s in k for s in ("format", "tok_fill", "span_index", "strip_write", "rl_", "tok_blocks")):
        print(k, {c: int(v) for c, v in sorted(d.items())})
PY
rm -rf $OUT/raw
