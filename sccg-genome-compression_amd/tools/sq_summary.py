#!/usr/bin/env python3
"""Per-kernel SQ counter summary of one rocprofv3 --pmc pass (diagnostics).

    python sq_summary.py <counter_collection.csv>

Prints, per kernel family, the counters summed over dispatches and divided by the dispatch count,
plus the wave-cycle split (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over
SQ_WAVE_CYCLES, MI355X_MICROARCH.md §rocprofv3 PMC slots).
"""
from __future__ import annotations

import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main() -> None:
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    with open(sys.argv[1]) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[k].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    for k in sorted(acc, key=lambda x: -acc[x].get("SQ_WAVE_CYCLES", 0)):
        c = acc[k]
        n = max(1, len(disp[k]))
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        parts = " ".join(f"{name}={v / n:.3g}" for name, v in sorted(c.items()))
        split = (f"wait {c.get('SQ_WAIT_ANY', 0) / wc:.2f} inst-stall {c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
                 f"active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}")
        print(f"{k:24s} n={n:3d} | {split} | {parts}")


if __name__ == "__main__":
    main()
