#!/usr/bin/env python3
"""Per-kernel-family time in the last MS milliseconds of a rocprofv3 kernel trace (diagnostics).

    python trace_kernels.py <kernel_trace.csv> [--last-ms MS]
"""
from __future__ import annotations

import argparse
import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last-ms", type=float, default=0.0)
    a = ap.parse_args()
    ks = []
    with open(a.csv) as f:
        for row in csv.DictReader(f):
            ks.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), short(row["Kernel_Name"])))
    if a.last_ms > 0:
        t_end = max(e for _, e, _ in ks)
        ks = [k for k in ks if k[0] >= t_end - a.last_ms * 1e6]
    d = defaultdict(lambda: [0, 0])
    for s, e, n in ks:
        d[n][0] += e - s
        d[n][1] += 1
    for n, (t, c) in sorted(d.items(), key=lambda x: -x[1][0]):
        print(f"{t / 1e3:8.1f} us  x{c:3d}  {n}")


if __name__ == "__main__":
    main()
