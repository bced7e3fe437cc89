#!/usr/bin/env python3
"""Kernel-by-kernel timeline of the last compress in a rocprofv3 --kernel-trace CSV (diagnostics).

    python trace_timeline.py <kernel_trace.csv> [--start-kernel k_first_match] [--nth -1]

Prints start offset, the idle gap before each kernel and its duration, from the first kernel of
the chosen compress (the n-th group opened by --start-kernel) until the next group starts.
"""
from __future__ import annotations

import argparse
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--start-kernel", default="k_first_match")
    ap.add_argument("--nth", type=int, default=-1)
    ap.add_argument("--min-gap-us", type=float, default=1000.0)
    a = ap.parse_args()
    ks = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(name), name))
    ks.sort()
    # group starts: a start kernel more than --min-gap-us after the previous group start
    starts = []
    for i, k in enumerate(ks):
        if a.start_kernel in k[3] and (not starts or k[0] - ks[starts[-1]][0] > a.min_gap_us * 1e3):
            starts.append(i)
    if not starts:
        sys.exit("no start kernel found")
    i0 = starts[a.nth]
    nxt = [s for s in starts if s > i0]
    i1 = nxt[0] if nxt else len(ks)
    t0, pe = ks[i0][0], ks[i0][0]
    busy = 0
    for s, e, n, _ in ks[i0:i1]:
        print(f"{(s - t0) / 1e3:8.1f} gap {(s - pe) / 1e3:6.1f} dur {(e - s) / 1e3:7.1f} {n}")
        busy += e - s
        pe = max(pe, e)
    print(f"span {(pe - t0) / 1e3:.1f} us, kernel time {busy / 1e3:.1f} us, {i1 - i0} kernels")


if __name__ == "__main__":
    main()
