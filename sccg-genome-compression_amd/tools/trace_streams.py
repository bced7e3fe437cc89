#!/usr/bin/env python3
"""Per-stream kernel timeline of the last compress in a rocprofv3 --kernel-trace CSV (diagnostics).

    python trace_streams.py <kernel_trace.csv> [--start-kernel k_find_header] [--n 80]

One line per kernel of the last group (a group opens at the start kernel more than 1 ms after the
previous group): start and end offset (us), stream, short name, grid size.
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
    ap.add_argument("--start-kernel", default="k_find_header")
    ap.add_argument("--n", type=int, default=80)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    starts = []
    for i, r in enumerate(rows):
        if a.start_kernel in r["Kernel_Name"] and (
                not starts or int(r["Start_Timestamp"]) - int(rows[starts[-1]]["Start_Timestamp"]) > 1_000_000):
            starts.append(i)
    if not starts:
        sys.exit("no start kernel found")
    i0 = starts[-1]
    t0 = int(rows[i0]["Start_Timestamp"])
    for r in rows[i0:i0 + a.n]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        print(f"{s:8.1f} {e:8.1f} s{r.get('Stream_Id', '?'):>3} {short(r['Kernel_Name']):24s} g{r.get('Grid_Size_X', '?')}")


if __name__ == "__main__":
    main()
