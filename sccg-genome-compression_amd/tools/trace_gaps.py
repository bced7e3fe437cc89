#!/usr/bin/env python3
"""GPU idle time between kernels in a rocprofv3 --kernel-trace CSV (diagnostics).

    python trace_gaps.py <kernel_trace.csv> [--last-ms MS]

Looks at the kernels of the last MS milliseconds of the trace (default: all), prints the busy
time (union of kernel intervals), the span, and the largest gaps with the kernels on each side:
gaps are host-side synchronisation and launch latency on the critical path.
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
    ap.add_argument("--last-ms", type=float, default=0.0)
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    ks = []
    with open(a.csv) as f:
        for row in csv.DictReader(f):
            ks.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), short(row["Kernel_Name"])))
    ks.sort()
    if a.last_ms > 0:
        t_end = max(e for _, e, _ in ks)
        ks = [k for k in ks if k[0] >= t_end - a.last_ms * 1e6]
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    prev_name = None
    for s, e, n in ks:
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev_name, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_name = n
    if cur_e is not None:
        busy += cur_e - cur_s
    span = ks[-1][1] - ks[0][0] if ks else 0
    print(f"kernels {len(ks)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(span - busy) / 1e6:.3f} ms  "
          f"gaps {len(gaps)}")
    for g, p, n in sorted(gaps, reverse=True)[: a.top]:
        print(f"  gap {g / 1e3:9.1f} us   after {p:24s} before {n}")


if __name__ == "__main__":
    main()
