#!/usr/bin/env python3
"""GPU occupancy of a rocprofv3 --kernel-trace CSV over its last `--window-ms` (diagnostics).

    python trace_busy.py <kernel_trace.csv> --window-ms 72

Prints the window's busy fraction (union of kernel intervals), the time with 1, 2, 3+ kernels in
flight, and per kernel family: summed duration, launches, and the time it ran alone."""
from __future__ import annotations

import argparse
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--window-ms", type=float, required=True)
    ap.add_argument("--windows", type=int, default=0,
                    help="also the busy fraction of this many consecutive windows back from the last kernel "
                         "(the last one usually holds the run's tail, not a step)")
    a = ap.parse_args()
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in csv.DictReader(open(a.csv))]
    t1 = max(e for _, e, _ in rows)
    if a.windows:
        merged: list[list[int]] = []
        for s, e, _ in sorted(rows):
            if merged and s <= merged[-1][1]:
                merged[-1][1] = max(merged[-1][1], e)
            else:
                merged.append([s, e])
        w = int(a.window_ms * 1e6)
        fr = []
        for k in range(a.windows):
            hi, lo = t1 - k * w, t1 - (k + 1) * w
            fr.append(sum(min(e, hi) - max(s, lo) for s, e in merged if e > lo and s < hi) / w)
        print("busy per window (last first): " + " ".join(f"{f:.3f}" for f in fr))
    t0 = t1 - int(a.window_ms * 1e6)
    rows = [(max(s, t0), e, n) for s, e, n in rows if e > t0]
    ev = sorted([(s, 1, i) for i, (s, _, _) in enumerate(rows)] + [(e, -1, i) for i, (_, e, _) in enumerate(rows)])
    live: set[int] = set()
    conc = collections.Counter()
    alone = collections.Counter()
    prev = t0
    for t, d, i in ev:
        if t > prev:
            conc[min(len(live), 3)] += t - prev
            if len(live) == 1:
                alone[rows[next(iter(live))][2]] += t - prev
        prev = t
        (live.add if d > 0 else live.discard)(i)
    span = t1 - t0
    print(f"window {span / 1e6:.3f} ms: idle {conc[0] / span:.1%}, 1 kernel {conc[1] / span:.1%}, "
          f"2 kernels {conc[2] / span:.1%}, 3+ {conc[3] / span:.1%}")
    tot = collections.Counter()
    cnt = collections.Counter()
    for s, e, n in rows:
        tot[n] += e - s
        cnt[n] += 1
    print(f"{'kernel':26s} {'sum ms':>8s} {'launches':>8s} {'alone ms':>8s}")
    for n, v in tot.most_common(30):
        print(f"{n:26s} {v / 1e6:8.3f} {cnt[n]:8d} {alone[n] / 1e6:8.3f}")


if __name__ == "__main__":
    main()
