#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (one counter per pass) per kernel.

    python pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>
                          [--stats <kernel_stats.csv>]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE
counts exactly half the bytes of a wide (16 B/lane) coalesced streaming read, so the corrected
read bytes are 2 x FETCH_SIZE for such kernels; narrower access widths are uncalibrated and are
reported with the same factor (stated in the JSON).  WRITE_SIZE is exact for 16-B stores.
"""
from __future__ import annotations

import csv
import json
import re
import sys
from collections import defaultdict

FAMILY = {  # kernel symbol fragment -> bench.py / sccg_profile family name
    "k_walk<false, true>": "walk_carry", "k_walk<true, true>": "walk_carry", "k_walk(": "walk", "k_walk<": "walk", "k_local_all": "local_segments", "k_local_pass<14>": "local_pass_k14", "k_local_pass<10>": "local_pass_k10",
    "k_strip_write": "fasta_strip", "k_filter_write": "n_filter", "k_runs_write": "run_extract", "k_runs_copy": "run_extract",
    "k_sweep_early<true>": "first_sweep_anchors",
    "k_run_textwrite": "run_text", "k_seg_textwrite": "local_emit", "k_anchor_build": "anchor_build", "k_key0<true>": "first_sweep_anchors", "k_chunk_text<true>": "match_emit",
    "k_presence": "presence_scan", "k_fullc": "fullc_scan", "k_match_textwrite": "match_emit",
    "k_tok_fill": "dc_decode", "k_format": "dc_format",
}


def short(name: str) -> str:
    for frag, fam in FAMILY.items():
        if frag in name:
            return fam
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:40]


def load(path: str, counter: str) -> dict:
    acc = defaultdict(lambda: [0.0, 0])
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            k = short(row["Kernel_Name"])
            acc[k][0] += float(row["Counter_Value"])
            acc[k][1] += 1
    return acc


def main() -> None:
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {"_note": "KiB counters per dispatch; hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE)*1024 "
                    "(gfx950 FETCH_SIZE = 1/2 of wide streaming reads; narrower widths uncalibrated)"}
    for k in sorted(set(fetch) | set(write)):
        f_kib = fetch[k][0] / fetch[k][1] if fetch[k][1] else 0.0
        w_kib = write[k][0] / write[k][1] if write[k][1] else 0.0
        out[k] = {"dispatches": max(fetch[k][1], write[k][1]), "fetch_kib": f_kib, "write_kib": w_kib,
                  "hbm_bytes_per_launch": (2.0 * f_kib + w_kib) * 1024.0}
    json.dump(out, open(sys.argv[3], "w"), indent=1, sort_keys=True)
    for k, v in out.items():
        if not k.startswith("_"):
            print(f"{k:28s} n={v['dispatches']:3d} fetch={v['fetch_kib']/1024:10.1f} MiB write={v['write_kib']/1024:9.1f} MiB")


if __name__ == "__main__":
    main()
