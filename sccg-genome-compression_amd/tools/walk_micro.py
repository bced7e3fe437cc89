#!/usr/bin/env python3
"""Walk-step micro-workloads (diagnostics): the global walk (sccg_walk_range from the true start) on
sequences built to isolate one regime of compression.cpp:64-161's loop --
  dense:   a 171-bp tandem array (3 % divergent copies) against a 1e-2 SNP copy: a match every
           ~25 target bases, the serial chains of the T2T-like pairs' arrays;
  aligned: random sequence against a 1e-3 SNP copy: a match every ~1 kb (the hg regime);
  stuck:   random sequence against an unrelated one: literal steps only (wide scans).
Prints per workload: matches, walk time per call, rounds.  Run under rocprofv3 --pmc for per-wave
instruction and wait counts of k_walk.

    python walk_micro.py [--n 4000000] [--reps 3] [--only dense]
"""
import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def mutate(rng, s: bytearray, snp: float) -> bytearray:
    out = bytearray(s)
    for i in range(len(out)):
        if rng.random() < snp:
            out[i] = rng.choice([c for c in b"ACGT" if c != out[i]])
    return out


def make(kind: str, n: int, seed: int):
    rng = random.Random(seed)
    if kind == "dense":
        unit = bytes(rng.choice(b"ACGT") for _ in range(171))
        R = bytearray(unit[i % 171] for i in range(n))
        R = mutate(rng, R, 0.03)
        T = mutate(rng, R, 0.01)
    elif kind == "aligned":
        R = bytearray(rng.choice(b"ACGT") for _ in range(n))
        T = mutate(rng, R, 0.001)
    else:
        R = bytearray(rng.choice(b"ACGT") for _ in range(n))
        T = bytearray(rng.choice(b"ACGT") for _ in range(n))
    return bytes(R), bytes(T)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    import sccg
    c = sccg.Context(0)
    for kind in ("dense", "aligned", "stuck"):
        if a.only and a.only != kind:
            continue
        R, T = make(kind, a.n, 5)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            m, ex = c.walk_range(R, T, 14, 100, 0, -1, len(T))
            ts.append(time.perf_counter() - t0)
        st = c.stats()
        print(json.dumps({"kind": kind, "n": a.n, "matches": len(m), "exit": ex, "ms": [round(t * 1e3, 3) for t in ts],
                          "rounds": st["walk_rounds"], "chunks": st["walk_chunks"]}), flush=True)
    c.close()


if __name__ == "__main__":
    main()
