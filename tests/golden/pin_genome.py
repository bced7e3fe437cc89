#!/usr/bin/env python3
"""Pin BASELINE configs[2] (and configs[4]'s 100 Mb shape) against the REAL reference.

Runs oracle/_ref/compression + decompression (compiled from /root/reference, stub 7z) on

  * the 24 synthetic hg18/hg19 chromosome pairs at their UCSC lengths (hg profile, seed = chromosome
    index 1..24, X = 23, Y = 24 -- exactly the pairs bench.py and tools/bench_configs.py compress),
  * the 100 Mb T2T-like pair (t2t profile, seed 7; the stuck / literal-heavy path),
  * BASELINE configs[4]'s shape at full size: the same 24 UCSC length pairs with the T2T-like
    profile (seed = chromosome index, names t2t_chr1 .. t2t_chrY -- exactly the pairs
    `bench.py`'s t2t_genome leg and `tools/bench_configs.py --genome-profile t2t` compress),

and writes their record / FASTA sha256 to genome_manifest.json.  Build container only: the
reference needs ~70 B of RAM per reference base (17.4 GB for chr1), so pairs run concurrently
under a RAM budget, largest first (about 20 min on 8 cores / 62 GB for the hg pairs; the
T2T-like pairs' stuck walk runs ~3 s per Mb, about an hour more).

    python tests/golden/pin_genome.py [--budget-gb 46] [--only chr21,t2t100]
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, TESTS)

MANIFEST = os.path.join(HERE, "genome_manifest.json")


def jobs() -> list[dict]:
    import synthlib  # noqa: F401  (package dir on sys.path)
    import multigpu
    out = []
    for i, (name, rl, tl) in enumerate(zip(multigpu.CHROMS, multigpu.HG18, multigpu.HG19)):
        out.append({"name": name, "profile": "hg", "ref_len": rl, "tgt_len": tl, "seed": i + 1})
    out.append({"name": "t2t100", "profile": "t2t", "ref_len": 100_000_000, "tgt_len": 100_000_000, "seed": 7})
    for i, (name, rl, tl) in enumerate(zip(multigpu.CHROMS, multigpu.HG18, multigpu.HG19)):
        out.append({"name": "t2t_" + name, "profile": "t2t", "ref_len": rl, "tgt_len": tl, "seed": i + 1})
    return out


def run_one(job: dict) -> dict:
    import synthlib
    from make_golden import run_reference
    rfa, tfa = synthlib.synth_pair(job["profile"], job["ref_len"], job["tgt_len"], job["seed"])
    t0 = time.time()
    res = run_reference(rfa, tfa)
    e = dict(job)
    e.update({"ref_fa_sha256": hashlib.sha256(rfa).hexdigest(), "tgt_fa_sha256": hashlib.sha256(tfa).hexdigest(),
              "compress_rc": res["compress_rc"],
              "record_sha256": hashlib.sha256(res["record"]).hexdigest() if res["record"] is not None else None,
              "record_len": len(res["record"]) if res["record"] is not None else None,
              "decompress_rc": res["decompress_rc"],
              "fasta_sha256": hashlib.sha256(res["fasta"]).hexdigest() if res["fasta"] else None,
              "reference_wall_s": round(time.time() - t0, 1)})
    return e


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--budget-gb", type=float, default=46.0)
    ap.add_argument("--max-par", type=int, default=7)
    ap.add_argument("--only", default="")
    ap.add_argument("--one", default="", help=argparse.SUPPRESS)
    args = ap.parse_args()
    todo = jobs()
    if args.one:
        job = next(j for j in todo if j["name"] == args.one)
        print(json.dumps(run_one(job)), flush=True)
        return
    done = {}
    if os.path.exists(MANIFEST):
        done = {e["name"]: e for e in json.load(open(MANIFEST))}
    keep = set(args.only.split(",")) if args.only else None
    todo = [j for j in todo if (keep is None or j["name"] in keep) and j["name"] not in done]
    todo.sort(key=lambda j: -j["ref_len"])
    est = lambda j: 72e-9 * j["ref_len"] + 1.5   # GB: reference heap + the two FASTA copies
    running: dict = {}
    budget = args.budget_gb
    while todo or running:
        for name, (p, j) in list(running.items()):
            if p.poll() is not None:
                out = p.stdout.read()
                del running[name]
                if p.returncode != 0:
                    print(f"{name}: failed rc={p.returncode}", file=sys.stderr, flush=True)
                    continue
                e = json.loads(out.strip().splitlines()[-1])
                done[name] = e
                print(f"{name}: rc={e['compress_rc']} {e['record_len']} B {e['reference_wall_s']} s", flush=True)
                with open(MANIFEST, "w") as f:
                    json.dump(sorted(done.values(), key=lambda e: jobs_order(e["name"])), f, indent=1)
        used = sum(est(j) for _, j in running.values())
        for j in list(todo):
            if len(running) >= args.max_par:
                break
            if used + est(j) <= budget or not running:
                todo.remove(j)
                p = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--one", j["name"]],
                                     stdout=subprocess.PIPE, text=True)
                running[j["name"]] = (p, j)
                used += est(j)
        time.sleep(2)


def jobs_order(name: str) -> int:
    return [j["name"] for j in jobs()].index(name)


if __name__ == "__main__":
    main()
