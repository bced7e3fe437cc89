#!/usr/bin/env python3
"""Pin the full BASELINE configs[1] size against the REAL reference: run oracle/_ref (compiled from
/root/reference) on the chr1-sized synthetic pair (hg profile, |R| = 247,249,719, |T| = 249,250,621,
seed 1) and add its record/FASTA sha256 to synth_manifest.json.  Build container only; ~5 min of
single-threaded CPU and ~17 GB of RAM for the reference.

    python tests/golden/pin_chr1.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE)))

import synthlib  # noqa: E402
from make_golden import run_reference  # noqa: E402

ENTRY = ("hg", 247_249_719, 249_250_621, 1)


def main() -> None:
    prof, rl, tl, seed = ENTRY
    rfa, tfa = synthlib.synth_pair(prof, rl, tl, seed)
    res = run_reference(rfa, tfa)
    e = {"profile": prof, "ref_len": rl, "tgt_len": tl, "seed": seed,
         "ref_fa_sha256": hashlib.sha256(rfa).hexdigest(), "tgt_fa_sha256": hashlib.sha256(tfa).hexdigest(),
         "compress_rc": res["compress_rc"], "record_sha256": hashlib.sha256(res["record"]).hexdigest(),
         "record_len": len(res["record"]),
         "fasta_sha256": hashlib.sha256(res["fasta"]).hexdigest() if res["fasta"] else None}
    path = os.path.join(HERE, "synth_manifest.json")
    man = [m for m in json.load(open(path))
           if (m["profile"], m["ref_len"], m["tgt_len"], m["seed"]) != ENTRY]
    man.append(e)
    with open(path, "w") as f:
        json.dump(man, f, indent=1)
    print(e)


if __name__ == "__main__":
    main()
