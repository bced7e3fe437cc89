#!/usr/bin/env python3
"""Regenerate the golden fixtures from the REAL reference (oracle/_ref, built from
/root/reference by `make -C oracle ref`).  Run in the build container only:

    python tests/golden/make_golden.py [--force]     (--force: rewrite existing fixtures too)

Writes
  tests/golden/cases/<name>.json.gz   inputs + the reference's outputs and exit codes
  tests/golden/synth_manifest.json    sha256 of the reference's record text / reconstruction
                                      for larger generator seeds (the inputs are regenerated
                                      from tools/synth.c by the tests; only hashes are kept)
The reference binaries run with the stub 7z (oracle/stub7z) on PATH; stdout is discarded.
"""
from __future__ import annotations

import base64
import gzip
import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))

import fuzzgen  # noqa: E402
import synthlib  # noqa: E402

REF_BIN = os.path.join(REPO, "oracle", "_ref")
STUB = os.path.join(REPO, "oracle", "stub7z")

N_LOCAL = 24
N_GLOBAL = 12
N_PAREN = 16   # targets whose literals hold '(' ')' ',' (delta_encode's own token scan)
SYNTH_SEEDS = [  # (profile, ref_len, tgt_len, seed)
    ("hg", 300_000, 301_000, 1),
    ("hg", 2_000_000, 2_003_000, 2),
    ("local", 2_000_000, 2_000_000, 3),
    ("t2t", 1_000_000, 1_000_000, 4),
    ("hg", 8_000_000, 8_020_000, 21),
]


def run_reference(ref_fa: bytes, tgt_fa: bytes) -> dict:
    env = dict(os.environ, PATH=STUB + os.pathsep + os.environ.get("PATH", ""))
    with tempfile.TemporaryDirectory() as d:
        rp, tp = os.path.join(d, "ref.fa"), os.path.join(d, "tgt.fa")
        open(rp, "wb").write(ref_fa)
        open(tp, "wb").write(tgt_fa)
        out = os.path.join(d, "out")
        c = subprocess.run([os.path.join(REF_BIN, "compression"), rp, tp, out], env=env,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        rec_path = os.path.join(out, "compressed_genome.txt")
        rec = open(rec_path, "rb").read() if os.path.exists(rec_path) else None
        res = {"compress_rc": c.returncode, "record": rec, "decompress_rc": None, "fasta": None}
        if c.returncode == 0:
            dec = os.path.join(d, "dec")
            dc = subprocess.run([os.path.join(REF_BIN, "decompression"), rec_path + ".7z", rp, dec],
                                env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            res["decompress_rc"] = dc.returncode
            fp = os.path.join(dec, "reconstructed_genome.fa")
            if dc.returncode == 0 and os.path.exists(fp):
                res["fasta"] = open(fp, "rb").read()
        return res


def b64(x: bytes | None):
    return None if x is None else base64.b64encode(x).decode()


def main() -> None:
    if not os.path.exists(os.path.join(REF_BIN, "compression")):
        sys.exit("oracle/_ref not built: run `make -C oracle ref` (needs /root/reference)")
    cases = {}
    for i in range(N_LOCAL):
        cases[f"local_{i:02d}"] = fuzzgen.local_case(i)
    for i in range(N_GLOBAL):
        cases[f"global_{i:02d}"] = fuzzgen.global_case(i)
    for i in range(N_PAREN):
        cases[f"paren_{i:02d}"] = fuzzgen.paren_case(i)
    cases.update(fuzzgen.quirk_cases())
    outdir = os.path.join(HERE, "cases")
    os.makedirs(outdir, exist_ok=True)
    force = "--force" in sys.argv
    for name, (rfa, tfa) in sorted(cases.items()):
        if not force and os.path.exists(os.path.join(outdir, name + ".json.gz")):
            continue   # fixtures are deterministic; keep the committed files byte-stable
        res = run_reference(rfa, tfa)
        doc = {"name": name, "ref_fa": b64(rfa), "tgt_fa": b64(tfa),
               "compress_rc": res["compress_rc"], "record": b64(res["record"]),
               "decompress_rc": res["decompress_rc"], "fasta": b64(res["fasta"])}
        with gzip.open(os.path.join(outdir, name + ".json.gz"), "wt") as f:
            json.dump(doc, f)
        print(f"{name:32s} rc={res['compress_rc']}/{res['decompress_rc']} "
              f"rec={len(res['record'] or b'')}B")
    manifest = []
    for prof, rl, tl, seed in SYNTH_SEEDS:
        rfa, tfa = synthlib.synth_pair(prof, rl, tl, seed)
        res = run_reference(rfa, tfa)
        manifest.append({"profile": prof, "ref_len": rl, "tgt_len": tl, "seed": seed,
                         "ref_fa_sha256": hashlib.sha256(rfa).hexdigest(),
                         "tgt_fa_sha256": hashlib.sha256(tfa).hexdigest(),
                         "compress_rc": res["compress_rc"],
                         "record_sha256": hashlib.sha256(res["record"]).hexdigest(),
                         "record_len": len(res["record"]),
                         "fasta_sha256": hashlib.sha256(res["fasta"]).hexdigest() if res["fasta"] else None})
        print(manifest[-1])
    with open(os.path.join(HERE, "synth_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
