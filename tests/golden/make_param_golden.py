#!/usr/bin/env python3
"""Fixtures for the NON-PARITY parameter overrides (sccg_params), made by the
REAL reference with its constants changed: `make -C oracle ref-param K=<k> M=<m>` compiles
/root/reference/compression.cpp with `int k = 14;` / `int m = 100;` (compression.cpp:373, :376)
substituted on the compiler's stdin (oracle/_ref/compression_k<k>_m<m>; no source is written).
Run in the build container only:

    python tests/golden/make_param_golden.py

Writes tests/golden/params.json.gz: per case the generator (tests/fuzzgen.py kind + seed, whose
inputs the tests regenerate and check by sha256), the parameter set, and the reference's record
text and exit code.  They pin oracle/'s orc_compress_params (local = 1, the reference's own
controller with the changed constants); the GPU's overrides are checked against that oracle.
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

STUB = os.path.join(REPO, "oracle", "stub7z")
# (k, m, generator, seeds)
SETS = [
    (21, 100, "global", range(0, 10)),
    (21, 100, "local", range(0, 8)),
    (17, 100, "global", range(0, 6)),
    (32, 100, "global", range(0, 6)),
    (12, 30, "global", range(0, 6)),
    (14, 50, "global", range(0, 8)),
    (14, 127, "global", range(0, 6)),
    (14, 0, "global", range(0, 4)),
]


def ref_binary(k: int, m: int) -> str:
    path = os.path.join(REPO, "oracle", "_ref", f"compression_k{k}_m{m}")
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref-param", f"K={k}", f"M={m}"], check=True)
    return path


def run(binary: str, rfa: bytes, tfa: bytes) -> tuple[int, bytes | None]:
    env = dict(os.environ, PATH=STUB + os.pathsep + os.environ.get("PATH", ""))
    with tempfile.TemporaryDirectory() as d:
        rp, tp, out = os.path.join(d, "r.fa"), os.path.join(d, "t.fa"), os.path.join(d, "o")
        open(rp, "wb").write(rfa)
        open(tp, "wb").write(tfa)
        c = subprocess.run([binary, rp, tp, out], env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        p = os.path.join(out, "compressed_genome.txt")
        return c.returncode, open(p, "rb").read() if os.path.exists(p) else None


def main() -> None:
    if not os.path.exists("/root/reference/compression.cpp"):
        sys.exit("reference sources absent")
    cases = []
    for k, m, gen, seeds in SETS:
        binary = ref_binary(k, m)
        for seed in seeds:
            rfa, tfa = (fuzzgen.global_case if gen == "global" else fuzzgen.local_case)(seed)
            rc, rec = run(binary, rfa, tfa)
            cases.append({"k": k, "m": m, "gen": gen, "seed": seed,
                          "ref_fa_sha256": hashlib.sha256(rfa).hexdigest(),
                          "tgt_fa_sha256": hashlib.sha256(tfa).hexdigest(),
                          "compress_rc": rc, "record": None if rec is None else base64.b64encode(rec).decode()})
            print(f"k={k:2d} m={m:3d} {gen}-{seed}: rc={rc} rec={len(rec or b'')}B")
    with gzip.open(os.path.join(HERE, "params.json.gz"), "wt") as f:
        json.dump(cases, f)


if __name__ == "__main__":
    main()
