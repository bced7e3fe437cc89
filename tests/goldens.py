"""Loader for tests/golden/cases/*.json.gz (made by tests/golden/make_golden.py from the real
reference binaries) and tests/golden/synth_manifest.json."""
from __future__ import annotations

import base64
import glob
import gzip
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
CASE_DIR = os.path.join(HERE, "golden", "cases")


def _d(x):
    return None if x is None else base64.b64decode(x)


def load_cases() -> list[dict]:
    cases = []
    for p in sorted(glob.glob(os.path.join(CASE_DIR, "*.json.gz"))):
        with gzip.open(p, "rt") as f:
            doc = json.load(f)
        for key in ("ref_fa", "tgt_fa", "record", "fasta"):
            doc[key] = _d(doc[key])
        cases.append(doc)
    return cases


def synth_manifest() -> list[dict]:
    with open(os.path.join(HERE, "golden", "synth_manifest.json")) as f:
        return json.load(f)
