"""Pin the CPU restatement (oracle/) against the reference's own outputs.

* every committed fixture (tests/golden/cases, produced by the compiled reference) must be
  reproduced byte-for-byte, including the exit-code behaviour;
* the larger generator seeds must hash to the reference's sha256 (synth_manifest.json);
* when oracle/_ref exists (the build container), a wider differential fuzz runs live.
"""
import hashlib
import os
import subprocess
import tempfile

import pytest

import fuzzgen
import goldens
import oraclelib
import synthlib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_BIN = os.path.join(REPO, "oracle", "_ref")
HAVE_REF = os.path.exists(os.path.join(REF_BIN, "compression"))


def _check_case(c):
    try:
        rec = oraclelib.compress(c["ref_fa"], c["tgt_fa"])
        rc = 0
    except oraclelib.OracleError as e:
        rec, rc = e.partial, 1
    assert rc == c["compress_rc"], c["name"]
    assert rec == c["record"], c["name"]
    if c["decompress_rc"] is None:
        return
    try:
        fa = oraclelib.decompress(rec, c["ref_fa"])
        drc = 0
    except oraclelib.OracleError:
        fa, drc = None, 1
    assert drc == c["decompress_rc"], c["name"]
    if drc == 0:
        assert fa == c["fasta"], c["name"]


def test_golden_fixtures(golden_cases):
    assert len(golden_cases) >= 40
    for c in golden_cases:
        _check_case(c)


def test_quirk_b1_sentinel(golden_cases):
    c = next(c for c in golden_cases if c["name"] == "b1_pn0_sentinel")
    # the tie between candidate 0 and candidate 100 goes to 100 (compression.cpp:125)
    assert b"(100,30)" in c["record"]


def test_quirk_b2_stuck(golden_cases):
    c = next(c for c in golden_cases if c["name"] == "b2_stuck_walk")
    tail = c["record"].rsplit(b")", 1)[1]
    assert len(tail) > 5000 and set(tail) <= set(b"ACGT")


@pytest.mark.parametrize("entry", goldens.synth_manifest(), ids=lambda e: f"{e['profile']}-{e['seed']}")
def test_synth_manifest(entry):
    if entry["ref_len"] > 3_000_000:
        pytest.skip("large seed: covered on the GPU box")
    rfa, tfa = synthlib.synth_pair(entry["profile"], entry["ref_len"], entry["tgt_len"], entry["seed"])
    assert hashlib.sha256(rfa).hexdigest() == entry["ref_fa_sha256"]
    assert hashlib.sha256(tfa).hexdigest() == entry["tgt_fa_sha256"]
    rec = oraclelib.compress(rfa, tfa)
    assert hashlib.sha256(rec).hexdigest() == entry["record_sha256"]
    fa = oraclelib.decompress(rec, rfa)
    assert hashlib.sha256(fa).hexdigest() == entry["fasta_sha256"]


def _run_ref(rfa, tfa):
    env = dict(os.environ, PATH=os.path.join(REPO, "oracle", "stub7z") + os.pathsep + os.environ["PATH"])
    with tempfile.TemporaryDirectory() as d:
        rp, tp = os.path.join(d, "r.fa"), os.path.join(d, "t.fa")
        open(rp, "wb").write(rfa)
        open(tp, "wb").write(tfa)
        subprocess.run([os.path.join(REF_BIN, "compression"), rp, tp, os.path.join(d, "o")], env=env,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True)
        return open(os.path.join(d, "o", "compressed_genome.txt"), "rb").read()


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built (reference sources absent)")
@pytest.mark.parametrize("kind,seed", [("local", s) for s in range(100, 160)] +
                         [("global", s) for s in range(100, 124)])
def test_differential_vs_reference(kind, seed):
    rfa, tfa = (fuzzgen.local_case if kind == "local" else fuzzgen.global_case)(seed)
    assert oraclelib.compress(rfa, tfa) == _run_ref(rfa, tfa)


def _run_ref_decompress(rec, rfa):
    """decompression <arc> <ref> <out> with the stub 7z (which copies the archive to out/<stem>)."""
    env = dict(os.environ, PATH=os.path.join(REPO, "oracle", "stub7z") + os.pathsep + os.environ["PATH"])
    with tempfile.TemporaryDirectory() as d:
        ap, rp = os.path.join(d, "compressed_genome.txt.7z"), os.path.join(d, "r.fa")
        open(ap, "wb").write(rec)
        open(rp, "wb").write(rfa)
        p = subprocess.run([os.path.join(REF_BIN, "decompression"), ap, rp, os.path.join(d, "o")], env=env,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        if p.returncode:
            return p.returncode, None
        return 0, open(os.path.join(d, "o", "reconstructed_genome.fa"), "rb").read()


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built (reference sources absent)")
@pytest.mark.parametrize("seed", range(16))
def test_close_paren_literals_vs_reference(seed):
    """')' bytes in the target survive delta_encode and decode as literals (decompression.cpp:231-234)."""
    rfa, tfa = fuzzgen.close_paren_case(seed)
    rec = oraclelib.compress(rfa, tfa)
    assert rec == _run_ref(rfa, tfa)
    rc, fa = _run_ref_decompress(rec, rfa)
    try:
        assert (rc, fa) == (0, oraclelib.decompress(rec, rfa))
    except oraclelib.OracleError as e:
        assert rc != 0 and e.rc != 0


# ---- parameter overrides (sccg_params) ----------------------------------------
@pytest.mark.parametrize("case", goldens.param_cases(), ids=lambda c: f"k{c['k']}-m{c['m']}-{c['gen']}{c['seed']}")
def test_param_fixtures(case):
    """orc_compress_params reproduces the reference built with other k / m (make_param_golden.py)."""
    rfa, tfa = goldens.param_inputs(case)
    try:
        rec, rc = oraclelib.compress_params(rfa, tfa, k=case["k"], m=case["m"]), 0
    except oraclelib.OracleError as e:
        rec, rc = e.partial, 1
    assert rc == case["compress_rc"]
    assert rec == case["record"]


def _run_ref_param(k, m, rfa, tfa):
    binary = os.path.join(REF_BIN, f"compression_k{k}_m{m}")
    env = dict(os.environ, PATH=os.path.join(REPO, "oracle", "stub7z") + os.pathsep + os.environ["PATH"])
    with tempfile.TemporaryDirectory() as d:
        rp, tp = os.path.join(d, "r.fa"), os.path.join(d, "t.fa")
        open(rp, "wb").write(rfa)
        open(tp, "wb").write(tfa)
        subprocess.run([binary, rp, tp, os.path.join(d, "o")], env=env, stdout=subprocess.DEVNULL,
                       stderr=subprocess.DEVNULL, check=True)
        return open(os.path.join(d, "o", "compressed_genome.txt"), "rb").read()


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_BIN, "compression_k21_m100")),
                    reason="reference k=21 variant not built (make -C oracle ref-param K=21)")
@pytest.mark.parametrize("seed", range(200, 212))
def test_param_k21_differential_vs_reference(seed):
    rfa, tfa = fuzzgen.global_case(seed)
    assert oraclelib.compress_params(rfa, tfa, k=21) == _run_ref_param(21, 100, rfa, tfa)


def test_param_local0_is_the_global_pass():
    """local = 0 gives the global pass alone: on a case the reference switches on, the same text."""
    for seed in range(4):
        rfa, tfa = fuzzgen.global_case(seed)
        rec = oraclelib.compress(rfa, tfa)
        if oraclelib.last_mode()[0]:
            assert oraclelib.compress_params(rfa, tfa, local=0) == rec
