"""GPU: the non-parity parameter overrides (sccg_params, include/sccg.h).

The reference hard-codes k = 14, m = 100 (compression.cpp:373-379).  Other values have no reference
output of their own, so the chain of evidence is
  * tests/golden/params.json.gz: the reference compiled with other k / m (make_param_golden.py);
    test_oracle_golden.py::test_param_fixtures pins the oracle's orc_compress_params to it;
  * here: the GPU against those fixtures where it runs the same controller (local = 1, m override),
    and against the pinned oracle for the global walk at other k (local = 0, 1 <= k <= 32), plus
    round trips through the (parameter-free) decompression.
"""
import random

import pytest

import fuzzgen
import goldens
import oraclelib
import synthlib
from pkg import sccg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = sccg.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("case", [c for c in goldens.param_cases() if c["k"] == 14],
                         ids=lambda c: f"m{c['m']}-{c['gen']}{c['seed']}")
def test_m_override_vs_reference_variant(ctx, case):
    rfa, tfa = goldens.param_inputs(case)
    assert case["compress_rc"] == 0
    assert ctx.compress(rfa, tfa, m=case["m"]) == case["record"]


@pytest.mark.parametrize("k", [4, 8, 12, 15, 16, 17, 21, 24, 32])
@pytest.mark.parametrize("seed", range(6))
def test_global_k_vs_oracle(ctx, k, seed):
    rfa, tfa = fuzzgen.global_case(seed)
    want = oraclelib.compress_params(rfa, tfa, k=k, local=0)
    got = ctx.compress(rfa, tfa, k=k, local=0)
    assert got == want
    assert ctx.stats()["mode_global"] == 1
    assert ctx.reconstruct(got, rfa) == oraclelib.decompress(want, rfa)


@pytest.mark.parametrize("k,m", [(21, 100), (21, 30), (18, 127), (32, 0), (16, 64)])
def test_global_k_m_medium_vs_oracle(ctx, k, m):
    rfa, tfa = synthlib.synth_pair("hg", 2_000_000, 2_003_000, 5 + k)
    assert ctx.compress(rfa, tfa, k=k, m=m, local=0) == oraclelib.compress_params(rfa, tfa, k=k, m=m, local=0)


@pytest.mark.parametrize("k", [21, 28])
def test_t2t_k_vs_oracle(ctx, k):
    """Literal-heavy (stuck) walks: frozen chunks and chains with the longer keys."""
    rfa, tfa = synthlib.synth_pair("t2t", 1_000_000, 1_000_000, 40 + k)
    assert ctx.compress(rfa, tfa, k=k, local=0) == oraclelib.compress_params(rfa, tfa, k=k, local=0)


def test_local0_k14_equals_switched_default(ctx):
    """local = 0 at the reference's k: the same text the default pipeline writes after a switch."""
    rfa, tfa = synthlib.synth_pair("hg", 1_000_000, 1_002_000, 3)
    rec = ctx.compress(rfa, tfa)
    assert ctx.stats()["mode_global"] == 1
    assert ctx.compress(rfa, tfa, local=0) == rec


@pytest.mark.parametrize("seed", range(12))
def test_match_seam_global_k(ctx, seed):
    rng = random.Random(5000 + seed)
    k = rng.choice([16, 17, 20, 21, 25, 31, 32])
    n = rng.randint(2000, 30000)
    sr = bytearray(rng.choice(b"ACGT") for _ in range(n))
    for _ in range(n // 300):   # repeats whose first KEY_K bases agree but whose k-mers do not
        a, b = rng.randrange(n - 40), rng.randrange(n - 40)
        sr[b:b + 15] = sr[a:a + 15]
    sr = bytes(sr)
    st = bytearray(sr)
    for i in range(len(st)):
        if rng.random() < 0.01:
            st[i] = rng.choice(b"ACGTN")
    cut = rng.randint(0, len(st))
    st = bytes(st[:cut]) + bytes(rng.choice(b"ACGT") for _ in range(rng.randint(0, 2000))) + bytes(st[cut:])
    assert ctx.match(sr, st, k, 100, True) == oraclelib.match(sr, st, k, 100, True)


def test_unsupported_params(ctx):
    rfa, tfa = fuzzgen.global_case(0)
    for bad in ({"k": 21}, {"k2": 9}, {"L": 500}, {"T2": 3}, {"m": 128, "local": 0}, {"k": 33, "local": 0},
                {"k": 0, "local": 0}):
        with pytest.raises(sccg.SccgError) as e:
            ctx.compress(rfa, tfa, **bad)
        assert e.value.rc == 8   # SCCG_E_UNSUPPORTED


def test_chr1_k21_roundtrip(ctx):
    """BASELINE configs[1] names k = 21: the chr1-sized pair through the global walk at k = 21
    (local = 0) must decompress to the input FASTA."""
    rfa, tfa = synthlib.synth_pair("hg", 247_249_719, 249_250_621, 1)
    rec = ctx.compress(rfa, tfa, k=21, local=0)
    st = ctx.stats()
    assert st["mode_global"] == 1 and st["target_bases"] == 249_250_621
    assert ctx.reconstruct(rec, rfa) == tfa
