"""GPU parity: the HIP path (through the C ABI) against the reference's fixtures and the oracle.

* every golden fixture (outputs of the compiled reference) byte-for-byte, compression and
  decompression, exit-code behaviour included;
* the larger generator seeds against the reference's sha256 (synth_manifest.json);
* seeded fuzz pairs against the CPU restatement (oracle/), local and global modes;
* the match_sequences seam (compression.cpp:36) against the oracle's records;
* full-size (chr1-shaped) round trip compress -> reconstruct == input FASTA.
"""
import hashlib
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


def _gpu_compress(ctx, rfa, tfa):
    try:
        return ctx.compress(rfa, tfa), 0
    except sccg.SccgError as e:
        return getattr(e, "partial", None), 1


def test_golden_compress(ctx, golden_cases):
    bad = []
    for c in golden_cases:
        rec, rc = _gpu_compress(ctx, c["ref_fa"], c["tgt_fa"])
        if rc != c["compress_rc"] or rec != c["record"]:
            bad.append(c["name"])
    assert not bad, bad


def test_golden_reconstruct(ctx, golden_cases):
    bad = []
    for c in golden_cases:
        if c["decompress_rc"] is None:
            continue
        try:
            fa, rc = ctx.reconstruct(c["record"], c["ref_fa"]), 0
        except sccg.SccgError:
            fa, rc = None, 1
        if rc != c["decompress_rc"] or (rc == 0 and fa != c["fasta"]):
            bad.append(c["name"])
    assert not bad, bad


@pytest.mark.parametrize("entry", goldens.synth_manifest(), ids=lambda e: f"{e['profile']}-{e['seed']}")
def test_synth_manifest(ctx, entry):
    rfa, tfa = synthlib.synth_pair(entry["profile"], entry["ref_len"], entry["tgt_len"], entry["seed"])
    rec = ctx.compress(rfa, tfa)
    assert len(rec) == entry["record_len"]
    assert hashlib.sha256(rec).hexdigest() == entry["record_sha256"]
    fa = ctx.reconstruct(rec, rfa)
    assert hashlib.sha256(fa).hexdigest() == entry["fasta_sha256"]


@pytest.mark.parametrize("kind,seed", [("local", s) for s in range(300, 340)] +
                         [("global", s) for s in range(300, 330)])
def test_fuzz_vs_oracle(ctx, kind, seed):
    rfa, tfa = (fuzzgen.local_case if kind == "local" else fuzzgen.global_case)(seed)
    want = oraclelib.compress(rfa, tfa)
    got, rc = _gpu_compress(ctx, rfa, tfa)
    assert rc == 0
    assert got == want
    assert _gpu_reconstruct(ctx, got, rfa) == _oracle_reconstruct(want, rfa)


def _gpu_reconstruct(ctx, rec, rfa):
    try:
        return 0, ctx.reconstruct(rec, rfa)
    except sccg.SccgError:
        return 1, None


def _oracle_reconstruct(rec, rfa):
    try:
        return 0, oraclelib.decompress(rec, rfa)
    except oraclelib.OracleError:
        return 1, None


def _rand(rng, n, alpha="ACGT"):
    return "".join(rng.choice(alpha) for _ in range(n)).encode()


@pytest.mark.parametrize("seed", range(40))
def test_match_seam_local(ctx, seed):
    rng = random.Random(seed)
    n = rng.choice([5, 13, 200, 999, 1000])
    sr = _rand(rng, n, rng.choice(["ACGT", "AC", "ACGTN", "A"]))
    st = bytearray(sr[: rng.randint(0, n)] + _rand(rng, rng.randint(0, 1000 - min(n, 1000)) // 2))
    for i in range(len(st)):
        if rng.random() < 0.02:
            st[i] = ord(rng.choice("ACGTNR"))
    st = bytes(st[:1000])
    for k in (14, 10):
        assert ctx.match(sr, st, k, 0, False, 1000 * seed) == oraclelib.match(sr, st, k, 0, False, 1000 * seed)


@pytest.mark.parametrize("seed", range(30))
def test_match_seam_global(ctx, seed):
    rng = random.Random(1000 + seed)
    n = rng.randint(2000, 40000)
    unit = _rand(rng, rng.randint(10, 200))
    sr = b"".join(unit if rng.random() < 0.2 else _rand(rng, rng.randint(20, 400)) for _ in range(n // 150))
    st = bytearray(sr)
    for i in range(len(st)):
        if rng.random() < 0.01:
            st[i] = ord(rng.choice("ACGT"))
    cut = rng.randint(0, len(st))
    st = bytes(st[:cut]) + _rand(rng, rng.randint(0, 3000)) + bytes(st[cut + rng.choice([0, 50, 300]):])
    assert ctx.match(sr, st, 14, 100, True) == oraclelib.match(sr, st, 14, 100, True)


def test_synth_medium_vs_oracle(ctx):
    rfa, tfa = synthlib.synth_pair("hg", 12_000_000, 12_030_000, 77)
    want = oraclelib.compress(rfa, tfa)
    assert ctx.compress(rfa, tfa) == want
    assert ctx.stats()["mode_global"] == 1


def test_t2t_vs_oracle(ctx):
    rfa, tfa = synthlib.synth_pair("t2t", 3_000_000, 3_000_000, 78)
    assert ctx.compress(rfa, tfa) == oraclelib.compress(rfa, tfa)


def test_local_large_vs_oracle(ctx):
    rfa, tfa = synthlib.synth_pair("local", 10_000_000, 10_000_000, 79)
    assert ctx.compress(rfa, tfa) == oraclelib.compress(rfa, tfa)
    assert ctx.stats()["mode_global"] == 0


def test_chr1_roundtrip(ctx):
    """Full BASELINE config size: compress then reconstruct must give back the input FASTA
    (the generator writes 50-column LF FASTA with a header, so the round trip is byte-exact)."""
    rfa, tfa = synthlib.synth_pair("hg", 247_249_719, 249_250_621, 1)
    rec = ctx.compress(rfa, tfa)
    st = ctx.stats()
    assert st["mode_global"] == 1 and st["target_bases"] == 249_250_621
    assert ctx.reconstruct(rec, rfa) == tfa


def _switch_case(seed: int, nseg: int = 2400, plant_at=None, gap=None):
    """Segment-kind patterns for the local->global switch (compression.cpp:462-473): identical
    segments (good), unrelated random ones (failed or mostly literal), half-copied ones (matched
    but > 50 % literal), all-N ones (failed, all N: resets the counter) and poly-A ones (failed,
    not N), in bursts of 1-3, with a planted 5-burst ending in a failure at a seed-dependent
    segment (or none).  gap = (start, length, kinds): a long run of segments drawn from `kinds`
    (e.g. only half-copied ones, or all-N: unproved segments that never switch)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    r = acgt[rng.integers(0, 4, nseg * 1000)]
    t = r.copy()
    kinds = np.zeros(nseg, dtype=np.int8)   # 0 copy, 1 random, 2 half, 3 N, 4 poly-A (fails)
    i = 0
    while i < nseg:
        i += int(rng.integers(2, 40))
        n = int(rng.integers(1, 4))   # bursts too short to switch on their own ...
        kinds[i:i + n] = rng.choice([1, 2, 3, 4], size=min(n, max(0, nseg - i)))
        i += n
    if gap is not None:
        g0, gl, gk = gap
        kinds[g0:g0 + gl] = rng.choice(list(gk), size=len(kinds[g0:g0 + gl]))
    plant = [None, 4, 5, 9, 63, 64, 65, 1000, 4095, nseg - 1][seed % 10] if plant_at is None else plant_at
    for p in (plant if isinstance(plant, (list, tuple)) else [plant]):   # (several windows: a list)
        if p is not None and p < nseg:
            kinds[max(0, p - 4):p + 1] = rng.choice([1, 2, 4], size=min(p + 1, 5))   # ... but this one
            kinds[p] = 4
    for s, k in enumerate(kinds):
        seg = slice(s * 1000, (s + 1) * 1000)
        if k == 1:
            t[seg] = acgt[rng.integers(0, 4, 1000)]
        elif k == 2:
            t[s * 1000 + 400:(s + 1) * 1000] = acgt[rng.integers(0, 4, 600)]
        elif k == 3:
            t[seg] = ord("N")
        elif k == 4:
            t[seg] = ord("A")
    fa = lambda name, x: b">" + name + b"\n" + b"\n".join(x[j:j + 60].tobytes() for j in range(0, len(x), 60)) + b"\n"
    return fa(b"r", r), fa(b"t", t)


class _exact:
    """The context in SCCG_OPT_EXACT_SWITCH mode for one test (stats report the first switch)."""

    def __init__(self, ctx, on=True):
        self.ctx, self.on = ctx, on

    def __enter__(self):
        self.ctx.exact_switch(self.on)

    def __exit__(self, *a):
        self.ctx.exact_switch(False)


def _probe_runs(nseg: int) -> list[range]:
    """The segment runs local.hip's k_local_probe classifies (PROBE_RUN 8, PROBE_RUNS 16, run r
    from (r + 1) nseg / 17 - 4; pairs of at least 512 segments)."""
    if nseg < 512:
        return []
    return [range(a, a + 8) for a in ((j + 1) * nseg // 17 - 4 for j in range(16))]


@pytest.mark.parametrize("exact", [True, False], ids=["exact", "probe"])
@pytest.mark.parametrize("seed", range(20))
def test_switch_window_vs_oracle(ctx, seed, exact):
    """The fused local kernel's switch detection against the oracle's state machine: the exact
    first switch in SCCG_OPT_EXACT_SWITCH mode; the default mode's probe reports a switch window
    at or after it (the record bytes and the mode are the same)."""
    rfa, tfa = _switch_case(seed)
    want = oraclelib.compress(rfa, tfa)
    mode_global, sw = oraclelib.last_mode()
    with _exact(ctx, exact):
        got, rc = _gpu_compress(ctx, rfa, tfa)
        st = ctx.stats()
    assert rc == 0
    assert bool(st["mode_global"]) == mode_global
    if exact or not mode_global:
        assert st["switch_segment"] == (sw if mode_global else -1)
    else:
        assert st["switch_segment"] >= sw
    assert got == want


# (nseg, planted windows): a first window the probe does not see and a later one inside probe run
# 0 / 8 / 15, a window only inside a probe run, windows straddling a run's first or last segment
# (its 5 segments are not all inside the run: the probe must not count it) and one at the last
# segment (no run covers the pair's end)
PROBE_CASES = [(2400, [40, 143]), (2400, [300, 1272]), (2400, [40, 2260]), (2400, [1274]), (2400, [2399]),
               (2400, [138]), (17000, [3000, 16003]), (17000, [10000])]


@pytest.mark.parametrize("nseg,plants", PROBE_CASES)
def test_switch_probe_vs_oracle(ctx, nseg, plants):
    """The mode probe (local.hip k_local_probe): a window inside a probed run decides the mode at
    once, and the record file equals the reference's wherever the first switch lies
    (compression.cpp:462-473 truncates the file, :484-574 regenerates it); with
    SCCG_OPT_EXACT_SWITCH the first switch is reported."""
    rfa, tfa = _switch_case(900 + nseg % 7 + plants[0], nseg=nseg, plant_at=plants)
    want = oraclelib.compress(rfa, tfa)
    mode_global, sw = oraclelib.last_mode()
    assert mode_global
    got, rc = _gpu_compress(ctx, rfa, tfa)
    st = ctx.stats()
    assert rc == 0 and got == want
    assert st["mode_global"] == 1 and st["switch_segment"] >= sw
    in_run = [r for r in _probe_runs(nseg) if st["switch_segment"] in r]
    if st["switch_segment"] != sw:   # a later window: the probe's, inside one of its runs
        assert in_run and st["switch_segment"] - 4 >= in_run[0].start
    with _exact(ctx):
        got2, rc2 = _gpu_compress(ctx, rfa, tfa)
        st2 = ctx.stats()
    assert rc2 == 0 and got2 == want and st2["switch_segment"] == sw


@pytest.mark.parametrize("seed", range(16, 64))
def test_paren_vs_oracle(ctx, seed):
    """Targets whose literals hold '(' ')' ',' digits: delta_encode's own token scan
    (compression.cpp:262-293, delta.hip), including its stoi failures (rc 1, absolute text)."""
    rfa, tfa = fuzzgen.paren_case(seed)
    try:
        want, wrc = oraclelib.compress(rfa, tfa), 0
    except oraclelib.OracleError as e:
        want, wrc = e.partial, 1
    got, rc = _gpu_compress(ctx, rfa, tfa)
    assert (rc, got) == (wrc, want)
    if rc == 0:
        assert _gpu_reconstruct(ctx, got, rfa) == _oracle_reconstruct(want, rfa)


@pytest.mark.parametrize("seed", range(24))
def test_close_paren_literals_vs_oracle(ctx, seed):
    """Targets whose only punctuation is ')': the record line holds ')' outside every token, which
    decompression.cpp:231-234 copies as a literal byte (round trip exact where the oracle's is)."""
    rfa, tfa = fuzzgen.close_paren_case(seed)
    want = oraclelib.compress(rfa, tfa)
    got, rc = _gpu_compress(ctx, rfa, tfa)
    assert (rc, got) == (0, want)
    assert _gpu_reconstruct(ctx, got, rfa) == _oracle_reconstruct(want, rfa)


@pytest.mark.parametrize("period", [1, 2, 3, 7])
def test_dense_case_and_n_alternation(ctx, period):
    """Soft-masking and N that flip every `period` bases over long stretches: up to one run per two
    bases in a formatter span (decompression.cpp:241-262 run lists), round trip exact."""
    rng = random.Random(900 + period)
    ref = _rand(rng, 300_000).decode()
    tgt = list(ref[:150_000] + _rand(rng, 3000).decode() + ref[150_000:])
    for i in range(20_000, 120_000):
        if (i // period) % 2:
            tgt[i] = tgt[i].lower()
    for i in range(200_000, 260_000, 2 * period):
        tgt[i] = "N" if (i // 7) % 2 else "n"
    rfa, tfa = fuzzgen.to_fasta(ref), fuzzgen.to_fasta("".join(tgt), ">alt")
    want = oraclelib.compress(rfa, tfa)
    got, rc = _gpu_compress(ctx, rfa, tfa)
    assert (rc, got) == (0, want)
    fa = ctx.reconstruct(got, rfa)
    assert fa == oraclelib.decompress(want, rfa)


@pytest.mark.parametrize("seed", range(4))
def test_token_copy_alignments(ctx, seed):
    """Record lines built by hand: tokens of length 0..70 (and some to 3000) at every source and
    destination alignment between literal runs of 1-5 bases, so the wave copy's byte head, 16-byte
    body and byte tail all meet every offset (decompression.cpp:210-236)."""
    rng = random.Random(700 + seed)
    ref = "".join(rng.choice("ACGT") for _ in range(20_000))
    rfa = fuzzgen.to_fasta(ref)
    toks, prev = [], 0
    for _ in range(3000):
        if rng.random() < 0.3:
            toks.append(rng.choice("ACGT") * rng.randint(1, 5))
        else:
            ln = rng.randint(0, 70) if rng.random() < 0.8 else rng.randint(70, 3000)
            p = rng.randint(0, len(ref) - ln)
            toks.append(f"({p - prev},{ln})")
            prev = p
    rec = ("\n\n" + "".join(toks)).encode()
    assert ctx.reconstruct(rec, rfa) == oraclelib.decompress(rec, rfa)


@pytest.mark.parametrize("seed", range(3))
def test_token_dense_blocks(ctx, seed):
    """Record lines whose 4 KiB output blocks hold hundreds of tokens of length 0..3 (the fused
    formatter stages up to 128 tokens per block in LDS and searches the global table beyond that),
    mixed with N / lowercase runs and literals, against the oracle (decompression.cpp:210-274)."""
    rng = random.Random(900 + seed)
    ref = "".join(rng.choice("ACGT") for _ in range(5_000))
    rfa = fuzzgen.to_fasta(ref)
    toks, prev, dec_len = [], 0, 0
    for _ in range(20_000):
        if rng.random() < 0.1:
            lit = rng.choice("ACGT") * rng.randint(1, 3)
            toks.append(lit)
            dec_len += len(lit)
        else:
            ln = rng.randint(0, 3)
            p = rng.randint(0, len(ref) - ln)
            toks.append(f"({p - prev},{ln})")
            prev = p
            dec_len += ln
    lower = f"(100,{dec_len // 3})" if seed else ""
    nline = "(50,7)" if seed == 2 else ""
    rec = (f"{lower}\n{nline}\n" + "".join(toks)).encode()
    assert ctx.reconstruct(rec, rfa) == oraclelib.decompress(rec, rfa)


_RUN_LINE_CASES = {
    "empty_lines": b"\n\n(0,10)", "one_n": b"\n(5,3)\n(0,10)", "lower_and_n": b"(2,4)\n(5,3)\n(0,10)AC",
    "n_tail": b"\n(10,2)\n(0,10)", "n_past": b"\n(20,5)\n(0,3)", "lower_singleton": b"7\n\n(0,10)",
    "n_items": b"\n1,3,2\n(0,10)", "hdr": b">chrX\n(1,2)\n(3,1)\n(0,10)", "lower_all": b"(0,10)\n\n(0,10)",
    "n_only": b"\n(0,4)\n", "many_runs": ("".join(f"{1 if i else 0}," for i in range(40))[:-1] + "\n\n(0,100)").encode(),
}


@pytest.mark.parametrize("name", sorted(_RUN_LINE_CASES))
def test_run_line_edges(ctx, name):
    """Hand-built run lines (decompression.cpp:126-207, :241-262): empty lines, singletons, a run at
    the sequence end, one past it (an error on both sides), a header; the run counts stay on the
    device and are read back once with the record line's."""
    rng = random.Random(1)
    rfa = fuzzgen.to_fasta("".join(rng.choice("ACGT") for _ in range(200)))
    rec = _RUN_LINE_CASES[name]
    try:
        want = oraclelib.decompress(rec, rfa)
    except oraclelib.OracleError:   # the reference exits 1 (or its behaviour is undefined)
        want = None
    if want is None:
        with pytest.raises(sccg.SccgError):
            ctx.reconstruct(rec, rfa)
    else:
        assert ctx.reconstruct(rec, rfa) == want


@pytest.mark.parametrize("pieces", ["safe", "mixed"])
def test_paren_large_vs_oracle(ctx, pieces):
    """Multi-tile scans of the paren path: a 3 Mb global-mode pair with punctuation literals."""
    import numpy as np
    rfa, tfa = synthlib.synth_pair("hg", 3_000_000, 3_010_000, 91)
    rng = np.random.default_rng(5 if pieces == "safe" else 6)
    pool = fuzzgen.SAFE_PIECES if pieces == "safe" else fuzzgen.SAFE_PIECES * 200 + fuzzgen.BAD_PIECES
    lines = tfa.split(b"\n")
    for j in rng.integers(1, len(lines) - 1, 3000):
        ln = lines[j]
        if ln and not ln.startswith(b">"):
            c = int(rng.integers(0, len(ln)))
            lines[j] = ln[:c] + pool[int(rng.integers(0, len(pool)))].encode() + ln[c:]
    tfa = b"\n".join(lines)
    try:
        want, wrc = oraclelib.compress(rfa, tfa), 0
    except oraclelib.OracleError as e:
        want, wrc = e.partial, 1
    got, rc = _gpu_compress(ctx, rfa, tfa)
    assert rc == wrc
    assert got == want


def test_trapped_chain_vs_oracle(ctx):
    """chr22-shaped pair (hg18/hg19 lengths, seed 22): from ~45.8 Mb on the reference walk is trapped
    on a poly-A window (chance hits keep nudging P), the case the walk re-speculates chunks for."""
    rfa, tfa = synthlib.synth_pair("hg", 49_691_432, 51_304_566, 22)
    got = ctx.compress(rfa, tfa)
    assert ctx.stats()["walk_rounds"] < 40
    assert got == oraclelib.compress(rfa, tfa)


def test_chr21_vs_oracle(ctx):
    """BASELINE configs[0] size: hg18/hg19 chr21 lengths (46.9 / 48.1 Mb), seed 21."""
    rfa, tfa = synthlib.synth_pair("hg", 46_944_323, 48_129_895, 21)
    assert ctx.compress(rfa, tfa) == oraclelib.compress(rfa, tfa)
    assert ctx.stats()["mode_global"] == 1


@pytest.mark.parametrize("seed", [81, 82, 83])
def test_t2t_seeds_vs_oracle(ctx, seed):
    """Literal-heavy walks (frozen and trapped chains, long literal gaps) at 4 Mb."""
    rfa, tfa = synthlib.synth_pair("t2t", 4_000_000, 4_000_000, seed)
    assert ctx.compress(rfa, tfa) == oraclelib.compress(rfa, tfa)


@pytest.mark.parametrize("seed", [7, 90])
def test_frozen_chains_vs_oracle(ctx, seed):
    """T2T-shaped pairs whose reference walk freezes right after its first step: the frozen-chain
    kernels (k_chain_scan / k_chain_step / k_chain_fill) walk most of the target; the record stream
    must still equal the oracle's."""
    rfa, tfa = synthlib.synth_pair("t2t", 8_000_000, 8_000_000, seed)
    got = ctx.compress(rfa, tfa)
    st = ctx.stats()
    assert st["walk_chains"] >= 1
    assert got == oraclelib.compress(rfa, tfa)


def _layout_fasta(rng, seq: str, case: str) -> bytes:
    """A target FASTA with an awkward byte layout around the run boundaries the strip emits."""
    if case == "crlf_ragged":   # CRLF, line widths 1..120, blank lines
        out, i = [">t crlf\r\n"], 0
        while i < len(seq):
            w = rng.randint(1, 120)
            out.append(seq[i:i + w] + "\r\n" + ("\r\n" if rng.random() < 0.05 else ""))
            i += w
        return "".join(out).encode()
    if case == "whitespace_gulfs":   # stretches of blank lines longer than 64 strip tiles inside runs
        gulf = "\n" * (70 * 4096 + 13)
        cut = [len(seq) // 5, len(seq) // 2, 4 * len(seq) // 5]
        parts, prev = [], 0
        for c in cut:
            parts.append(seq[prev:c])
            prev = c
        parts.append(seq[prev:])
        return (">t gulfs\n" + gulf.join(fuzzgen.to_fasta(p, None, 60).decode() for p in parts)).encode()
    if case == "tile_edges":   # newlines and run boundaries at strip-tile (4 KiB) edges, a long header
        hdr = ">" + "h" * 5000 + "\n"
        body = fuzzgen.to_fasta(seq, None, 4095).decode()   # lines of 4095 + '\n' = one tile each
        return (hdr + body).encode()
    if case == "no_final_newline":
        return fuzzgen.to_fasta(seq, ">t", 61, trailing_newline=False)
    raise ValueError(case)


@pytest.mark.parametrize("case", ["crlf_ragged", "whitespace_gulfs", "tile_edges", "no_final_newline"])
@pytest.mark.parametrize("seed", range(2))
def test_strip_run_events_vs_oracle(ctx, case, seed):
    """The target strip emits both run lines' boundaries (lowercase, compression.cpp:341-368; N,
    :527-555) per 4 KiB tile; runs that cross tiles, dropped bytes (CR, LF, blank-line gulfs wider
    than the tile look-back, a header longer than a tile) and runs open at the target's end must
    give the oracle's lines byte for byte (the record text holds both)."""
    rng = random.Random(1300 + seed)
    ref = _rand(rng, 400_000).decode()
    tgt = list(ref[:200_000] + _rand(rng, 2000).decode() + ref[200_000:])
    i = 0
    while i < len(tgt):   # soft-masked runs and N runs of every length, some across tile edges
        ln = rng.choice([1, 2, 3, 50, 700, 4096, 9000])
        kind = rng.random()
        for q in range(i, min(len(tgt), i + ln)):
            if kind < 0.35:
                tgt[q] = tgt[q].lower()
            elif kind < 0.45:
                tgt[q] = "N" if rng.random() < 0.9 else "n"
        i += ln + rng.choice([0, 1, 5, 300, 3000])
    for q in range(len(tgt) - 777, len(tgt)):   # a lowercase run open at the end
        tgt[q] = tgt[q].lower()
    rfa = fuzzgen.to_fasta(ref)
    tfa = _layout_fasta(rng, "".join(tgt), case)
    want = oraclelib.compress(rfa, tfa)
    got, rc = _gpu_compress(ctx, rfa, tfa)
    assert (rc, got) == (0, want)


def test_walk_rounds_deterministic(ctx, monkeypatch):
    """With deterministic anchor slots (SCCG_ANCHOR_DET=1: atomicMax) and the frozen / carry lists and
    trapped triggers in chunk order, a T2T-like pair (frozen and trapped stretches, many rounds) takes
    the same number of rounds and chains in every call, in this context and in a fresh one, and the
    record equals the oracle's."""
    monkeypatch.setenv("SCCG_ANCHOR_DET", "1")
    rfa, tfa = synthlib.synth_pair("t2t", 12_000_000, 12_000_000, 91)
    got, rounds = None, set()
    for _ in range(3):
        rec = ctx.compress(rfa, tfa)
        st = ctx.stats()
        rounds.add((st["walk_rounds"], st["walk_chains"]))
        got = got or rec
        assert rec == got
    with sccg.Context(0) as c2:
        assert c2.compress(rfa, tfa) == got
        st = c2.stats()
        rounds.add((st["walk_rounds"], st["walk_chains"]))
    assert len(rounds) == 1, rounds
    assert got == oraclelib.compress(rfa, tfa)


@pytest.mark.parametrize("plant", [16382, 16386, 16900, None])
def test_switch_deep_vs_oracle(ctx, plant):
    """Deep switch windows in a 17,000-segment pair (more segments than the pass has waves in
    flight: segments past a found switch are skipped, earlier ones finish) and a pair that stays
    local (every proved segment's records computed afterwards) -- against the oracle's state
    machine."""
    rfa, tfa = _switch_case(700 + (plant or 0) % 97, nseg=17000, plant_at=plant)
    want = oraclelib.compress(rfa, tfa)
    mode_global, sw = oraclelib.last_mode()
    with _exact(ctx):
        got, rc = _gpu_compress(ctx, rfa, tfa)
        st = ctx.stats()
    assert rc == 0
    assert bool(st["mode_global"]) == mode_global
    assert st["switch_segment"] == (sw if mode_global else -1)
    assert got == want
    got2, rc2 = _gpu_compress(ctx, rfa, tfa)   # default mode: the same bytes
    assert rc2 == 0 and got2 == want and ctx.stats()["mode_global"] == int(mode_global)


@pytest.mark.parametrize("kind", ["global", "local", "local0_params"])
def test_lean_strip_overflow_vs_oracle(ctx, kind):
    """Lean strips (round 6): a pair of >= 512 segments has its mode decided by the switch probe, so
    its strips write only T' and R' -- the probe gathers its segments of T and R from the FASTA, a
    pair that stays local gets T and R from a second write pass, and a tile with more run events
    than its slots (alternating case: a boundary every base) takes the run-line fallback over T,
    which writes T first.  Drifted (global), identical (stays local) and local = 0 pairs, each with
    an overflowing tile and N runs, against the oracle."""
    rng = random.Random({"global": 7, "local": 8, "local0_params": 9}[kind])
    ref = list(_rand(rng, 700_000).decode())
    if kind == "global":   # a 1.5 kb insertion every ~40 kb: segments drift apart
        tgt = []
        for i in range(0, len(ref), 40_000):
            tgt += ref[i:i + 40_000] + list(_rand(rng, 1500).decode())
    else:
        tgt = list(ref)
    for q in range(300_000, 312_000):   # alternating case: a run boundary at every base
        if q % 2:
            tgt[q] = tgt[q].lower()
    for a, ln in ((100_000, 5000), (450_001, 37), (650_000, 1)):
        for q in range(a, a + ln):
            tgt[q] = "N"
    rfa = fuzzgen.to_fasta("".join(ref))
    tfa = fuzzgen.to_fasta("".join(tgt))
    if kind == "local0_params":
        want = oraclelib.compress_params(rfa, tfa, local=0)
        got = ctx.compress(rfa, tfa, local=0)
        assert got == want
        return
    want = oraclelib.compress(rfa, tfa)
    mode_global, _ = oraclelib.last_mode()
    assert mode_global == (kind == "global")
    got, rc = _gpu_compress(ctx, rfa, tfa)
    assert (rc, got) == (0, want)
    assert ctx.stats()["mode_global"] == int(mode_global)
