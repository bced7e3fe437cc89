"""Small adversarial FASTA pairs for parity tests.

Pure-Python, seeded, deterministic.  Each generator returns (ref_fa: bytes, tgt_fa: bytes).
Large inputs come from the C generator (sccg-genome-compression_amd/tools/synth.c) instead.
"""
from __future__ import annotations

import random

ACGT = "ACGT"


def rand_seq(rng: random.Random, n: int, alphabet: str = ACGT) -> str:
    return "".join(rng.choice(alphabet) for _ in range(n))


def to_fasta(seq: str, header: str | None = ">seq", width: int = 50, crlf: bool = False,
             trailing_newline: bool = True) -> bytes:
    nl = "\r\n" if crlf else "\n"
    lines = []
    if header is not None:
        lines.append(header)
    for i in range(0, len(seq), width):
        lines.append(seq[i:i + width])
    text = nl.join(lines)
    if trailing_newline and lines:
        text += nl
    return text.encode("latin-1")


def mutate(rng: random.Random, s: str, snp: float = 0.01, indel: float = 0.002,
           max_indel: int = 8) -> str:
    out = []
    i = 0
    while i < len(s):
        u = rng.random()
        if u < snp:
            out.append(rng.choice([b for b in ACGT if b != s[i].upper()]))
            i += 1
        elif u < snp + indel:
            n = rng.randint(1, max_indel)
            if rng.random() < 0.5:
                out.append(rand_seq(rng, n))
            else:
                i += n
        else:
            out.append(s[i])
            i += 1
    return "".join(out)


def soft_mask(rng: random.Random, s: str, frac: float = 0.3) -> str:
    b = list(s)
    i = 0
    while i < len(b):
        i += rng.randint(0, 60)
        n = rng.randint(1, 40)
        if rng.random() < frac * 2:
            for j in range(i, min(i + n, len(b))):
                b[j] = b[j].lower()
        i += n
    return "".join(b)


def local_case(seed: int) -> tuple[bytes, bytes]:
    """Survey's local-mode fuzz: lengths 0-7000, widths 7/50/60/80, CRLF/LF, headers, a second
    '>' record, IUPAC, N blocks, lowercase, tandem duplications, indels."""
    rng = random.Random(seed)
    n = rng.choice([0, 5, 13, 600, 999, 1000, 1001, 2500, 4000, 7000])
    ref = rand_seq(rng, n)
    if rng.random() < 0.3 and n > 200:          # tandem duplication in the reference
        a = rng.randint(0, n - 100)
        ref = ref[:a] + ref[a:a + 50] * 3 + ref[a + 150:]
    tgt = mutate(rng, ref, snp=rng.choice([0.0, 0.002, 0.02, 0.3]), indel=rng.choice([0.0, 0.0005]))
    if rng.random() < 0.3 and len(tgt) > 100:   # N block
        a = rng.randint(0, len(tgt) - 50)
        tgt = tgt[:a] + "N" * rng.randint(1, 1200) + tgt[a:]
    if rng.random() < 0.2 and len(ref) > 100:
        a = rng.randint(0, len(ref) - 50)
        ref = ref[:a] + "N" * rng.randint(1, 300) + ref[a:]
    if rng.random() < 0.2 and tgt:              # IUPAC codes
        tgt = "".join(c if rng.random() > 0.01 else rng.choice("RYKMSWn") for c in tgt)
    if rng.random() < 0.5:
        tgt = soft_mask(rng, tgt)
    if rng.random() < 0.3:
        ref = soft_mask(rng, ref)
    width = rng.choice([7, 50, 60, 80])
    crlf = rng.random() < 0.25
    hdr = rng.choice([">tgt chr1", None, ">x"])
    tfa = to_fasta(tgt, hdr, width, crlf)
    if rng.random() < 0.2:                      # a second record: its '>' line becomes sequence
        tfa += to_fasta(soft_mask(rng, rand_seq(rng, rng.randint(1, 300))), ">second rec", width, crlf)
    rfa = to_fasta(ref, rng.choice([">ref", None]), rng.choice([50, 60, 70]), rng.random() < 0.2)
    return rfa, tfa


def global_case(seed: int) -> tuple[bytes, bytes]:
    """Survey's global-mode fuzz: repeat-rich references of 3-30 kb, an early 1.5-6 kb insertion
    (forces the switch), >150-bp deletions (stuck walks), N runs, SNPs."""
    rng = random.Random(10_000 + seed)
    n = rng.randint(3000, 30000)
    unit = rand_seq(rng, rng.randint(20, 300))
    parts = []
    while sum(map(len, parts)) < n:
        if rng.random() < 0.25:
            parts.append(mutate(rng, unit, snp=0.05, indel=0.0))
        elif rng.random() < 0.1:
            parts.append("A" * rng.randint(14, 40))
        else:
            parts.append(rand_seq(rng, rng.randint(50, 800)))
    ref = "".join(parts)[:n]
    tgt = mutate(rng, ref, snp=rng.choice([0.001, 0.01, 0.03]), indel=0.0005, max_indel=20)
    a = rng.randint(0, min(3000, len(tgt)))
    tgt = tgt[:a] + rand_seq(rng, rng.randint(1500, 6000)) + tgt[a:]
    for _ in range(rng.choice([0, 0, 1, 2])):
        if len(tgt) > 2000:
            d = rng.randint(0, len(tgt) - 1000)
            tgt = tgt[:d] + tgt[d + rng.randint(151, 600):]
    if rng.random() < 0.4:
        a = rng.randint(0, len(tgt))
        tgt = tgt[:a] + "N" * rng.randint(1, 500) + tgt[a:]
    if rng.random() < 0.4:
        a = rng.randint(0, len(ref))
        ref = ref[:a] + "N" * rng.randint(1, 500) + ref[a:]
    if rng.random() < 0.5:
        tgt = soft_mask(rng, tgt)
    hdr = rng.choice([">chrT", None])
    return to_fasta(ref, ">chrR"), to_fasta(tgt, hdr, rng.choice([50, 60]))


def quirk_cases() -> dict[str, tuple[bytes, bytes]]:
    """One fixture per SURVEY.md Appendix B quirk."""
    rng = random.Random(424242)
    cases: dict[str, tuple[bytes, bytes]] = {}
    # B1: pn==0 sentinel -- the same 30-mer at 0 and 100, then different bases.
    core = rand_seq(rng, 30)
    seg = core + rand_seq(rng, 70) + core + rand_seq(rng, 870)
    tgt = core + ("A" if seg[30] != "A" else "C") + rand_seq(rng, 969)
    cases["b1_pn0_sentinel"] = (to_fasta(seg), to_fasta(tgt, ">t"))
    # B2: global stuck walk after a 500-bp deletion (insertion first to force the switch).
    ref = rand_seq(rng, 12000)
    tgt = ref[:2000] + rand_seq(rng, 6000) + ref[2000:5000] + ref[5500:]
    cases["b2_stuck_walk"] = (to_fasta(ref), to_fasta(tgt, ">t"))
    # B3: dropped local segment -- an all-N target segment over a random reference segment.
    ref = rand_seq(rng, 5000)
    tgt = ref[:2000] + "N" * 1000 + ref[3000:]
    cases["b3_dropped_segment"] = (to_fasta(ref), to_fasta(tgt, ">t"))
    # B4: short last reference segment (< k) -> last target segment dropped.
    ref = rand_seq(rng, 3005)
    tgt = ref[:3000] + rand_seq(rng, 500)
    cases["b4_short_last_ref_segment"] = (to_fasta(ref), to_fasta(tgt, ">t"))
    # B5: success-but-bad-ratio segments increment the counter with no T2 check.
    ref = rand_seq(rng, 12000)
    bad = "".join(ref[i * 1000:i * 1000 + 20] + rand_seq(rng, 980) for i in range(3, 9))
    tgt = ref[:3000] + bad + rand_seq(rng, 2000) + ref[11000:]
    cases["b5_counter_no_check"] = (to_fasta(ref), to_fasta(tgt, ">t"))
    # B6: later '>' lines in a multi-record target become sequence.
    ref = rand_seq(rng, 2500)
    tfa = to_fasta(ref[:1200], ">first") + to_fasta(soft_mask(rng, ref[1200:]), ">second Rec")
    cases["b6_multirecord_target"] = (to_fasta(ref), tfa)
    # B7: reference 'n' (lowercase) handling differs between compressor and decompressor.
    ref = rand_seq(rng, 4000)
    refn = ref[:1000] + "nnnnnNNNNN" + ref[1000:]
    tgt = ref[:500] + rand_seq(rng, 5000) + ref[500:]
    cases["b7_reference_lowercase_n"] = (to_fasta(refn), to_fasta(tgt, ">t"))
    # B8: empty target -> empty record line -> decompressor rc 1.
    cases["b8_empty_target"] = (to_fasta(rand_seq(rng, 500)), b">only a header\n")
    # B9: round-trip formatting: 60-column CRLF input is rewritten to 50-column LF.
    ref = rand_seq(rng, 3000)
    cases["b9_crlf_width60"] = (to_fasta(ref), to_fasta(soft_mask(rng, mutate(rng, ref)), ">t", 60, True))
    # extra edge shapes
    cases["e_empty_reference"] = (b">r\n", to_fasta(rand_seq(rng, 1500), ">t"))
    cases["e_no_header_target"] = (to_fasta(ref), to_fasta(mutate(rng, ref), None))
    cases["e_iupac_codes"] = (to_fasta(ref), to_fasta("".join(
        c if rng.random() > 0.02 else rng.choice("RYKMSWBDHV") for c in mutate(rng, ref)), ">t"))
    cases["e_all_n_both"] = (to_fasta("N" * 2500), to_fasta("N" * 2300, ">t"))
    cases["e_target_shorter_than_k"] = (to_fasta(ref), to_fasta("ACGTACG", ">t"))
    cases["e_polyA_repeats"] = (to_fasta(("A" * 60 + rand_seq(rng, 40)) * 40),
                                to_fasta(mutate(rng, ("A" * 60 + rand_seq(rng, 40)) * 45), ">t"))
    return cases


# literal pieces every '(' of which converts under stoi (the record stays parseable) ...
SAFE_PIECES = [")", ",", "(12,", "(-5,", "(+7,", "(0000000000007,", "(2147483647,", "(-2147483648,",
               "(ACGT)", "()", "(1)", ",3)", "9", "-", "))", "(0,"]
# ... and ones that make it throw (out of int range, nothing to convert)
BAD_PIECES = ["(", "(99999999999,", "(2147483648,", "(,", "(A5,", "(("]


def close_paren_case(seed: int) -> tuple[bytes, bytes]:
    """Targets whose only punctuation is ')': delta_encode leaves every such byte alone, so the record
    line holds ')' outside any token, which decompression.cpp:231-234 copies as a literal."""
    rng = random.Random(60_000 + seed)
    rfa, tfa = global_case(seed) if seed % 2 else local_case(seed % 24)
    rate = rng.choice([0.001, 0.005, 0.02])
    out = []
    for ln in tfa.split(b"\n"):
        if ln.startswith(b">") or not ln:
            out.append(ln)
            continue
        b = bytearray()
        for c in ln:
            if rng.random() < rate:
                b += b")" * rng.randint(1, 3)
            b.append(c)
        out.append(bytes(b))
    return rfa, b"\n".join(out)


def paren_case(seed: int) -> tuple[bytes, bytes]:
    """Targets holding '(' ')' ',' digits and signs among the bases: literal bytes that
    delta_encode's own token scan (compression.cpp:262-293) pairs with the real "(p,l)" tokens.
    Local and global shapes; some make its stoi throw (the reference then exits 1)."""
    rng = random.Random(50_000 + seed)
    if seed % 2:
        rfa, tfa = global_case(seed)
    else:
        rfa, tfa = local_case(seed % 24 if seed % 4 else 6)
    lines = tfa.split(b"\n")
    out = []
    rate = rng.choice([0.002, 0.01, 0.05])
    pieces = [["(", ")", ","], SAFE_PIECES, SAFE_PIECES * 20 + BAD_PIECES][seed % 3]
    for ln in lines:
        if ln.startswith(b">") or not ln:
            out.append(ln)
            continue
        b = bytearray()
        for c in ln:
            if rng.random() < rate:
                b += rng.choice(pieces).encode()
            b.append(c)
        out.append(bytes(b))
    tfa = b"\n".join(out)
    if seed % 5 == 0:
        tfa += b"(" if tfa.endswith(b"\n") else b"\n("   # an opener without a closer at the end
    if seed % 7 == 0:
        tfa = tfa.replace(b"\n", b"(5,\n", 3)              # pieces at line ends / header
    return rfa, tfa
