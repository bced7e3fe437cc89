"""The local pass's class-0 proof (local.hip seg_prove) restated in Python and checked against the
oracle's per-segment walk (compression.cpp:400-416 via match_sequences, :36-179): whenever the proof
says "class 0" (the k = 14 pass succeeds and at most half of the target segment is literal), the
oracle's walk agrees -- on aligned, drifted, repetitive, N-heavy, short and unrelated segment pairs.
The proof is a sufficient condition only: a segment it does not settle is walked as before."""
import random

import pytest

import oraclelib

K, SEGB = 14, 1024


def prove(r: bytes, t: bytes) -> bool:
    """Mirror of seg_prove: diagonals from 8 sampled target k-mers (the lowest reference position of
    each), coverage by 14 equal bytes on a diagonal, per-16-position-lane read bounds."""
    nr, nt = len(r), len(t)
    lastr, lastk = nr - K, nt - K
    if lastr < 0 or lastk < 0:
        return False
    pure = set(b"ACGT")
    first = {}
    for p in range(lastr + 1):
        km = r[p:p + K]
        if set(km) <= pure:
            first.setdefault(km, p)
    diags = []
    for j in range(8):
        if len(diags) >= 4:
            break
        y = j * lastk // 8
        km = t[y:y + K]
        if not set(km) <= pure or km not in first:
            continue
        d = first[km] - y
        if d not in diags:
            diags.append(d)
    if not diags:
        return False
    rpad = r + bytes(SEGB - nr)
    cov = set()
    for d in diags:
        for i in range(lastk + 1):
            ra = (i // 16) * 16 + d
            if not (0 <= ra <= SEGB - 36) or not (0 <= i + d <= lastr):
                continue
            if t[i:i + K] == rpad[i + d:i + d + K]:
                cov.add(i)
    if not cov:
        return False
    unc = lastk + 1 - len(cov)
    return 2 * (unc + (nt - 1 - lastk)) <= nt


def oracle_class(r: bytes, t: bytes) -> int:
    """The reference's segment class: 0 good, 1 bad ratio, 2 no match (non-N), 3 no match (all N)."""
    recs = oraclelib.match(r, t, K, 0, False, 0)
    non_n = any(c != ord("N") for c in t)
    if any(kind for kind, _, _, _ in recs):
        lit = sum(l for kind, _, l, _ in recs if not kind)
        return 1 if (2 * lit > len(t) and non_n) else 0
    return 2 if non_n else 3


def mutate(rng, s: bytes, snp: float, indel: float) -> bytes:
    out = bytearray()
    for c in s:
        x = rng.random()
        if x < snp:
            out.append(rng.choice([b for b in b"ACGT" if b != c]))
        elif x < snp + indel:
            if rng.random() < 0.5:
                out.extend(rng.choice(b"ACGT") for _ in range(rng.randint(1, 8)))
                out.append(c)
        else:
            out.append(c)
    return bytes(out)


def cases(seed: int, n: int):
    rng = random.Random(seed)
    for _ in range(n):
        kind = rng.choice(["aligned", "drift", "tandem", "nrun", "short", "unrelated", "lowcomp", "half"])
        base = bytes(rng.choice(b"ACGT") for _ in range(3000))
        if kind == "tandem":
            unit = bytes(rng.choice(b"ACGT") for _ in range(rng.randint(2, 40)))
            base = (unit * (3000 // len(unit) + 1))[:3000]
            base = mutate(rng, base, 0.02, 0.0)
        if kind == "lowcomp":
            base = bytes(rng.choice(b"AT") for _ in range(3000))
        off = rng.randint(0, 900)
        r = base[off:off + 1000]
        if kind == "aligned":
            t = mutate(rng, r, 0.002, 0.0)
        elif kind == "drift":
            sh = rng.choice([-1, 1]) * rng.randint(1, 700)
            t = mutate(rng, base[off + sh if off + sh >= 0 else 0:][:1000], 0.01, 0.002)
        elif kind == "nrun":
            t = bytearray(mutate(rng, r, 0.005, 0.0))
            a = rng.randint(0, 999)
            b = min(1000, a + rng.randint(1, 900))
            t[a:b] = b"N" * (b - a)
            t = bytes(t)
            if rng.random() < 0.3:
                r = bytes(r[:a]) + b"N" * (b - a) + bytes(r[b:])
        elif kind == "short":
            ln = rng.randint(1, 60)
            r, t = r[:rng.randint(1, 1000)], mutate(rng, r[:ln], 0.01, 0.0)
        elif kind == "unrelated":
            t = bytes(rng.choice(b"ACGT") for _ in range(1000))
        elif kind == "half":
            t = r[:rng.randint(300, 700)] + bytes(rng.choice(b"ACGT") for _ in range(1000))
            t = t[:1000]
        else:
            t = mutate(rng, r, 0.02, 0.003)
        yield kind, r[:1000], t[:1000]


@pytest.mark.parametrize("seed", range(4))
def test_class0_proof_is_sound(seed):
    proved = 0
    for kind, r, t in cases(5000 + seed, 300):
        if prove(r, t):
            proved += 1
            assert oracle_class(r, t) == 0, (kind, r, t)
    assert proved > 30   # (the aligned-like cases are proved: the proof is not vacuous)


def full_class(r: bytes, t: bytes) -> int:
    """The reference's segment class with both passes (compression.cpp:400-460): k = 14, then
    k2 = 10 when the first finds no match."""
    non_n = any(c != ord("N") for c in t)
    for k in (14, 10):
        recs = oraclelib.match(r, t, k, 0, False, 0)
        if any(kind for kind, _, _, _ in recs):
            lit = sum(l for kind, _, l, _ in recs if not kind)
            return 1 if (2 * lit > len(t) and non_n) else 0
    return 2 if non_n else 3


def hits10(r: bytes, t: bytes) -> int:
    """Mirror of seg_hits<10>: target positions whose 10-mer occurs among the reference's."""
    ks = {r[p:p + 10] for p in range(len(r) - 9)}
    return sum(1 for y in range(len(t) - 9) if t[y:y + 10] in ks)


@pytest.mark.parametrize("seed", range(4))
def test_probe_hit_count_rule(seed):
    """k_local_probe's class from the k2 hit count (pure ACGT segment pairs): no hit position means
    neither pass matches (class 2); fewer than nt / 28 means any match the passes take leaves more
    than half of the segment literal (class 1) -- each match of length l covers l - k + 1 hit
    positions and every 14-mer hit is a 10-mer hit, so at most 14 h10 bases match."""
    fired = 0
    rng = random.Random(900 + seed)
    extra = []
    for _ in range(60):   # sparse chance hits: unrelated segments with planted 10-40 base copies
        r = bytes(rng.choice(b"ACGT") for _ in range(1000))
        t = bytearray(rng.choice(b"ACGT") for _ in range(rng.choice([1000, 1000, 400, 37])))
        for _ in range(rng.randint(0, 3)):
            ln = rng.randint(10, 40)
            a, b = rng.randint(0, 1000 - ln), rng.randint(0, max(0, len(t) - ln))
            t[b:b + ln] = r[a:a + ln]
        extra.append(("planted", r, bytes(t)))
    for kind, r, t in list(cases(7000 + seed, 200)) + extra:
        if not (set(r) <= set(b"ACGT") and set(t) <= set(b"ACGT")) or not t:
            continue
        h = hits10(r, t)
        if h == 0 or 28 * h < len(t):
            fired += 1
            assert full_class(r, t) == (2 if h == 0 else 1), (kind, h, r, t)
    assert fired > 40
