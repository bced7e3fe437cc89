"""CPU: the local pass's fast class-0 proof (local.hip fast_class0) never contradicts the reference.

The switch scan of the local pass (compression.cpp:372-474) needs only each segment's class; the
proof classifies a full 1000-base segment pair as class 0 (k = 14 matches, literal ratio <= 0.5)
from five probe k-mers' diagonals and the target positions none of them covers, without the walk.  This restates the
proof in Python exactly as the kernel computes it and checks, over segment pairs built to sit on
both sides of its bound (shifted copies with substitutions, indels, N runs, lowercase, repeats),
that every pair it accepts is class 0 by the oracle's own match_sequences (orc_match, pinned
against the compiled reference).
"""
import random

import oraclelib

K, SEG = 14, 1000
PROBES = (40, 260, 480, 700, 920)
CODE = {ord("A"): 0, ord("C"): 1, ord("G"): 2, ord("T"): 3}


def key(s: bytes, i: int):
    """packed code of the k-mer at i, or None when it holds a byte other than A/C/G/T (exotic)"""
    v = 0
    for q in range(K):
        c = CODE.get(s[i + q])
        if c is None:
            return None
        v |= c << (2 * q)
    return v


def fast_class0(r: bytes, t: bytes) -> bool:
    """local.hip fast_class0 on uppercased full segments"""
    nr, nt = len(r), len(t)
    if nr != SEG or nt != SEG:
        return False
    rkeys = [key(r, p) for p in range(nr - K + 1)]
    diags = []
    for sp in PROBES:
        if sp + K > nt:
            continue
        pk = key(t, sp)
        if pk is None:
            continue
        hits = [p for p, kk in enumerate(rkeys) if kk == pk]
        if hits and hits[0] - sp not in diags:
            diags.append(hits[0] - sp)

    def eq(j, d):
        return j < nt and 0 <= j + d < nr and t[j] == r[j + d]

    uncovered = 0
    for j in range(nt):
        if not any(all(eq(j + i, d) for i in range(K)) for d in diags):
            uncovered += 1
    return 2 * uncovered <= nt


def oracle_class(r: bytes, t: bytes) -> int:
    """class of the segment by the reference's k = 14 pass (compression.cpp:402-416): 0 good,
    1 success-but-bad, 2/3 failed (the k = 10 retry never yields class 0)"""
    recs = oraclelib.match(r, t, K, 0, False)
    if not any(kind == 1 for kind, _, _, _ in recs):
        return 2
    lit = sum(l for kind, _, l, _ in recs if kind == 0)
    non_n = any(c != ord("N") for c in t)
    return 1 if (lit / len(t) > 0.5 and non_n) else 0


def rand_seq(rng, n, alphabet=b"ACGT"):
    return bytes(rng.choice(alphabet) for _ in range(n))


def mutate(rng, s: bytes, sub: float, indel: float) -> bytes:
    out = bytearray()
    i = 0
    while i < len(s):
        u = rng.random()
        if u < sub:
            out.append(rng.choice([c for c in b"ACGT" if c != s[i]]))
            i += 1
        elif u < sub + indel:
            if rng.random() < 0.5:
                out += rand_seq(rng, rng.randint(1, 20))
            else:
                i += rng.randint(1, 20)
        else:
            out.append(s[i])
            i += 1
    return bytes(out)


def cases(seed: int, n: int):
    rng = random.Random(seed)
    for _ in range(n):
        base = rand_seq(rng, 3 * SEG)
        kind = rng.randrange(6)
        if kind == 5:   # tandem repeat: many candidates per k-mer
            unit = rand_seq(rng, rng.randint(2, 40))
            base = (unit * (3 * SEG // len(unit) + 1))[: 3 * SEG]
            base = mutate(rng, base, 0.02, 0.0)[: 3 * SEG].ljust(3 * SEG, b"A")
        d = rng.choice([0, 0, rng.randint(-40, 40), rng.randint(-600, 600)])
        r = base[SEG: 2 * SEG]
        sub = rng.choice([0.0, 0.001, 0.01, 0.03, 0.05, 0.2])
        tt = mutate(rng, base, sub, rng.choice([0.0, 0.0, 0.001, 0.01]))
        t = (tt[SEG + d: 2 * SEG + d] + rand_seq(rng, SEG))[:SEG]
        if kind == 1:   # an N run in both
            a, b = sorted(rng.sample(range(SEG), 2))
            r = r[:a] + b"N" * (b - a) + r[b:]
            t = t[:a] + b"N" * (b - a) + t[b:]
        elif kind == 2:   # an N run in the target only
            a, b = sorted(rng.sample(range(SEG), 2))
            t = t[:a] + b"N" * (b - a) + t[b:]
        yield r, t


def test_fast_proof_never_contradicts_the_reference():
    accepted = 0
    for i, (r, t) in enumerate(cases(1234, 400)):
        if fast_class0(r, t):
            accepted += 1
            assert oracle_class(r, t) == 0, i
    assert accepted > 150   # the proof takes the bulk of the aligned segments


def test_fast_proof_bound_edges():
    """substitutions on one diagonal right at the bound (2 B <= nt) and one past it"""
    rng = random.Random(7)
    for d in (0, 5, -5, 300, -300, 440, -440):
        for extra in (0, 1, 2):
            base = rand_seq(rng, 3 * SEG)
            r = base[SEG: 2 * SEG]
            t = bytearray(base[SEG + d: 2 * SEG + d])
            budget = (SEG // 2 - abs(d) - 2 * (K - 1)) // K + extra
            pos = rng.sample(range(max(0, -d), min(SEG, SEG - d)), max(0, budget)) if budget > 0 else []
            for p in pos:
                t[p] = next(c for c in b"ACGT" if c != t[p])
            t = bytes(t)
            if fast_class0(r, t):
                assert oracle_class(r, t) == 0, (d, extra)
