"""CPU analysis (diagnostics, no GPU): per-segment class-0 proof and oracle class up to the local->global switch
of a synthetic pair, and the runs of unproved segments.  Usage: local_runs.py PROFILE REF_LEN TGT_LEN SEED"""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
import synthlib, oraclelib
from test_local_proof_cpu import prove

def seq_of(fa: bytes) -> bytes:
    out = []
    for line in fa.split(b"\n"):
        if line.startswith(b">"):
            continue
        out.append(line.strip())
    return b"".join(out).upper()

def seg_class(r, t):
    non_n = any(c != ord("N") for c in t)
    for k in (14, 10):
        recs = oraclelib.match(r, t, k, 0, False, 0)
        if any(kind for kind, _, _, _ in recs):
            lit = sum(l for kind, _, l, _ in recs if not kind)
            return 1 if (2 * lit > len(t) and non_n) else 0
    return 2 if non_n else 3

prof, rl, tl, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
rfa, tfa = synthlib.synth_pair(prof, rl, tl, seed)
R, T = seq_of(rfa), seq_of(tfa)
L = 1000
nseg = min((len(R) + L - 1) // L, (len(T) + L - 1) // L)
cnt = 0
cls, prv = [], []
t0 = time.time()
sw = None
for s in range(nseg):
    r, t = R[s * L:(s + 1) * L], T[s * L:(s + 1) * L]
    c = seg_class(r, t)
    p = prove(r, t)
    if p:
        assert c == 0
    cls.append(c); prv.append(p)
    if c in (1, 2):
        cnt += 1
    else:
        cnt = 0
    if c == 2 and len(cls) >= 5 and all(x in (1, 2) for x in cls[-5:-1]):
        sw = s
        break
print("switch", sw, "segments", len(cls), "time", round(time.time() - t0, 1))
npv = [i for i, p in enumerate(prv) if not p]
print("non-proven", len(npv), "class counts", {c: cls.count(c) for c in range(4)})
print("non-proven class0", sum(1 for i in npv if cls[i] == 0))
# runs of non-proven
runs = []
i = 0
while i < len(prv):
    if not prv[i]:
        j = i
        while j < len(prv) and not prv[j]:
            j += 1
        runs.append((i, j - i)); i = j
    else:
        i += 1
long = [r for r in runs if r[1] >= 5]
print("runs", len(runs), "in runs>=5:", sum(l for _, l in long), "long runs", long[:20])
hist = {}
for _, l in runs:
    hist[min(l, 10)] = hist.get(min(l, 10), 0) + 1
print("run length hist", sorted(hist.items()))
