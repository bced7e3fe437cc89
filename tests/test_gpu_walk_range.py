"""GPU: sccg_walk_range -- the global walk (compression.cpp:64-161) from an arbitrary state until an
index, on the HIP chunk machinery restricted to [x0, x_end) -- and one chromosome's walk split
across two ranks with it as the engine (multigpu.split_walk).

* against the oracle's orc_walk_range (the pinned restatement) from the true start, from states on
  the true walk, from arbitrary (wrong) states, and over ranges ending anywhere;
* two gloo ranks in two processes, both on GPU 0, each walking its half through
  sccg_walk_range_device: the stitched walk's record line gives the sha256 the compiled reference
  pinned for the chr21 pair (configs[0]'s pair) and the 100 Mb T2T-like pair.
"""
import hashlib
import json
import os
import random
import socket

import pytest
import torch.multiprocessing as mp

from pkg import sccg  # (puts the package directory on sys.path first)
import multigpu
import oraclelib
import synthlib

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def ctx():
    c = sccg.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("profile,rl,tl,seed", [("hg", 600_000, 601_500, 71), ("t2t", 800_000, 800_000, 72),
                                                ("hg", 2_000_000, 2_003_000, 73), ("t2t", 1_500_000, 1_500_000, 74)])
def test_walk_range_vs_oracle(ctx, profile, rl, tl, seed):
    rfa, tfa = synthlib.synth_pair(profile, rl, tl, seed)
    R, T = oraclelib.global_sequences(rfa, tfa)
    rng = random.Random(seed)
    full, fex = oraclelib.walk_range(R, T, 14, 100, 0, -1, len(T))
    got, gex = ctx.walk_range(R, T, 14, 100, 0, -1, len(T))
    assert (got, gex) == (full, fex)
    states = [(0, -1, len(T) // 3), (0, -1, 5)]
    for _ in range(6):   # states on the true walk, ranges ending anywhere
        i = rng.randrange(len(full)) if full else 0
        t, p, l = full[i] if full else (0, 0, 0)
        x0 = t + l
        states.append((x0, p + l - 1, x0 + rng.randint(0, len(T) - x0 + 100)))
    for _ in range(6):   # arbitrary states (a speculative guess)
        x0 = rng.randrange(len(T))
        states.append((x0, rng.randrange(len(R)), x0 + rng.randint(1, 400_000)))
    states.append((len(T) - 3, 10, len(T) + 50))
    for x0, p0, xe in states:
        want = oraclelib.walk_range(R, T, 14, 100, x0, p0, xe)
        assert ctx.walk_range(R, T, 14, 100, x0, p0, xe) == want, (x0, p0, xe)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, name):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        e = {m["name"]: m for m in json.load(open(os.path.join(HERE, "golden", "genome_manifest.json")))}[name]
        rfa, tfa = synthlib.synth_pair(e["profile"], e["ref_len"], e["tgt_len"], e["seed"])
        R, T = oraclelib.global_sequences(rfa, tfa)
        dev = torch.device("cuda", 0)
        d_r = torch.frombuffer(bytearray(R), dtype=torch.uint8).to(dev)
        d_t = torch.frombuffer(bytearray(T), dtype=torch.uint8).to(dev)
        c = sccg.Context(0)
        calls = []

        def walker(x0, p0, x_end):
            calls.append((x0, p0, x_end))
            return c.walk_range_device(d_r.data_ptr(), len(R), d_t.data_ptr(), len(T), 14, 100, x0, p0, x_end)

        def guess(h):   # the diagonal of a 32-mer of T' near h found in R' (as the chunks' anchors vote)
            for y in range(h, min(len(T) - 32, h + 8 * 512), 512):
                p = R.find(T[y:y + 32])
                if p >= 0:
                    return max(0, min(len(R) - 1, p - (y - h) - 1))
            return int(h * len(R) / max(1, len(T)))

        got = multigpu.split_walk(walker, len(T), guess)
        rec = c.compress(rfa, tfa) if rank == 0 else None
        c.close()
        q.put((rank, got, calls, rec))
    finally:
        dist.destroy_process_group()


def _record_line(T: bytes, matches) -> bytes:
    out, prev_end, prev_p = [], 0, 0
    for t, p, l in matches:
        out.append(T[prev_end:t])
        out.append(b"(%d,%d)" % (p - prev_p, l))
        prev_p, prev_end = p, t + l
    out.append(T[prev_end:])
    return b"".join(out)


@pytest.mark.parametrize("name", ["chr21", "t2t100"])
def test_split_walk_gpu_world2(name):
    pins = {m["name"]: m for m in json.load(open(os.path.join(HERE, "golden", "genome_manifest.json")))}
    if name not in pins:
        pytest.skip(f"{name} not pinned")
    e = pins[name]
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_worker, args=(r, 2, port, q, name)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (g, c, rec) for r, g, c, rec in (q.get(timeout=240) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    stitched, _, rec = res[0]
    assert res[1][0] is None
    rfa, tfa = synthlib.synth_pair(e["profile"], e["ref_len"], e["tgt_len"], e["seed"])
    R, T = oraclelib.global_sequences(rfa, tfa)
    head = rec.rsplit(b"\n", 1)[0]
    whole = head + b"\n" + _record_line(T, stitched)
    assert hashlib.sha256(whole).hexdigest() == e["record_sha256"]
    # rank 1 walked its half at least once (and again if its guessed entry was not rank 0's exit)
    assert len(res[1][1]) >= 1


def test_carry_chains_under_poor_speculation_vs_oracle():
    """SCCG_ANCHOR_SHIFT=-2 (a quarter-size anchor table: most chunks' first guesses are wrong)
    makes the rounds lean on carry chains (k_walk<., true> commits the chunks it carries into)
    next to frozen (T2T-like) and trapped chunks; the whole walk and walks from mid-states must
    still be the oracle's sequential walk (orc_walk_range).  A child process: the knob is read
    once per process."""
    import subprocess
    import sys
    code = (
        "import json, sys\n"
        f"sys.path.insert(0, {HERE!r})\n"
        "import synthlib, oraclelib\n"
        "from pkg import sccg\n"
        "c = sccg.Context(0)\n"
        "out = []\n"
        "for prof, n, seed in (('hg', 3_000_000, 81), ('t2t', 3_000_000, 82), ('t2t', 6_000_000, 83)):\n"
        "    rfa, tfa = synthlib.synth_pair(prof, n, n, seed)\n"
        "    R, T = oraclelib.global_sequences(rfa, tfa)\n"
        "    full = oraclelib.walk_range(R, T, 14, 100, 0, -1, len(T))\n"
        "    got = c.walk_range(R, T, 14, 100, 0, -1, len(T))\n"
        "    rounds = c.stats()['walk_rounds']\n"
        "    ok = got == full\n"
        "    m = full[0]\n"
        "    if m:\n"
        "        t, p, l = m[len(m) // 2]\n"
        "        ok = ok and c.walk_range(R, T, 14, 100, t + l, p + l - 1, len(T)) == "
        "oraclelib.walk_range(R, T, 14, 100, t + l, p + l - 1, len(T))\n"
        "    out.append((prof, seed, ok, rounds, len(m)))\n"
        "print(json.dumps(out))\n"
    )
    env = dict(os.environ, SCCG_ANCHOR_SHIFT="-2")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert all(ok for _, _, ok, _, _ in res), res
