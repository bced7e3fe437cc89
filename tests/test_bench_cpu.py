"""bench.py's N > 1 path on CPU (gloo, world_size 2): the timed region's barrier + MAX over ranks,
the gather of every rank's per-chromosome record streams to rank 0, the per-rank totals summed
over ranks, the pin check on the gathered streams, and the CPU-baseline pointer an N > 1 line
carries.  The bench's own functions run, with fake record streams instead of GPU compression
(the per-pair independence of compression.cpp:584-610 is what makes the shard + gather exact)."""
import hashlib
import os
import socket
import sys
import time

import torch.multiprocessing as mp

from pkg import PKG_DIR  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_stream(name: str) -> bytes:
    return (f">{name}\n" + "acgt" * (len(name) + 3) + "\n\n" + f"(0,{len(name) * 7})ACGT").encode()


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import multigpu
        names = multigpu.CHROMS
        mine = [names[i] for i in multigpu.lpt_shard(multigpu.HG19, world)[rank]]
        results = {n: (torch.frombuffer(bytearray(_fake_stream(n)), dtype=torch.uint8), {"target_bases": len(n)})
                   for n in mine}
        calls = [0]

        def step():
            calls[0] += 1
            time.sleep(0.03 * (rank + 1))   # rank 1 is the slow one

        dt = bench.timed_region(step, 3, 1, world)
        streams = bench.gather_streams(results, mine, world, torch.device("cpu"))
        tot = {"target_bases": sum(len(n) for n in mine), "pairs": len(mine)}
        job, per_rank = bench.job_totals(tot, world)
        pins = {n: {"record_sha256": hashlib.sha256(_fake_stream(n)).hexdigest()} for n in names}
        pins["chr7"] = {"record_sha256": "0" * 64}   # a deliberate mismatch
        parity = bench.check_pins(streams, pins)
        q.put((rank, {"dt": dt, "calls": calls[0], "streams": streams, "job": job, "per_rank": per_rank,
                      "parity": parity, "cpu_ptr": bench.cpu_baseline_pointer()}))
    finally:
        dist.destroy_process_group()


def test_bench_distributed_pieces_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import multigpu
    r0, r1 = res[0], res[1]
    # exactly K timed steps after W warm-up steps; the time is the slow rank's, on both ranks
    assert r0["calls"] == r1["calls"] == 4
    assert r0["dt"] == r1["dt"] >= 3 * 0.06
    # rank 0 holds every chromosome's stream, byte for byte; rank 1 holds none
    assert r1["streams"] is None
    assert r0["streams"] == {n: _fake_stream(n) for n in multigpu.CHROMS}
    # totals: summed over ranks, identical on both
    assert r0["job"] == r1["job"] == {"target_bases": sum(len(n) for n in multigpu.CHROMS), "pairs": 24}
    assert [t["pairs"] for t in r0["per_rank"]] == [len(p) for p in multigpu.lpt_shard(multigpu.HG19, 2)]
    # pins: all 24 checked on rank 0, the planted mismatch found
    assert r0["parity"]["pinned_checked"] == 24 and r0["parity"]["pinned_mismatch"] == ["chr7"]
    assert r1["parity"] is None
    # N > 1 lines point at the N = 1 CPU baseline
    ptr = r0["cpu_ptr"]
    assert ptr is not None and ptr["value"] > 0 and "N = 1" in ptr["measured_in"]


class _FakeLane:
    stream = None


class _FakePool:
    """bench.LanePool's interface: run(order, job) does every pair on some lane."""

    def __init__(self, n_lanes=2):
        self.lanes = [_FakeLane() for _ in range(n_lanes)]

    def run(self, order, job):
        for i, n in enumerate(order):
            job(self.lanes[i % len(self.lanes)], n)

    def sync(self):
        pass


def _step_worker(rank, world, port, q):
    """bench.make_step -- the step main() times -- with a fake compress job, gloo world 2."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import multigpu
        names = multigpu.CHROMS
        mine = [names[i] for i in multigpu.lpt_shard(multigpu.HG19, world)[rank]]
        order = sorted(mine, key=lambda n: -multigpu.HG19[names.index(n)])
        results = {}

        def job(lane, name):   # the fake compress: the pair's record stream into results
            results[name] = (torch.frombuffer(bytearray(_fake_stream(name)), dtype=torch.uint8), {})

        gather = multigpu.StreamGather()
        step = bench.make_step(_FakePool(), order, job, results, gather)
        # host synchronisation inside the timed steps: device reads and host-side collectives
        syncs = []
        watch = {"item": torch.Tensor, "tolist": torch.Tensor, "cpu": torch.Tensor, "numpy": torch.Tensor}
        saved = {k: getattr(c, k) for k, c in watch.items()}
        saved_sync, saved_ago, saved_ag = torch.cuda.synchronize, dist.all_gather_object, dist.all_gather
        counting = [False]

        def wrap(name, f):
            def g(*a, **k):
                if counting[0]:
                    syncs.append(name)
                return f(*a, **k)
            return g
        for k, c in watch.items():
            setattr(c, k, wrap(k, saved[k]))
        torch.cuda.synchronize = wrap("cuda.synchronize", saved_sync)
        dist.all_gather_object = wrap("all_gather_object", saved_ago)
        dist.all_gather = wrap("all_gather", saved_ag)
        try:
            step()   # warm-up: the gather's plan (outside the timed region in bench.main)

            def counted_step():
                counting[0] = True
                step()
                counting[0] = False
            dt = bench.timed_region(counted_step, 3, 0, world)
        finally:
            for k, c in watch.items():
                setattr(c, k, saved[k])
            torch.cuda.synchronize, dist.all_gather_object, dist.all_gather = saved_sync, saved_ago, saved_ag
        got = gather.result()
        streams = {n: bytes(t.numpy().tobytes()) for n, t in got.items()} if got is not None else None
        # a record stream whose length left the plan is refused, not truncated
        results[order[0]] = (torch.zeros(3, dtype=torch.uint8), {})
        try:
            gather.step({n: results[n][0] for n in order})
            refused = False
        except RuntimeError:
            refused = True
        q.put((rank, {"dt": dt, "syncs": syncs, "streams": streams, "refused": refused,
                      "recv_bytes": sum(int(t.numel()) for t in gather.recv.values())}))
    finally:
        dist.destroy_process_group()


def test_bench_step_gather_no_host_sync_gloo_world2():
    """bench.make_step at N = 2 (gloo): rank 0 ends up with every chromosome's stream, the step
    reads nothing back and runs no host-side collective (timed_region's barrier + MAX are outside it),
    rank 0 receives exactly the other rank's bytes (no padding to the largest), and a stream whose
    length left the plan is refused."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_step_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import multigpu
    r0, r1 = res[0], res[1]
    assert r0["streams"] == {n: _fake_stream(n) for n in multigpu.CHROMS}
    assert r1["streams"] is None
    assert r0["syncs"] == [] and r1["syncs"] == [], (r0["syncs"], r1["syncs"])
    rank1 = [multigpu.CHROMS[i] for i in multigpu.lpt_shard(multigpu.HG19, 2)[1]]
    assert r0["recv_bytes"] == sum(len(_fake_stream(n)) for n in rank1)
    assert r0["refused"] and r1["refused"]


def test_job_models_say_what_they_count():
    """roofline_job's design model (what this design moves: byte copies, no k-mer index) and
    SURVEY §8(d)'s model (2-bit packing, a 4|R'| CSR index this design never builds)."""
    import bench
    nT, nR, nRp, out, tfa, rfa = 249_250_621, 247_249_719, 225_000_000, 6_700_000, 254_000_000, 252_000_000
    d = bench.design_alg_bytes(tfa, rfa, nT, nR, nRp, out, True)
    assert d == tfa + rfa + (nT + nRp) + out + nRp + 0.5 * nT   # (lean strips: T', R' only; run lines from the strip)
    d_local = bench.design_alg_bytes(tfa, rfa, nT, nR, nRp, out, False)
    assert d_local == tfa + rfa + 2 * (nT + nR) + out + 2 * min(nT, nR)
    s = bench.survey_alg_bytes(nT, nR, nRp, out)
    assert s == 1.25 * (nT + nR) + 0.25 * nR + 4 * nRp + 0.5 * nT + out
