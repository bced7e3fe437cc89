"""N>1 path on CPU: LPT sharding and the record-stream gather over a world_size-2 gloo group."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from pkg import PKG_DIR  # noqa: F401
import multigpu

# UCSC chromInfo lengths: hg19 chr1..22, X, Y (targets)
HG19 = multigpu.HG19


def test_lpt_partitions_everything_once():
    for world in (1, 2, 4, 8):
        parts = multigpu.lpt_shard(HG19, world)
        flat = sorted(i for p in parts for i in p)
        assert flat == list(range(len(HG19)))


def test_lpt_balance_matches_survey():
    # max/mean 1.0 (G=1), 1.002 (2), 1.008 (4), 1.038 (8)
    assert multigpu.max_over_mean(HG19, 1) == pytest.approx(1.0)
    assert multigpu.max_over_mean(HG19, 2) < 1.01
    assert multigpu.max_over_mean(HG19, 4) < 1.02
    assert multigpu.max_over_mean(HG19, 8) < 1.05


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = {f"chr{i}": (f"rec-{i}-" * (i + rank + 1)).encode() for i in multigpu.lpt_shard([5, 3, 8, 1, 0], world)[rank]}
        if rank == 1:
            mine["empty"] = b""
        got = multigpu.gather_records(mine)
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


def test_gather_records_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] is None
    shard = multigpu.lpt_shard([5, 3, 8, 1, 0], 2)
    want = {}
    for r in range(2):
        for i in shard[r]:
            want[f"chr{i}"] = (f"rec-{i}-" * (i + r + 1)).encode()
    want["empty"] = b""
    assert res[0] == want


def _root_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = [5, 0, 17][rank]
        buf = torch.arange(64, dtype=torch.uint8) + 10 * rank   # capacity > n, like bench's d_out
        got = multigpu.gather_to_root(buf, n)
        short = torch.full((2,), rank + 1, dtype=torch.uint8)    # shorter than the largest part
        got2 = multigpu.gather_to_root(short, 2)
        q.put((rank, None if got is None else [g.tolist() for g in got],
               None if got2 is None else [g.tolist() for g in got2]))
    finally:
        dist.destroy_process_group()


def test_gather_to_root_gloo_world3():
    """The bench's and the genome driver's exchange: sizes all-gather + gather to rank 0 only."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_root_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = {r: (a, b) for r, a, b in (q.get(timeout=120) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] == (None, None) and res[2] == (None, None)
    parts, parts2 = res[0]
    assert parts == [[(i + 10 * r) % 256 for i in range(n)] for r, n in enumerate([5, 0, 17])]
    assert parts2 == [[r + 1] * 2 for r in range(3)]


def test_pack_unpack_records():
    import torch
    d = {"chr2": b"abc", "chrX": b"", "chr1": bytes(range(256)) * 3}
    buf = multigpu.pack_records(d, torch.device("cpu"))
    assert multigpu.unpack_records(buf.numpy().tobytes()) == d
    assert multigpu.unpack_records(multigpu.pack_records({}, torch.device("cpu")).numpy().tobytes()) == {}


def test_emitter_status_and_7z(tmp_path):
    """genome.py's rank-0 output side: file layout, the reference's 7z argv, per-chromosome rc."""
    import genome
    import sccg
    fake = tmp_path / "fake7z"
    log = tmp_path / "argv.log"
    fake.write_text(f"#!/bin/bash\necho \"$@\" >> {log}\ncp \"$4\" \"$3\"\n")
    fake.chmod(0o755)
    out = tmp_path / "out"
    em = genome.Emitter(str(out), True, str(fake))
    em.emit('chr1"$(touch pwned)', b"rec1", 0)
    em.emit("chr2", b"abs-text", sccg.SCCG_E_DELTA_STOI)
    em.emit("chr3", b"", 2)
    assert em.wait() == 1
    p1 = out / 'chr1"$(touch pwned)' / "compressed_genome.txt"
    assert p1.read_bytes() == b"rec1" and (p1.parent / "compressed_genome.txt.7z").read_bytes() == b"rec1"
    assert not (tmp_path / "pwned").exists() and not os.path.exists("pwned")
    assert (out / "chr2" / "compressed_genome.txt").read_bytes() == b"abs-text"
    assert not (out / "chr2" / "compressed_genome.txt.7z").exists()
    assert not (out / "chr3").exists()
    assert log.read_text().count("a -mx=9") == 1
    em2 = genome.Emitter(str(out), True, str(fake))
    em2.emit("chr4", b"x", 0)
    assert em2.wait() == 0


class _FakeCtx:
    """Stands in for sccg.Context on CPU: the record text is a function of the two inputs."""

    def compress(self, ref, tgt):
        return b"REC:" + tgt[::-1] + b"|" + ref[:3]

    def stats(self):
        return {"target_bases": 0}

    def close(self):
        pass


def _genome_worker(rank, world, port, q, root):
    import torch
    import torch.distributed as dist
    import genome
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        names = ["chrA", "chrB", "chrC", "chrD", "chrE"]
        sizes = [os.path.getsize(os.path.join(root, "tgt", n + ".fa")) for n in names]
        mine = [names[i] for i in multigpu.lpt_shard(sizes, world)[rank]]
        em = genome.Emitter(os.path.join(root, "out"), False) if rank == 0 else None

        def make_ctx():
            if rank == 1:
                raise RuntimeError("no usable GPU (injected)")
            return _FakeCtx()

        parts, stats = genome.compress_shard(mine, os.path.join(root, "ref"), os.path.join(root, "tgt"), make_ctx, em, 2)
        all_stats = genome.collect(names, parts, stats, em, torch.device("cpu"), world)
        rc = em.wait() if rank == 0 else None
        q.put((rank, mine, rc, {n: v["rc"] for n, v in all_stats.items()}))
    finally:
        dist.destroy_process_group()


def test_genome_failing_rank_gloo_world2(tmp_path):
    """A rank whose context cannot be created still enters the gather: no hang; its chromosomes
    come back failed (rc), the healthy rank's are written, and the job's rc is 1 (genome.py)."""
    root = tmp_path
    for d in ("ref", "tgt"):
        (root / d).mkdir()
    for i, n in enumerate(["chrA", "chrB", "chrC", "chrD", "chrE"]):
        (root / "ref" / f"{n}.fa").write_bytes(b">r\nACGT" * (i + 1))
        (root / "tgt" / f"{n}.fa").write_bytes(b">t\nTTGCA" * (5 - i) * 3)
    (root / "tgt" / "chrE.fa").write_bytes(b">t\nAC")
    os.remove(root / "ref" / "chrE.fa")   # an unreadable pair on whichever rank holds it
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_genome_worker, args=(r, 2, port, q, str(root))) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (mine, rc, st) for r, mine, rc, st in (q.get(timeout=120) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    mine0, rc0, st0 = res[0]
    mine1, _, _ = res[1]
    assert rc0 == 1
    import genome
    for n in mine1:
        assert st0[n] != 0   # rank 1 had no context (or the file is missing)
        assert not (root / "out" / n).exists()
    for n in mine0:
        if n == "chrE":
            assert st0[n] == genome.SCCG_E_IO
            continue
        assert st0[n] == 0
        tgt = (root / "tgt" / f"{n}.fa").read_bytes()
        ref = (root / "ref" / f"{n}.fa").read_bytes()
        assert (root / "out" / n / "compressed_genome.txt").read_bytes() == _FakeCtx().compress(ref, tgt)


class _FakeFilesCtx(_FakeCtx):
    """Also stands in for sccg_compress_files (rank 0's path in genome.run_job)."""

    def compress_files(self, ref_path, tgt_path, out_path):
        ref = open(ref_path, "rb").read()
        tgt = open(tgt_path, "rb").read()
        with open(out_path, "wb") as f:
            f.write(self.compress(ref, tgt))


def _run_job_worker(rank, world, port, q, root, out_name, cost):
    import torch
    import torch.distributed as dist
    import genome
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        names = ["chrA", "chrB", "chrC", "chrD", "chrE"]
        rc, summary = genome.run_job(names, os.path.join(root, "ref"), os.path.join(root, "tgt"),
                                     os.path.join(root, out_name), _FakeFilesCtx, rank, world, torch.device("cpu"),
                                     contexts=2, run_7z=False, err_hip=2, cost=cost)
        q.put((rank, rc, None if summary is None else {n: v["rc"] for n, v in summary["per_chrom"].items()}))
    finally:
        dist.destroy_process_group()


def _make_pairs(root):
    for d in ("ref", "tgt"):
        (root / d).mkdir()
    for i, n in enumerate(["chrA", "chrB", "chrC", "chrD", "chrE"]):
        (root / "ref" / f"{n}.fa").write_bytes(b">r\nACGT" * (i + 1))
        (root / "tgt" / f"{n}.fa").write_bytes(b">t\nTTGCA" * (5 - i) * 3)


def _spawn(fn, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=120) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("cost", [None, {"chrE": 1000.0, "chrA": 1.0}])
def test_genome_run_job_gloo_world2(tmp_path, cost):
    """genome.py's job as main() runs it: rank 0 writes its own pairs through compress_files, rank 1's
    texts come over the gather and are written by rank 0 -- every pair once, byte for byte, rc 0;
    sharding by a measured cost (T2T-like pairs) instead of target size changes only who does what."""
    import genome
    _make_pairs(tmp_path)
    res = _spawn(_run_job_worker, 2, str(tmp_path), "out", cost)
    rc0, st0 = res[0]
    assert res[1] == [0, None]
    assert rc0 == 0 and sorted(st0) == ["chrA", "chrB", "chrC", "chrD", "chrE"] and set(st0.values()) == {0}
    for n in st0:
        ref = (tmp_path / "ref" / f"{n}.fa").read_bytes()
        tgt = (tmp_path / "tgt" / f"{n}.fa").read_bytes()
        assert (tmp_path / "out" / n / "compressed_genome.txt").read_bytes() == _FakeCtx().compress(ref, tgt)
    if cost:   # the costly pair sits alone on its rank
        sizes = [os.path.getsize(tmp_path / "tgt" / f"{n}.fa") for n in sorted(st0)]
        w = [cost.get(n, s) for n, s in zip(sorted(st0), sizes)]
        assert [4] in multigpu.lpt_shard(w, 2)
    assert genome.SCCG_E_OUT != genome.SCCG_E_IO


def test_genome_unwritable_out_dir_fails_job(tmp_path):
    """rank 0's files path with an output folder it cannot create -- every pair is reported
    failed (SCCG_E_OUT) and the job's rc is 1, instead of the worker thread dying silently."""
    import genome
    _make_pairs(tmp_path)
    blocker = tmp_path / "out"
    blocker.write_bytes(b"a file where the output folder should be")
    em = genome.Emitter(str(blocker), False)
    names = ["chrA", "chrB", "chrC"]
    stats = genome.compress_shard_files(names, str(tmp_path / "ref"), str(tmp_path / "tgt"), _FakeFilesCtx, em, 2,
                                        contexts=2)
    assert {n: v["rc"] for n, v in stats.items()} == {n: genome.SCCG_E_OUT for n in names}
    assert em.wait() == 1


def test_genome_worker_closes_context_on_error(tmp_path):
    """A context whose compress_files raises something unexpected: the pair fails, the context is
    still closed, the other pairs go on."""
    import genome
    _make_pairs(tmp_path)
    closed = []

    class Boom(_FakeFilesCtx):
        def compress_files(self, ref_path, tgt_path, out_path):
            if "chrB" in ref_path:
                raise ValueError("boom")
            super().compress_files(ref_path, tgt_path, out_path)

        def close(self):
            closed.append(1)

    em = genome.Emitter(str(tmp_path / "out"), False)
    stats = genome.compress_shard_files(["chrA", "chrB", "chrC"], str(tmp_path / "ref"), str(tmp_path / "tgt"), Boom, em,
                                        2, contexts=1)
    assert stats["chrB"]["rc"] != 0 and stats["chrA"]["rc"] == 0 and stats["chrC"]["rc"] == 0
    assert closed == [1] and em.wait() == 1


def test_cost_weights_one_unit():
    """genome.py --cost: pairs missing from the cost file are weighed in the file's unit (median
    cost per target byte), not in bytes next to milliseconds."""
    import genome
    names, sizes = ["a", "b", "c", "d"], [100_000_000, 200_000_000, 50_000_000, 150_000_000]
    w = genome.cost_weights(names, sizes, {"a": 10.0, "b": 30.0, "c": 5.0})
    assert w[:3] == [10.0, 30.0, 5.0]
    assert w[3] == pytest.approx(150_000_000 * 1e-7)   # median of 1e-7, 1.5e-7, 1e-7 ms per byte
    parts = multigpu.lpt_shard(w, 2)   # 30 | 15 + 10 + 5 (in bytes, "d" would sit alone on a rank)
    assert sorted(sum(w[i] for i in p) for p in parts) == [30.0, 30.0]
