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
