#!/usr/bin/env python3
"""Whole-genome compression across the GPUs of one node (BASELINE configs[2]).

    python genome.py --ref-dir hg18/ --tgt-dir hg19/ --out out/              # 1 GPU
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        genome.py --ref-dir hg18/ --tgt-dir hg19/ --out out/                # 8 GPUs

Every `<name>.fa` present in both directories is one reference invocation (compression.cpp
main with argv[1]=ref, argv[2]=target).  Pairs are LPT-sharded by target size, compressed on the
rank's GPU through the C ABI, and the record texts are gathered to rank 0 over RCCL; rank 0 writes
`<out>/<name>/compressed_genome.txt` (compression.cpp:329) and runs the same
`7z a -mx=9 "<...>.7z" "<...>"` (compression.cpp:308) unless --no-7z.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

SCCG_E_IO = 100    # a FASTA file could not be read (host side; no library call was made)
SCCG_E_OUT = 101   # the output folder could not be written (host side)


class Emitter:
    """Rank 0's output side: <out>/<name>/compressed_genome.txt (compression.cpp:329) and the
    reference's `7z a -mx=9 <txt>.7z <txt>` (compression.cpp:308) per chromosome, started as soon as
    that chromosome's text is on rank 0 so LZMA2 runs beside the GPU work still queued
    (SURVEY §8(f)2).  Per-chromosome exit status follows the reference CLI: a stoi failure inside
    delta_encode leaves the (absolute-position) text written and skips 7z; any other error writes
    nothing; both make the job's rc 1."""

    def __init__(self, out_dir: str, run_7z: bool, seven_zip: str = "7z"):
        self.out_dir, self.run_7z, self.seven_zip = out_dir, run_7z, seven_zip
        self.procs: list = []
        self.rc = 0
        self.done: set[str] = set()

    def emit(self, name: str, rec: bytes, rc_n: int) -> None:
        try:
            self._emit(name, rec, rc_n)
        except OSError as e:   # an unwritable output folder: this chromosome fails, the job goes on
            print(f"Error: {name}: {e}", file=sys.stderr)
            self.rc = 1

    def _emit(self, name: str, rec: bytes, rc_n: int) -> None:
        import sccg
        self.done.add(name)
        if rc_n and rc_n != sccg.SCCG_E_DELTA_STOI:
            what = {SCCG_E_IO: "cannot read the FASTA files",
                    SCCG_E_OUT: "cannot write the output folder"}.get(rc_n) or sccg.ERRORS.get(rc_n, rc_n)
            print(f"Error: {name}: {what}", file=sys.stderr)
            self.rc = 1
            return
        d = os.path.join(self.out_dir, name)
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, "compressed_genome.txt")
        with open(path, "wb") as f:
            f.write(rec)
        self.written(name, path, rc_n)

    def written(self, name: str, path: str, rc_n: int) -> None:
        """The record file of `name` is closed at `path` (by emit, or by sccg_compress_files
        itself): start its 7z now, unless its delta_encode failed (stoi: text kept, no 7z)."""
        self.done.add(name)
        if rc_n:
            print(f"Error: {name}: stoi", file=sys.stderr)
            self.rc = 1
            return
        if self.run_7z:
            # argv list, no shell: chromosome names come from file names
            self.procs.append(subprocess.Popen([self.seven_zip, "a", "-mx=9", path + ".7z", path],
                                               stdout=subprocess.DEVNULL))

    def wait(self) -> int:
        for p in self.procs:
            r = p.wait()
            if r != 0:
                print(f"Greska prilikom komprimiranja datoteke 7-zipom: {r} !", file=sys.stderr)
                self.rc = 1
        self.procs = []
        return self.rc


def compress_pair_files(ctx, ref_path: str, tgt_path: str, out_dir: str, name: str, em: Emitter | None) -> dict:
    """One pair from FASTA files straight to <out_dir>/<name>/compressed_genome.txt through
    sccg_compress_files (pinned staging, compression.cpp:181-331 without 7z), then its 7z through
    the Emitter.  Returns the pair's stats with its rc (the CLI's failure points as error codes)."""
    import sccg
    d = os.path.join(out_dir, name)
    path = os.path.join(d, "compressed_genome.txt")
    rc_n, st = 0, {}
    try:
        os.makedirs(d, exist_ok=True)
        ctx.compress_files(ref_path, tgt_path, path)
        st = ctx.stats()
    except sccg.SccgError as e:
        rc_n = e.rc
    except OSError as e:   # an unwritable output folder: this chromosome fails, the job goes on
        print(f"Error: {name}: {e}", file=sys.stderr)
        rc_n = SCCG_E_OUT
    except Exception as e:   # noqa: BLE001  (anything else still fails only this pair)
        print(f"Error: {name}: {e}", file=sys.stderr)
        rc_n = sccg.ERR_CODES["SCCG_E_HIP"]
    if em is not None:
        if rc_n and rc_n != sccg.SCCG_E_DELTA_STOI:
            em.emit(name, b"", rc_n)
        else:
            em.written(name, path, rc_n)
    return dict(st, rc=rc_n)


def compress_shard(mine: list[str], ref_dir: str, tgt_dir: str, make_ctx, em: Emitter | None,
                   err_hip: int) -> tuple[dict, dict]:
    """Compress this rank's pairs.  Never raises: a rank that fails (no context, an unreadable
    file, a failing pair) must still enter the gather, or every other rank would hang in the
    collective.  Failures become per-pair error codes (rc) that travel with the stats; rank 0
    reports them as the reference CLI would (compression.cpp:188-191, 203-206: exit 1).
    `make_ctx()` returns an object with compress(ref, tgt) / stats() / close() (sccg.Context)."""
    import sccg
    parts: dict[str, bytes] = {}
    stats: dict[str, dict] = {}
    ctx = None
    try:
        ctx = make_ctx()
    except Exception as e:   # noqa: BLE001
        print(f"Error: no context: {e}", file=sys.stderr)
    for n in mine:
        rec, rc_n, st = b"", 0, {}
        try:
            ref = open(os.path.join(ref_dir, n + ".fa"), "rb").read()
            tgt = open(os.path.join(tgt_dir, n + ".fa"), "rb").read()
        except OSError as e:
            print(f"Error: {n}: {e}", file=sys.stderr)
            rc_n = SCCG_E_IO
        if not rc_n and ctx is None:
            rc_n = err_hip
        if not rc_n:
            # keep a failing pair's rc and whatever text it produced, as the reference CLI does
            try:
                rec = ctx.compress(ref, tgt)
                st = ctx.stats()
            except sccg.SccgError as e:
                rec, rc_n = getattr(e, "partial", None) or b"", e.rc
            except Exception as e:   # noqa: BLE001
                print(f"Error: {n}: {e}", file=sys.stderr)
                rec, rc_n = b"", err_hip
        stats[n] = dict(st, rc=rc_n)
        if em is not None:
            em.emit(n, rec, rc_n)      # rank 0's own chromosomes: 7z starts now
        else:
            parts[n] = rec
    if ctx is not None:
        try:
            ctx.close()
        except Exception:   # noqa: BLE001
            pass
    return parts, stats


def compress_shard_files(mine: list[str], ref_dir: str, tgt_dir: str, make_ctx, em: Emitter, err_hip: int,
                         contexts: int = 2) -> dict:
    """Rank 0's own pairs: FASTA files -> record files through sccg_compress_files, `contexts`
    library contexts each driven by its own host thread (one pair's file reads and copies overlap
    another's kernels), 7z started per pair as its file closes.  Never raises (see compress_shard)."""
    import threading
    stats: dict[str, dict] = {}
    todo = sorted(mine, key=lambda n: -os.path.getsize(os.path.join(tgt_dir, n + ".fa"))
                  if os.path.exists(os.path.join(tgt_dir, n + ".fa")) else 0)
    lock = threading.Lock()

    def worker():
        ctx = None
        try:
            ctx = make_ctx()
        except Exception as e:   # noqa: BLE001
            print(f"Error: no context: {e}", file=sys.stderr)
        try:
            while True:
                with lock:
                    if not todo:
                        break
                    n = todo.pop(0)
                if ctx is None:
                    with lock:
                        stats[n] = {"rc": err_hip}
                        em.emit(n, b"", err_hip)
                    continue
                try:
                    st = compress_pair_files(ctx, os.path.join(ref_dir, n + ".fa"), os.path.join(tgt_dir, n + ".fa"),
                                             em.out_dir, n, None)
                except Exception as e:   # noqa: BLE001  (never lose a pair: it is reported failed)
                    print(f"Error: {n}: {e}", file=sys.stderr)
                    st = {"rc": err_hip}
                with lock:
                    stats[n] = st
                    if st["rc"] and st["rc"] != sccg_delta_stoi():
                        em.emit(n, b"", st["rc"])
                    else:
                        em.written(n, os.path.join(em.out_dir, n, "compressed_genome.txt"), st["rc"])
        finally:
            if ctx is not None:
                try:
                    ctx.close()
                except Exception:   # noqa: BLE001
                    pass

    ths = [threading.Thread(target=worker) for _ in range(max(1, contexts))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return stats


def sccg_delta_stoi() -> int:
    import sccg
    return sccg.SCCG_E_DELTA_STOI


def collect(names: list[str], parts: dict, stats: dict, em: Emitter | None, dev, world: int) -> dict:
    """The job's exchange: every rank's record texts and stats to rank 0 (multigpu.gather_records
    + gather_to_root); rank 0 emits the chromosomes it did not compress itself (a pair no rank
    reported counts as failed).  Returns all stats on rank 0, this rank's elsewhere."""
    import torch
    import multigpu
    if world <= 1:
        return stats
    merged = multigpu.gather_records(parts, device=dev)
    st_blob = json.dumps(stats).encode()
    got = multigpu.gather_to_root(torch.frombuffer(bytearray(st_blob), dtype=torch.uint8).to(dev), len(st_blob))
    if got is None:
        return stats
    all_stats: dict = {}
    for g in got:
        all_stats.update(json.loads(g.cpu().numpy().tobytes()))
    for n in names:
        if n not in em.done:
            if n in merged and n in all_stats:
                em.emit(n, merged[n], all_stats[n]["rc"])
            else:
                print(f"Error: {n}: no rank reported it", file=sys.stderr)
                em.rc = 1
    return all_stats


def cost_weights(names: list, sizes: list, cost: dict) -> list:
    """LPT weights in one unit: a pair the cost file lists weighs its measured cost; a pair it does
    not list weighs its target size scaled by the median cost per byte of the listed pairs (a bare
    byte count next to costs of ~10 ms would put that pair alone on a rank)."""
    per_byte = sorted(cost[n] / s for n, s in zip(names, sizes) if n in cost and s > 0)
    scale = per_byte[len(per_byte) // 2] if per_byte else 1.0
    return [float(cost[n]) if n in cost else s * scale for n, s in zip(names, sizes)]


def load_cost(path: str) -> dict:
    with open(path) as f:
        return json.load(f)


def run_job(names: list[str], ref_dir: str, tgt_dir: str, out_dir: str, make_ctx, rank: int, world: int, dev,
            contexts: int = 2, run_7z: bool = True, seven_zip: str = "7z", err_hip: int | None = None,
            cost: dict | None = None) -> tuple[int, dict | None]:
    """The whole job on one rank: shard, compress, gather, emit.  Rank 0 writes its own pairs'
    record files straight from the library (sccg_compress_files) and the other ranks' after the
    gather.  `cost` (name -> measured cost, e.g. per-pair GPU ms) shards by cost instead of target
    size (a T2T-like pair's walk time is not proportional to its length).  Returns (rc, summary)
    on rank 0 and (0, None) elsewhere."""
    import multigpu
    if err_hip is None:
        import sccg
        err_hip = sccg.ERR_CODES["SCCG_E_HIP"]
    sizes = [os.path.getsize(os.path.join(tgt_dir, n + ".fa")) if os.path.exists(os.path.join(tgt_dir, n + ".fa"))
             else 0 for n in names]
    weights = cost_weights(names, sizes, cost) if cost else sizes
    mine = [names[i] for i in multigpu.lpt_shard(weights, world)[rank]]
    em = Emitter(out_dir, run_7z, seven_zip) if rank == 0 else None
    t0 = time.perf_counter()
    if em is not None:   # rank 0: files straight to record files (sccg_compress_files)
        parts, stats = {}, compress_shard_files(mine, ref_dir, tgt_dir, make_ctx, em, err_hip, contexts)
    else:
        parts, stats = compress_shard(mine, ref_dir, tgt_dir, make_ctx, em, err_hip)
    t_comp = time.perf_counter() - t0
    all_stats = collect(names, parts, stats, em, dev, world)
    if rank != 0:
        return 0, None
    rc = em.wait()
    return rc, {"chromosomes": len(names), "target_fasta_bytes": sum(sizes), "ranks": world,
                "compress_seconds_rank0": t_comp, "per_chrom": all_stats}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref-dir", required=True)
    ap.add_argument("--tgt-dir", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--names", default="", help="comma-separated subset (default: all common *.fa)")
    ap.add_argument("--no-7z", action="store_true")
    ap.add_argument("--contexts", type=int, default=2, help="rank 0: library contexts (host threads) on its GPU")
    ap.add_argument("--cost", default="", help="JSON file {name: measured cost} to shard by (default: target size)")
    args = ap.parse_args(argv)

    import torch
    import torch.distributed as dist
    import multigpu
    import sccg

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    names = sorted(f[:-3] for f in os.listdir(args.tgt_dir)
                   if f.endswith(".fa") and os.path.exists(os.path.join(args.ref_dir, f)))
    if args.names:
        keep = set(args.names.split(","))
        names = [n for n in names if n in keep]
    rc, summary = run_job(names, args.ref_dir, args.tgt_dir, args.out, lambda: sccg.Context(local), rank, world, dev,
                          contexts=args.contexts, run_7z=not args.no_7z,
                          cost=load_cost(args.cost) if args.cost else None)
    if rank == 0:
        print(json.dumps(summary))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())
