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
        import sccg
        self.done.add(name)
        if rc_n and rc_n != sccg.SCCG_E_DELTA_STOI:
            print(f"Error: {name}: {sccg.ERRORS.get(rc_n, rc_n)}", file=sys.stderr)
            self.rc = 1
            return
        d = os.path.join(self.out_dir, name)
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, "compressed_genome.txt")
        with open(path, "wb") as f:
            f.write(rec)
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


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref-dir", required=True)
    ap.add_argument("--tgt-dir", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--names", default="", help="comma-separated subset (default: all common *.fa)")
    ap.add_argument("--no-7z", action="store_true")
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
    sizes = [os.path.getsize(os.path.join(args.tgt_dir, n + ".fa")) for n in names]
    mine = [names[i] for i in multigpu.lpt_shard(sizes, world)[rank]]
    em = Emitter(args.out, not args.no_7z) if rank == 0 else None

    t0 = time.perf_counter()
    parts: dict[str, bytes] = {}
    stats: dict[str, dict] = {}
    with sccg.Context(local) as ctx:
        for n in mine:
            ref = open(os.path.join(args.ref_dir, n + ".fa"), "rb").read()
            tgt = open(os.path.join(args.tgt_dir, n + ".fa"), "rb").read()
            # a failing pair must not leave this rank out of the gather (the others would hang):
            # keep its rc and whatever text it produced, as the reference CLI does
            try:
                rec, rc_n = ctx.compress(ref, tgt), 0
            except sccg.SccgError as e:
                rec, rc_n = getattr(e, "partial", None) or b"", e.rc
            stats[n] = dict(ctx.stats(), rc=rc_n)
            if em is not None:
                em.emit(n, rec, rc_n)      # rank 0's own chromosomes: 7z starts now
            else:
                parts[n] = rec
    t_comp = time.perf_counter() - t0
    all_stats = stats
    if world > 1:
        merged = multigpu.gather_records(parts, device=dev)
        st_blob = json.dumps(stats).encode()
        got = multigpu.gather_to_root(torch.frombuffer(bytearray(st_blob), dtype=torch.uint8).to(dev),
                                      len(st_blob))
        if got is not None:
            all_stats = {}
            for g in got:
                all_stats.update(json.loads(g.cpu().numpy().tobytes()))
            for n in names:
                if n not in em.done:
                    em.emit(n, merged[n], all_stats[n]["rc"])
    rc = 0
    if rank == 0:
        rc = em.wait()
        print(json.dumps({"chromosomes": len(names), "target_fasta_bytes": sum(sizes), "ranks": world,
                          "compress_seconds_rank0": t_comp, "per_chrom": all_stats}))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())
