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

    t0 = time.perf_counter()
    parts: dict[str, torch.Tensor] = {}
    stats = {}
    with sccg.Context(local) as ctx:
        for n in mine:
            ref = open(os.path.join(args.ref_dir, n + ".fa"), "rb").read()
            tgt = open(os.path.join(args.tgt_dir, n + ".fa"), "rb").read()
            rec = ctx.compress(ref, tgt)
            stats[n] = ctx.stats()
            parts[n] = torch.frombuffer(bytearray(rec), dtype=torch.uint8).to(dev) if rec else \
                torch.zeros(0, dtype=torch.uint8, device=dev)
    t_comp = time.perf_counter() - t0
    if world > 1:
        merged = multigpu.gather_records(parts, device=dev)
    else:
        merged = {n: t.cpu().numpy().tobytes() for n, t in parts.items()}
    rc = 0
    if rank == 0:
        # 7z per chromosome (compression.cpp:308), all archives compressed concurrently on the host
        # (LZMA2 on ~80 MB of record text is the job's remaining CPU time)
        procs = []
        for n in names:
            d = os.path.join(args.out, n)
            os.makedirs(d, exist_ok=True)
            path = os.path.join(d, "compressed_genome.txt")
            with open(path, "wb") as f:
                f.write(merged[n])
            if not args.no_7z:
                procs.append(subprocess.Popen(f'7z a -mx=9 "{path}.7z" "{path}"', shell=True, stdout=subprocess.DEVNULL))
        for p in procs:
            r = p.wait()
            if r != 0:
                print(f"Greska prilikom komprimiranja datoteke 7-zipom: {r} !", file=sys.stderr)
                rc = 1
        total = sum(sizes)
        print(json.dumps({"chromosomes": len(names), "target_fasta_bytes": total, "ranks": world,
                          "compress_seconds_rank0": t_comp, "per_chrom": {n: stats.get(n) for n in mine}}))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())
