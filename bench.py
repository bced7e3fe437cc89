#!/usr/bin/env python3
"""bench.py -- target bases compressed per second on MI355X (BASELINE.json metric).

Workload (configs[1]): a chr1-sized hg19-vs-hg18 pair (|R| = 247,249,719, |T| = 249,250,621),
synthetic (tools/synth.c "hg" profile; real FASTA is not available offline).  One step = the whole
hot path on resident inputs: both FASTA texts already in HBM -> compressed_genome.txt bytes in
HBM (ingest, lowercase line, local segments + switch, N line, N erase, global walk, delta-encoded
record text).  7z is outside the path, as in the reference's own timing split.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Multi-GPU: chromosomes are independent, so every rank compresses its own chr1-shaped pair
(seed 1+rank; weak scaling) and the per-chromosome record streams are gathered to rank 0 over
RCCL inside the step, as the whole-genome driver does.

Printed (rank 0): one JSON line with value = all ranks' target bases / max-over-ranks time, the
roofline of the dominant kernel (HIP events on the library's stream, algorithmic bytes from
DESIGN.md §4) and the reference CPU path timed on a bounded sample on this host.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(REPO, "sccg-genome-compression_amd")
sys.path.insert(0, PKG_DIR)

CHR1 = (247_249_719, 249_250_621)   # hg18 / hg19 chr1 (UCSC chromInfo)
HBM_PEAK_GBS = 8000.0               # MI355X_MICROARCH.md: 8.0 TB/s spec
METRIC = "target bases compressed/sec at 1/2/4/8 GPUs; bit-exact record stream vs CPU ref"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes(kernel: str, shape: dict) -> float | None:
    """Algorithmic HBM bytes of ONE launch of `kernel` for this workload."""
    nT, nR = shape["target_bases"], shape["reference_bases"]
    if kernel == "fasta_strip":       # read the FASTA, write the kept bytes (target and reference launch)
        return (shape["tgt_fa"] + nT + shape["ref_fa"] + nR) / 2.0
    if kernel == "local_segments":    # both segment strings once + records and stats
        lead = min(nR, nT)
        return 2.0 * lead + (lead / 1000.0) * (1024 + 32)
    if kernel == "walk":              # every target base once + the matched reference bases once
        return None                   # per-launch bytes vary by round; see walk_bytes below
    if kernel in ("run_extract", "n_filter"):
        return float(nT + nT)
    if kernel == "first_sweep_anchors":   # R' once + one 8-byte anchor slot per 32 reference bases
        return float(nR + nR / 32 * 8)
    return None


def cpu_baseline(sample_bases: int) -> dict | None:
    """The reference compression.cpp (oracle/_ref, built from /root/reference) on a bounded
    sample of the same workload shape, single-threaded, stub 7z, stdout discarded."""
    import synth
    ref_bin = os.path.join(REPO, "oracle", "_ref", "compression")
    kind = "reference"
    if not os.path.exists(ref_bin):
        ref_bin = os.path.join(REPO, "oracle", "sccg_oracle")
        kind = "port"
        if not os.path.exists(ref_bin):
            return None
    rl, tl = sample_bases, sample_bases + sample_bases // 400
    rfa, tfa = synth.synth_pair("hg", rl, tl, 101)
    d = tempfile.mkdtemp(prefix="sccg_cpu_")
    try:
        rp, tp = os.path.join(d, "ref.fa"), os.path.join(d, "tgt.fa")
        open(rp, "wb").write(rfa)
        open(tp, "wb").write(tfa)
        env = dict(os.environ, PATH=os.path.join(REPO, "oracle", "stub7z") + os.pathsep + os.environ.get("PATH", ""))
        if kind == "reference":
            cmd = [ref_bin, rp, tp, os.path.join(d, "out")]
        else:
            cmd = [ref_bin, "compress", rp, tp, os.path.join(d, "out.txt")]
        t0 = time.perf_counter()
        p = subprocess.run(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=600)
        dt = time.perf_counter() - t0
        if p.returncode != 0:
            return None
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return {"value": tl / dt, "unit": "target bases/s", "cores": 1, "kind": kind,
            "sample": f"hg-profile synthetic pair |R|={rl:,} |T|={tl:,} (seed 101), wall {dt:.2f} s, "
                      f"single-threaded, stub 7z, stdout to /dev/null"}


def load_pmc(kernel: str) -> float | None:
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc summary, if any."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None
    try:
        doc = json.load(open(path))
        return doc.get(kernel, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu-sample", type=int, default=10_000_000, help="reference CPU sample size (bases)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the round-trip parity check")
    ap.add_argument("--no-prof", action="store_true", help="no per-kernel HIP events in the timed region (A/B of their cost)")
    ap.add_argument("--ref-len", type=int, default=CHR1[0])
    ap.add_argument("--tgt-len", type=int, default=CHR1[1])
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import sccg
    import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    t0 = time.perf_counter()
    rfa, tfa = synth.synth_pair("hg", args.ref_len, args.tgt_len, 1 + rank)
    log(f"[rank {rank}] generated pair in {time.perf_counter() - t0:.1f} s "
        f"({len(rfa):,} + {len(tfa):,} FASTA bytes)")
    d_ref = torch.frombuffer(bytearray(rfa), dtype=torch.uint8).to(dev)
    d_tgt = torch.frombuffer(bytearray(tfa), dtype=torch.uint8).to(dev)
    ctx = sccg.Context(local)
    cap = ctx.compress_bound(len(rfa), len(tfa))
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    import multigpu
    gathered: list = [None]

    def step() -> int:
        n = ctx.compress_device(d_ref.data_ptr(), len(rfa), d_tgt.data_ptr(), len(tfa), d_out.data_ptr(), cap, stream)
        if world > 1:
            # per-chromosome record streams -> rank 0 over RCCL (multigpu.gather_to_root, the
            # genome driver's exchange): one size all-gather, then a gather of each rank's output
            # prefix straight out of d_out; only rank 0 receives
            gathered[0] = multigpu.gather_to_root(d_out, n)
        return n

    for _ in range(args.warmup):
        n_out = step()
    ctx.profile(not args.no_prof)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        n_out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    prof = ctx.profile_get()
    ctx.profile(False)
    st = ctx.stats()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    gather_ok = None
    if world > 1 and rank == 0:
        parts = gathered[0]
        gather_ok = all(p.numel() > 0 for p in parts) and torch.equal(parts[0], d_out[:n_out])
        if not gather_ok:
            raise SystemExit("bench: gathered record streams are wrong (empty part or rank 0 mismatch)")
    parity = None
    if not args.no_check:
        rec = d_out[:n_out].cpu().numpy().tobytes()
        fa = ctx.reconstruct(rec, rfa)
        parity = {"roundtrip_exact": fa == tfa, "record_sha256": hashlib.sha256(rec).hexdigest(),
                  "record_bytes": len(rec)}

    if rank == 0:
        nT = st["target_bases"]
        value = world * nT * args.steps / dt
        shape = {"target_bases": nT, "reference_bases": st["reference_bases"], "tgt_fa": len(tfa), "ref_fa": len(rfa)}
        kernels = {k: {"ms_per_step": v[0] / args.steps, "launches_per_step": v[1] / args.steps,
                       "avg_launch_ms": v[0] / v[1]} for k, v in prof.items()}
        roof = None
        if prof:
            dom = max(prof, key=lambda k: prof[k][0])
            avg_ms = prof[dom][0] / prof[dom][1]
            alg = algorithmic_bytes(dom, shape)
            if dom == "walk":
                # whole-walk algorithmic bytes (2 B per target base: T' once + R' along matches)
                alg = 2.0 * nT * args.steps / prof[dom][1]
            if alg is not None:
                achieved = alg / (avg_ms * 1e-3) / 1e9
                traffic = load_pmc(dom)
                roof = {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                        "traffic": traffic, "alg_bytes_per_launch": alg, "avg_launch_ms": avg_ms}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args.cpu_sample)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "target bases/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (tools/synth.c hg profile, seed 1+rank); real hg18/hg19 unavailable offline",
            "config": {"workload": "hg19-vs-hg18 chr1-sized pair (BASELINE configs[1]), one pair per GPU",
                       "reference_bases": st["reference_bases"], "target_bases": nT,
                       "mode": "global" if st["mode_global"] else "local",
                       "switch_segment": st["switch_segment"], "matches": st["n_matches"],
                       "walk_rounds": st["walk_rounds"], "walk_chunks": st["walk_chunks"],
                       "parallelism": f"chromosome-sharded x{world}, RCCL gather of record streams"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity": parity,
            "kernels": kernels,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
