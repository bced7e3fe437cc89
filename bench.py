#!/usr/bin/env python3
"""bench.py -- target bases compressed per second on MI355X (BASELINE.json metric).

Workload (BASELINE configs[2], the north-star job): the whole hg19-vs-hg18 genome -- the 24
chromosome pairs chr1..22, X, Y at their UCSC lengths (hg18 = reference, hg19 = target,
multigpu.HG18 / HG19), synthetic (tools/synth.c "hg" profile, seed = chromosome index 1..24; real
FASTA is not available offline).  One compression.cpp invocation per pair, exactly as the
reference runs it (compression.cpp:584-610), at the reference's own parameters (k = 14, m = 100,
compression.cpp:373-379).

One step = every pair of this rank's LPT shard compressed on its GPU (FASTA texts already resident
in HBM -> compressed_genome.txt bytes in HBM: ingest, lowercase line, local segments + switch, N
line, N erase, global walk, delta-encoded record text), then the per-chromosome record streams
gathered to rank 0 over RCCL (the job's only exchange).  7z is outside the path, as in the
reference's own timing split.  `--contexts C` runs C library contexts per GPU, each driven by its
own host thread, so one pair's host round trips overlap another pair's kernels.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Printed (rank 0): one JSON line.  value = the genome's target bases / max-over-ranks step time
(strong scaling: the job is fixed, N GPUs share it); roofline of the dominant kernel (HIP events
on the launching streams, SURVEY §8(d) algorithmic bytes) and of the whole job; the reference
compression.cpp timed on this host on BASELINE configs[0] (the chr21 pair); the chr1 record
stream reconstructed on the GPU (configs[3]); per-chromosome sha256 checked against the
reference's, pinned in tests/golden/genome_manifest.json.
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
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(REPO, "sccg-genome-compression_amd")
sys.path.insert(0, PKG_DIR)

HBM_PEAK_GBS = 8000.0               # MI355X_MICROARCH.md: 8.0 TB/s spec
METRIC = "target bases compressed/sec at 1/2/4/8 GPUs; bit-exact record stream vs CPU ref"
MANIFEST = os.path.join(REPO, "tests", "golden", "genome_manifest.json")
# GPU_MAX_HW_QUEUES for the run: 0 keeps the environment's (HIP's default, 4).  Measured on the
# genome bench (profiles/r03_ab.txt): 2 contexts with 4 queues 24.1-24.5 ms per step, with 8 queues
# 28.0-28.3 ms, 3 contexts with 8-12 queues 26.0-31.3 ms, 1 context 29.8-29.9 ms.
HW_QUEUES_DEFAULT = 0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def walk_alg_bytes(nT: int) -> float:
    """the walk's share of B_global, 0.5 B per target base (packed target + packed
    reference along the matches)."""
    return 0.5 * nT


def job_alg_bytes(nT: int, nR: int, nRp: int, out: int) -> float:
    """SURVEY §8(d) B_global = 1.25(|T|+|R|) + 0.25|R| + 4|R'| + 0.5|T| + |out|."""
    return 1.25 * (nT + nR) + 0.25 * nR + 4.0 * nRp + 0.5 * nT + out


def kernel_alg_bytes(kernel: str, tot: dict) -> float | None:
    """Algorithmic HBM bytes of one STEP of `kernel` summed over the step's pairs."""
    if kernel == "walk":
        return walk_alg_bytes(tot["target_bases"])
    if kernel == "fasta_strip":          # read the FASTA, write the stripped and the N-erased copies
        return tot["tgt_fa"] + tot["ref_fa"] + 2.0 * (tot["target_bases"] + tot["reference_bases"])
    if kernel == "run_extract":          # T once
        return float(tot["target_bases"])
    if kernel == "first_sweep_anchors":  # R' once + one 8-byte anchor slot per 32 reference bases
        return tot["reference_bases"] * (1.0 + 8.0 / 32.0)
    if kernel == "local_segments":       # both segment strings (up to the switch, bounded by all of them)
        return 2.0 * min(tot["target_bases"], tot["reference_bases"])
    return None


def load_manifest() -> dict:
    try:
        return {e["name"]: e for e in json.load(open(MANIFEST))}
    except Exception:
        return {}


def cpu_baseline(timeout_s: int) -> dict | None:
    """The reference compression.cpp (oracle/_ref, compiled from /root/reference's sources) on
    BASELINE configs[0]: the chr21 pair (hg18 chr21 = 46,944,323 vs hg19 chr21 = 48,129,895,
    seed 21 -- the same pair the genome job compresses), single-threaded, stub 7z, stdout to
    /dev/null.  Falls back to the C restatement (oracle/sccg_oracle) if the reference binary is
    absent.  The record sha256 is compared with the pinned manifest."""
    import multigpu
    import synth
    ref_bin = os.path.join(REPO, "oracle", "_ref", "compression")
    kind = "reference"
    if not os.path.exists(ref_bin):
        ref_bin = os.path.join(REPO, "oracle", "sccg_oracle")
        kind = "port"
        if not os.path.exists(ref_bin):
            return None
    i = multigpu.CHROMS.index("chr21")
    rl, tl = multigpu.HG18[i], multigpu.HG19[i]
    rfa, tfa = synth.synth_pair("hg", rl, tl, i + 1)
    d = tempfile.mkdtemp(prefix="sccg_cpu_")
    try:
        rp, tp = os.path.join(d, "ref.fa"), os.path.join(d, "tgt.fa")
        open(rp, "wb").write(rfa)
        open(tp, "wb").write(tfa)
        del rfa, tfa
        env = dict(os.environ, PATH=os.path.join(REPO, "oracle", "stub7z") + os.pathsep + os.environ.get("PATH", ""))
        if kind == "reference":
            outp = os.path.join(d, "out")
            cmd = [ref_bin, rp, tp, outp]
            rec_path = os.path.join(outp, "compressed_genome.txt")
        else:
            rec_path = os.path.join(d, "out.txt")
            cmd = [ref_bin, "compress", rp, tp, rec_path]
        t0 = time.perf_counter()
        p = subprocess.run(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=timeout_s)
        dt = time.perf_counter() - t0
        if p.returncode != 0:
            return None
        sha = hashlib.sha256(open(rec_path, "rb").read()).hexdigest()
    except subprocess.TimeoutExpired:
        return None
    finally:
        shutil.rmtree(d, ignore_errors=True)
    pin = load_manifest().get("chr21", {}).get("record_sha256")
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": tl / dt, "unit": "target bases/s", "cores": 1, "kind": kind,
            "sample": f"BASELINE configs[0]: hg19-vs-hg18 chr21-sized synthetic pair |R|={rl:,} |T|={tl:,} (seed 21), "
                      f"wall {dt:.1f} s, single-threaded ({cpu}), stub 7z, stdout to /dev/null",
            "record_matches_pinned": (sha == pin) if pin else None}


def end_to_end(ctx, rfa: bytes, tfa: bytes, pinned_sha: str | None, reps: int = 3) -> dict:
    """SURVEY §8(d)'s end-to-end rate: FASTA files -> compressed_genome.txt closed (7z excluded),
    through sccg_compress_files (host reads into pinned staging, H2D overlapped with the reading and
    the reference's GPU work, record text written back).  Files sit in the page cache (written just
    before), so this is the host-memory + PCIe path, not the disk's."""
    d = tempfile.mkdtemp(prefix="sccg_e2e_")
    try:
        rp, tp, op = os.path.join(d, "ref.fa"), os.path.join(d, "tgt.fa"), os.path.join(d, "compressed_genome.txt")
        open(rp, "wb").write(rfa)
        open(tp, "wb").write(tfa)
        ctx.compress_files(rp, tp, op)   # warm: staging buffers, device buffers
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            n = ctx.compress_files(rp, tp, op)
            ts.append(time.perf_counter() - t0)
        rec = open(op, "rb").read()
        nT = ctx.stats()["target_bases"]
    finally:
        shutil.rmtree(d, ignore_errors=True)
    dt = min(ts)
    sha = hashlib.sha256(rec).hexdigest()
    return {"workload": "chr1 pair: FASTA files (page cache) -> compressed_genome.txt closed, 7z excluded",
            "target_bases": nT, "fasta_bytes": len(rfa) + len(tfa), "record_bytes": n, "ms": dt * 1e3,
            "ms_all": [round(t * 1e3, 2) for t in ts], "bases_per_s": nT / dt,
            "host_to_file_GBps": (len(rfa) + len(tfa)) / dt / 1e9,
            "record_matches_pinned": (sha == pinned_sha) if pinned_sha else None}


class Lane:
    """One library context + its stream, output buffer and host thread."""

    def __init__(self, sccg, torch, dev, cap: int, device_index: int):
        self.ctx = sccg.Context(device_index)
        self.stream = torch.cuda.Stream(dev)
        self.out = torch.empty(cap, dtype=torch.uint8, device=dev)
        self.cap = cap


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--contexts", type=int, default=2, help="library contexts (host threads) per GPU")
    ap.add_argument("--queue", choices=["lpt", "twoend"], default="lpt",
                    help="pair order over the contexts: largest first onto the first free context (lpt), or "
                         "even contexts from the largest end and odd ones from the smallest (twoend)")
    ap.add_argument("--hw-queues", type=int, default=HW_QUEUES_DEFAULT,
                    help="GPU_MAX_HW_QUEUES for this process (0: leave the environment's)")
    ap.add_argument("--workload", choices=["genome", "chr1"], default="genome",
                    help="genome: BASELINE configs[2] (default); chr1: one chr1-sized pair per rank (configs[1] shape)")
    ap.add_argument("--names", default="", help="comma-separated subset of chromosomes (diagnostics)")
    ap.add_argument("--cpu-timeout", type=int, default=300)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the pinned sha256 checks")
    ap.add_argument("--no-decomp", action="store_true", help="skip the configs[3] reconstruction")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (files) measurement")
    ap.add_argument("--no-prof", action="store_true", help="no per-kernel HIP events in the timed region")
    args = ap.parse_args()
    if args.hw_queues > 0:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(args.hw_queues, 32))   # before HIP initialises

    import torch
    import torch.distributed as dist
    import multigpu
    import sccg
    import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    # ---- the job: chromosome pairs, LPT-sharded by target size (multigpu.lpt_shard)
    if args.workload == "genome":
        jobs = [(n, multigpu.HG18[i], multigpu.HG19[i], i + 1) for i, n in enumerate(multigpu.CHROMS)]
        if args.names:
            keep = set(args.names.split(","))
            jobs = [j for j in jobs if j[0] in keep]
        mine = [jobs[i] for i in multigpu.lpt_shard([j[2] for j in jobs], world)[rank]]
    else:
        jobs = [(f"chr1_r{r}", multigpu.HG18[0], multigpu.HG19[0], 1 + r) for r in range(world)]
        mine = [jobs[rank]]

    # ---- inputs: generated on the host (threads: the C generator releases the GIL), then resident
    t0 = time.perf_counter()
    pairs: dict = {}
    host_fa: dict = {}
    lock = threading.Lock()

    def gen(job):
        name, rl, tl, seed = job
        rfa, tfa = synth.synth_pair("hg", rl, tl, seed)
        with lock:
            host_fa[name] = (rfa, tfa)

    ths = [threading.Thread(target=gen, args=(j,)) for j in mine]
    nthr = 8
    for b in range(0, len(ths), nthr):
        for t in ths[b:b + nthr]:
            t.start()
        for t in ths[b:b + nthr]:
            t.join()
    for name, rl, tl, seed in mine:
        rfa, tfa = host_fa[name]
        pairs[name] = (torch.frombuffer(bytearray(rfa), dtype=torch.uint8).to(dev), len(rfa),
                       torch.frombuffer(bytearray(tfa), dtype=torch.uint8).to(dev), len(tfa))
    keep_chr1 = host_fa.get("chr1") or host_fa.get(f"chr1_r{rank}")
    tgt_fa_bytes = sum(len(v[1]) for v in host_fa.values())
    ref_fa_bytes = sum(len(v[0]) for v in host_fa.values())
    host_fa.clear()
    torch.cuda.synchronize()
    log(f"[rank {rank}] {len(mine)} pairs generated and resident in {time.perf_counter() - t0:.1f} s "
        f"({ref_fa_bytes + tgt_fa_bytes:,} FASTA bytes)")

    n_lanes = max(1, min(args.contexts, len(mine)))
    cap = max(sccg.Context.compress_bound_static(p[1], p[3]) for p in pairs.values())
    lanes = [Lane(sccg, torch, dev, cap, local) for _ in range(n_lanes)]
    order = sorted(pairs, key=lambda n: -pairs[n][3])   # largest first onto the first free lane
    results: dict = {}      # name -> (device tensor of its record text, stats)
    errors: list = []

    # persistent lane threads: a step releases them through one barrier and joins them at another
    # (no thread start per step)
    nxt = [0, len(order) - 1]   # next from the largest end, next from the smallest end
    qlock = threading.Lock()
    lane_idx = {id(ln): i for i, ln in enumerate(lanes)}
    go = threading.Barrier(n_lanes + 1)
    done = threading.Barrier(n_lanes + 1)
    stop = [False]

    def worker(lane: Lane) -> None:
        torch.cuda.set_device(dev)
        while True:
            go.wait()
            if stop[0]:
                return
            try:
                small_end = args.queue == "twoend" and lane_idx[id(lane)] % 2 == 1
                while True:
                    with qlock:
                        if nxt[0] > nxt[1]:
                            break
                        if small_end:
                            name = order[nxt[1]]
                            nxt[1] -= 1
                        else:
                            name = order[nxt[0]]
                            nxt[0] += 1
                    dr, rn, dt_, tn = pairs[name]
                    n = lane.ctx.compress_device(dr.data_ptr(), rn, dt_.data_ptr(), tn, lane.out.data_ptr(), lane.cap,
                                                 lane.stream.cuda_stream)
                    st = lane.ctx.stats()
                    prev = results.get(name)
                    with torch.cuda.stream(lane.stream):
                        buf = prev[0] if prev is not None and prev[0].numel() == n else \
                            torch.empty(n, dtype=torch.uint8, device=dev)
                        buf.copy_(lane.out[:n])   # the pair's record stream, kept for the gather
                    results[name] = (buf, st)
            except Exception as e:   # noqa: BLE001 -- reported after the step
                errors.append(e)
            done.wait()

    lane_threads = [threading.Thread(target=worker, args=(ln,), daemon=True) for ln in lanes]
    for t in lane_threads:
        t.start()

    def run_shard() -> None:
        nxt[0], nxt[1] = 0, len(order) - 1
        go.wait()
        done.wait()
        if errors:
            raise errors[0]

    gathered: list = [None]

    def step() -> None:
        run_shard()
        for ln in lanes:
            ln.stream.synchronize()
        if world > 1:
            # per-chromosome record streams -> rank 0 over RCCL (multigpu.gather_records): one size
            # all-gather, then one gather of each rank's packed streams; only rank 0 receives
            gathered[0] = multigpu.gather_records({n: results[n][0] for n in order}, device=dev)

    for _ in range(args.warmup):
        step()
    lanes[0].ctx.profile(not args.no_prof)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    prof = lanes[0].ctx.profile_get()
    lanes[0].ctx.profile(False)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # ---- per-rank totals (all ranks' target bases make up the whole job)
    tot = {"target_bases": sum(results[n][1]["target_bases"] for n in order),
           "reference_bases": sum(results[n][1]["reference_bases"] for n in order),
           "record_bytes": sum(int(results[n][0].numel()) for n in order),
           "tgt_fa": tgt_fa_bytes, "ref_fa": ref_fa_bytes}
    totals = [tot]
    if world > 1:
        got = [None] * world
        dist.all_gather_object(got, tot)
        totals = got
    job = {k: sum(t[k] for t in totals) for k in tot}

    # ---- parity: every chromosome's record stream against the reference's pinned sha256
    parity = None
    if not args.no_check:
        streams = {}
        if world > 1:
            if rank == 0:
                streams = gathered[0]
        else:
            streams = {n: results[n][0].cpu().numpy().tobytes() for n in order}
        if rank == 0:
            pins = load_manifest()
            checked = [n for n in streams if n in pins and args.workload == "genome"]
            bad = [n for n in checked if hashlib.sha256(streams[n]).hexdigest() != pins[n]["record_sha256"]]
            parity = {"chromosomes": len(streams), "pinned_checked": len(checked), "pinned_mismatch": bad,
                      "reference": "oracle/_ref (compression.cpp compiled unchanged), tests/golden/genome_manifest.json"}
            if args.workload == "chr1":
                parity["record_sha256"] = hashlib.sha256(next(iter(streams.values()))).hexdigest()
            if bad:
                raise SystemExit(f"bench: record streams differ from the reference for {bad}")

    # ---- configs[3]: the chr1 record stream back to FASTA on this GPU (rank 0, outside the step)
    decomp = None
    if rank == 0 and not args.no_decomp and keep_chr1 is not None:
        name = "chr1" if "chr1" in results else f"chr1_r{rank}"
        rfa_h, tfa_h = keep_chr1
        dr, rn, _, _ = pairs[name]
        rec = results[name][0]
        ctx = lanes[0].ctx
        s = lanes[0].stream
        need = ctx.reconstruct_device(dr.data_ptr(), rn, rec.data_ptr(), rec.numel(), 0, 0, s.cuda_stream)
        d_fa = torch.empty(need + 64, dtype=torch.uint8, device=dev)
        ks = max(3, args.steps)
        ctx.reconstruct_device(dr.data_ptr(), rn, rec.data_ptr(), rec.numel(), d_fa.data_ptr(), need + 64, s.cuda_stream)
        s.synchronize()
        t1 = time.perf_counter()
        for _ in range(ks):
            n_fa = ctx.reconstruct_device(dr.data_ptr(), rn, rec.data_ptr(), rec.numel(), d_fa.data_ptr(), need + 64,
                                          s.cuda_stream)
        s.synchronize()
        ddt = (time.perf_counter() - t1) / ks
        # per-kernel HIP events in separate calls: around the reconstruction's short kernels they
        # cost ~10 % of its time (the timed calls above run without them)
        dprof = {}
        if not args.no_prof:
            ctx.profile(True)
            for _ in range(ks):
                ctx.reconstruct_device(dr.data_ptr(), rn, rec.data_ptr(), rec.numel(), d_fa.data_ptr(), need + 64,
                                       s.cuda_stream)
            s.synchronize()
            dprof = ctx.profile_get()
            ctx.profile(False)
        exact = d_fa[:n_fa].cpu().numpy().tobytes() == tfa_h
        nTd = ctx.stats()["target_bases"]
        b_dec = rec.numel() + rn + n_fa + nTd   # SURVEY §8(d) B_decomp = |rec| + |R| + |T_fa| + |T_matched| (<= |T|)
        decomp = {"workload": "BASELINE configs[3]: chr1 record stream -> FASTA on 1 GPU", "target_bases": nTd,
                  "ms": ddt * 1e3, "bases_per_s": nTd / ddt, "roundtrip_exact": exact,
                  "roofline_job": {"bound": "hbm", "alg_bytes": b_dec, "achieved": b_dec / ddt / 1e9,
                                   "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": b_dec / ddt / 1e9 / HBM_PEAK_GBS},
                  "kernels": {k: {"ms_per_call": v[0] / ks, "launches_per_call": v[1] / ks} for k, v in dprof.items()}}
        if not exact:
            raise SystemExit("bench: chr1 reconstruction differs from the target FASTA")

    e2e = None
    if rank == 0 and not args.no_e2e and keep_chr1 is not None:
        pin = load_manifest().get("chr1", {}).get("record_sha256") if args.workload == "genome" else None
        e2e = end_to_end(lanes[0].ctx, keep_chr1[0], keep_chr1[1], pin)

    if rank == 0:
        value = job["target_bases"] * args.steps / dt
        ms_step = dt * 1e3 / args.steps
        kernels = {k: {"ms_per_step": v[0] / args.steps, "launches_per_step": v[1] / args.steps,
                       "avg_launch_ms": v[0] / v[1]} for k, v in prof.items()}
        roof = None
        if prof:
            dom = max(prof, key=lambda k: prof[k][0])
            alg_step = kernel_alg_bytes(dom, tot)
            if alg_step is not None:
                launches_step = prof[dom][1] / args.steps
                avg_ms = prof[dom][0] / prof[dom][1]
                alg = alg_step / launches_step
                achieved = alg / (avg_ms * 1e-3) / 1e9
                roof = {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                        "alg_bytes_per_launch": alg, "avg_launch_ms": avg_ms,
                        "alg_model": "SURVEY §8(d): walk = 0.5 B per target base (packed T' + packed R' along matches)"
                        if dom == "walk" else "DESIGN.md §4"}
                pmc = load_pmc(dom)
                if pmc:
                    roof["traffic"] = pmc["hbm_bytes_per_launch"]
                    roof["traffic_over_alg"] = round(pmc["hbm_bytes_per_launch"] / alg, 3)
                    roof["traffic_source"] = pmc["source"]
        nRp = sum(results[n][1]["reference_bases"] for n in order)   # |R'| <= |R| (N erased); bound
        b_job = sum(job_alg_bytes(results[n][1]["target_bases"], results[n][1]["reference_bases"],
                                  results[n][1]["reference_bases"], int(results[n][0].numel())) for n in order)
        if world > 1:
            b_job = b_job * job["target_bases"] / max(1, tot["target_bases"])   # other ranks: same model per base
        roof_job = {"bound": "hbm", "alg_bytes_per_step": b_job, "achieved": b_job / (ms_step * 1e-3) / 1e9,
                    "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                    "frac": b_job / (ms_step * 1e-3) / 1e9 / (HBM_PEAK_GBS * world),
                    "model": "SURVEY §8(d) B_global = 1.25(|T|+|R|) + 0.25|R| + 4|R'| + 0.5|T| + |out| (|R'| taken as |R|)"}
        del nRp
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args.cpu_timeout)
        per = {n: {"mode": "global" if results[n][1]["mode_global"] else "local",
                   "rounds": results[n][1]["walk_rounds"], "matches": results[n][1]["n_matches"],
                   "record_bytes": int(results[n][0].numel())} for n in order}
        wl = ("hg19-vs-hg18 whole genome: 24 chromosome pairs at UCSC lengths (BASELINE configs[2])"
              if args.workload == "genome" else "hg19-vs-hg18 chr1-sized pair per GPU (BASELINE configs[1] shape)")
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "target bases/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong" if args.workload == "genome" else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (tools/synth.c hg profile, seed = chromosome index); real hg18/hg19 unavailable offline",
            "config": {"workload": wl, "chromosomes": len(jobs), "pairs_rank0": len(order),
                       "target_bases": job["target_bases"], "reference_bases": job["reference_bases"],
                       "k": 14, "m": 100, "params": "reference constants (compression.cpp:373-379), local controller on",
                       "contexts_per_gpu": n_lanes, "pair_queue": args.queue, "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                       "parallelism": f"LPT chromosome shard x{world}, RCCL gather of record streams to rank 0",
                       "record_bytes": job["record_bytes"]},
            "roofline": roof,
            "roofline_job": roof_job,
            "cpu_baseline": cpu,
            "parity": parity,
            "decompress": decomp,
            "end_to_end": e2e,
            "kernels": kernels,
            "per_chromosome_rank0": per,
        }
        print(json.dumps(line), flush=True)
    stop[0] = True
    go.wait()
    for t in lane_threads:
        t.join()
    for ln in lanes:
        ln.ctx.close()
    if world > 1:
        dist.destroy_process_group()


def load_pmc(kernel: str) -> dict | None:
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc summary of this bench."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    try:
        doc = json.load(open(path))
        v = doc.get(kernel, {}).get("hbm_bytes_per_launch")
        return {"hbm_bytes_per_launch": v, "source": doc.get("_source", path)} if v else None
    except Exception:
        return None


if __name__ == "__main__":
    main()
