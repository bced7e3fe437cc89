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
on the launching streams, SURVEY §8(d) algorithmic bytes) and of the whole job (DESIGN.md §4's
design model beside SURVEY §8(d)'s); the reference compression.cpp timed on this host on
BASELINE configs[0] (the chr21 pair); the chr1 record stream reconstructed on the GPU
(configs[3]); the T2T-like genome (configs[4]'s shape, 24 pairs at UCSC lengths); the whole
genome from FASTA files to record files (with and without the 7z step); per-chromosome sha256
checked against the reference's, pinned in tests/golden/genome_manifest.json.

The distributed pieces (timed_region, gather_streams, job_totals, check_pins) take the process
group from torch.distributed and are exercised with gloo on CPU by tests/test_bench_cpu.py.
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
DOMINANT = "walk"   # the step's dominant kernel family (k_walk: ~35 % of the kernel time)
CPU_BASELINE_N1 = os.path.join(REPO, "profiles", "cpu_baseline.json")   # the N = 1 line's measurement


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ------------------------------------------------------------------------------------------------
# algorithmic byte models
# ------------------------------------------------------------------------------------------------
def walk_alg_bytes(nT: int) -> float:
    """the walk's share of B_global, 0.5 B per target base (packed target + packed
    reference along the matches)."""
    return 0.5 * nT


def survey_alg_bytes(nT: int, nR: int, nRp: int, out: int) -> float:
    """SURVEY §8(d) B_global = 1.25(|T|+|R|) + 0.25|R| + 4|R'| + 0.5|T| + |out|.  Its 4|R'| term is
    a CSR k-mer position index, which this design never builds."""
    return 1.25 * (nT + nR) + 0.25 * nR + 4.0 * nRp + 0.5 * nT + out


def design_alg_bytes(tfa: int, rfa: int, nT: int, nR: int, nRp: int, out: int, mode_global: bool) -> float:
    """What this design must move at least, per pair: both FASTA texts read once
    and their stripped + N-erased copies written (ingest, compression.cpp:181-220, :523-557; the run
    lines' boundaries, :341-368 and :527-555, come out of the target's strip, so T is not read
    again for them), R' read once by the first-step sweep (the exact ungated first step, :64-161
    with pme == -1), the walk's 0.5 B per target base, and the record text written.
    The local pass (compression.cpp:372-481) is counted only for the segments of a pair that stays
    local (both segment strings once).  Round 6: a pair whose mode the switch probe decides writes
    only the N-erased copies T' and R' (the unfiltered T and R are read only by a local pass; the
    probe gathers its 128 segments of them from the FASTA), counted as |T| + |R'| (|T'| <= |T|)."""
    ingest = tfa + rfa + (nT + nRp if mode_global else 2.0 * (nT + nR))
    b = ingest + out
    if mode_global:
        b += nRp + walk_alg_bytes(nT)
    else:
        b += 2.0 * min(nT, nR)
    return b


def kernel_alg_bytes(kernel: str, tot: dict) -> float | None:
    """Algorithmic HBM bytes of one STEP of `kernel` summed over the step's pairs."""
    if kernel == "walk":
        return walk_alg_bytes(tot["target_bases"])
    if kernel == "fasta_strip":          # read the FASTA, write the N-erased copies (+ the stripped ones: local pairs)
        return tot["tgt_fa"] + tot["ref_fa"] + tot.get("strip_out_bytes", 2.0 * (tot["target_bases"] + tot["reference_bases"]))
    if kernel == "run_extract":          # the strip's per-tile run-event counts and flags (12 B per 4 KiB
        return 12.0 * tot["target_bases"] / 4096.0   # tile; the events themselves are a few bytes per run)
    if kernel == "first_sweep_anchors":  # R' once + one 8-byte anchor slot per 64 reference bases
        return tot["walk_reference_bases"] * (1.0 + 8.0 / 64.0)
    if kernel == "local_segments":       # both segment strings (up to the switch, bounded by all of them)
        return 2.0 * min(tot["target_bases"], tot["reference_bases"])
    return None


def load_manifest() -> dict:
    try:
        return {e["name"]: e for e in json.load(open(MANIFEST))}
    except Exception:
        return {}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ------------------------------------------------------------------------------------------------
# distributed pieces (RCCL on the GPU box, gloo in tests/test_bench_cpu.py)
# ------------------------------------------------------------------------------------------------
def timed_region(step, steps: int, warmup: int, world: int, sync=lambda: None, device=None) -> float:
    """W untimed steps, then exactly K steps between a barrier + device sync on both sides; the
    MAX over ranks of the elapsed time (the job ends with its slowest rank)."""
    import torch
    import torch.distributed as dist
    for _ in range(warmup):
        step()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def make_step(pool, order: list, job, results: dict, gather=None):
    """One step: every pair of this rank's shard compressed on its lanes (pool.run), then -- N > 1 --
    the per-chromosome record streams queued to rank 0 (multigpu.StreamGather: point-to-point,
    unpadded, behind the lanes' streams).  The step reads nothing back from the device and never
    waits for it; timed_region's final device sync is the only synchronisation.  The gather's plan
    (the stream lengths, an all_gather_object) is made in the first, untimed call."""

    def step() -> None:
        pool.run(order, job)
        if gather is not None:
            parts = {n: results[n][0] for n in order}
            if gather.plan_lengths is None:
                pool.sync()
                gather.plan(parts, parts[order[0]].device if order else None)
            gather.step(parts, after=[ln.stream for ln in pool.lanes])
    return step


def gather_streams(results: dict, order: list, world: int, device) -> dict | None:
    """Every rank's per-chromosome record streams on rank 0 (multigpu.gather_records: one size
    all-gather + one gather to rank 0); None on the other ranks."""
    import multigpu
    if world <= 1:
        return {n: results[n][0].cpu().numpy().tobytes() for n in order}
    return multigpu.gather_records({n: results[n][0] for n in order}, device=device)


def job_totals(tot: dict, world: int) -> tuple[dict, list]:
    """Per-rank totals summed over the ranks (all_gather_object), and the per-rank list."""
    import torch.distributed as dist
    totals = [tot]
    if world > 1:
        got = [None] * world
        dist.all_gather_object(got, tot)
        totals = got
    return {k: sum(t[k] for t in totals) for k in tot}, totals


def check_pins(streams: dict | None, pins: dict) -> dict | None:
    """sha256 of each gathered record stream against the reference's pinned one (rank 0)."""
    if streams is None:
        return None
    checked = [n for n in streams if n in pins]
    bad = [n for n in checked if hashlib.sha256(streams[n]).hexdigest() != pins[n]["record_sha256"]]
    return {"chromosomes": len(streams), "pinned_checked": len(checked), "pinned_mismatch": bad,
            "reference": "oracle/_ref (compression.cpp compiled unchanged), tests/golden/genome_manifest.json"}


def cpu_baseline_pointer() -> dict | None:
    """N > 1 lines: the CPU baseline is measured by the N = 1 run only (rank 0, bounded sample);
    repeat its committed value with a pointer to it."""
    try:
        doc = json.load(open(CPU_BASELINE_N1))
    except Exception:
        return None
    out = dict(doc)
    out["measured_in"] = os.path.relpath(CPU_BASELINE_N1, REPO) + " (the N = 1 bench line; not re-run at N > 1)"
    return out


def box_cpu_share() -> int:
    """Host cores this process may use: its affinity mask, capped at the GPU box's share per GPU
    (16; the box's os.cpu_count() is the whole machine's)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(n, 16))


def cpu_genome_estimate(box_chr21_wall_s: float | None = None, cores: int | None = None) -> dict | None:
    """The whole hg19-vs-hg18 genome on THIS host's cores, from the reference's own walls: the 24
    per-pair walls in the manifest (compiled reference, measured once by tests/golden/pin_genome.py
    in the build container) give the pairs' relative costs; they are scaled to this host by its own
    chr21 wall measured in this run (cpu_baseline, the same compiled reference on the same pair) over
    the manifest's chr21 wall.  Makespan = LPT of the scaled walls over P = this host's core share.
    Without this run's chr21 wall nothing is estimated (no field mixes two machines)."""
    import multigpu
    pins = load_manifest()
    walls = [pins[n]["reference_wall_s"] for n in multigpu.CHROMS if n in pins and "reference_wall_s" in pins[n]]
    c21 = pins.get("chr21", {}).get("reference_wall_s")
    if len(walls) < len(multigpu.CHROMS) or not c21 or not box_chr21_wall_s:
        return None
    scale = box_chr21_wall_s / c21
    walls = [w * scale for w in walls]
    nT = sum(multigpu.HG19)
    P = cores or box_cpu_share()
    loads = [sum(walls[i] for i in part) for part in multigpu.lpt_shard(walls, P)]
    return {"cpu_seconds": round(sum(walls), 1), "target_bases": nT, "bases_per_s_one_core": nT / sum(walls),
            "cores": P, "lpt_makespan_s": round(max(loads), 1), "bases_per_s_on_P_cores": nT / max(loads),
            "host": {"cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(), "core_share": box_cpu_share()},
            "scale_from_chr21": round(scale, 4),
            "note": f"compiled reference (oracle/_ref, g++ -O2, stub 7z) on this host: its chr21 wall in this run "
                    f"({box_chr21_wall_s:.1f} s) x the 24 pairs' relative walls from tests/golden/genome_manifest.json "
                    f"(one machine's ratios, chr21 there {c21:.1f} s); makespan = LPT over P cores of this host, "
                    f"RAM permitting (chr1 alone needs 17.4 GB)"}


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
    return {"value": tl / dt, "unit": "target bases/s", "cores": 1, "kind": kind, "wall_s": dt,
            "sample": f"BASELINE configs[0]: hg19-vs-hg18 chr21-sized synthetic pair |R|={rl:,} |T|={tl:,} (seed 21), "
                      f"wall {dt:.1f} s, single-threaded ({cpu_model()}), stub 7z, stdout to /dev/null",
            "record_matches_pinned": (sha == pin) if pin else None}


def chr1_k21(lane: Lane, pair: tuple, tfa: bytes, dev, reps: int = 5) -> dict:
    """BASELINE configs[1] as written: the chr1 pair with k = 21 (a non-parity override -- the
    reference hard-codes k = 14, compression.cpp:373 -- so the global walk runs with local = 0),
    HBM-resident inputs, one lane; the record stream is reconstructed on the GPU and compared with
    the target FASTA byte for byte."""
    import torch
    dr, rn, dt_, tn = pair
    ctx, s = lane.ctx, lane.stream

    def once():
        return ctx.compress_device(dr.data_ptr(), rn, dt_.data_ptr(), tn, lane.out.data_ptr(), lane.cap, s.cuda_stream,
                                   k=21, local=0)
    once()
    s.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        n = once()
        s.synchronize()
        ts.append(time.perf_counter() - t0)
    st = ctx.stats()
    rec = lane.out[:n].clone()
    need = ctx.reconstruct_device(dr.data_ptr(), rn, rec.data_ptr(), n, 0, 0, s.cuda_stream)
    d_fa = torch.empty(need + 64, dtype=torch.uint8, device=dev)
    n_fa = ctx.reconstruct_device(dr.data_ptr(), rn, rec.data_ptr(), n, d_fa.data_ptr(), need + 64, s.cuda_stream)
    s.synchronize()
    exact = d_fa[:n_fa].cpu().numpy().tobytes() == tfa
    dt = sorted(ts)[len(ts) // 2]
    return {"workload": "BASELINE configs[1]: hg19-vs-hg18 chr1-sized pair, k = 21 (non-parity override, local = 0), "
                        "1 GPU, one lane", "k": 21, "target_bases": st["target_bases"], "ms": dt * 1e3,
            "ms_all": [round(t * 1e3, 3) for t in ts], "bases_per_s": st["target_bases"] / dt,
            "walk_rounds": st["walk_rounds"], "matches": st["n_matches"], "record_bytes": n,
            "record_sha256": hashlib.sha256(rec.cpu().numpy().tobytes()).hexdigest(), "roundtrip_exact": exact}


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


class LanePool:
    """Persistent lane threads: run(job) hands every lane the same pair queue (largest first onto
    the first free lane) through one barrier and joins them at another (no thread start per step).
    job(lane, name) does one pair on that lane."""

    def __init__(self, lanes: list, dev):
        import torch
        self.lanes, self.dev = lanes, dev
        self.go = threading.Barrier(len(lanes) + 1)
        self.done = threading.Barrier(len(lanes) + 1)
        self.lock = threading.Lock()
        self.queue: list = []
        self.job = None
        self.errors: list = []
        self.stop = False

        def worker(lane):
            torch.cuda.set_device(dev)
            while True:
                self.go.wait()
                if self.stop:
                    return
                try:
                    while True:
                        with self.lock:
                            if not self.queue:
                                break
                            name = self.queue.pop(0)
                        self.job(lane, name)
                except Exception as e:   # noqa: BLE001 -- reported after the step
                    self.errors.append(e)
                self.done.wait()

        self.threads = [threading.Thread(target=worker, args=(ln,), daemon=True) for ln in lanes]
        for t in self.threads:
            t.start()

    def run(self, order: list, job) -> None:
        self.queue = list(order)
        self.job = job
        self.go.wait()
        self.done.wait()
        if self.errors:
            raise self.errors[0]

    def sync(self) -> None:
        for ln in self.lanes:
            ln.stream.synchronize()

    def close(self) -> None:
        self.stop = True
        self.go.wait()
        for t in self.threads:
            t.join()


def gen_pairs(jobs: list, profile: str, dev, keep_host: set) -> tuple[dict, dict, int, int]:
    """Synthetic pairs (threads: the C generator releases the GIL), uploaded to HBM.  Returns
    {name: (d_ref, |ref FASTA|, d_tgt, |tgt FASTA|)}, the host FASTA of the names in keep_host, and
    the FASTA byte totals."""
    import torch
    import synth
    host, lock = {}, threading.Lock()

    def gen(job):
        name, rl, tl, seed = job
        rfa, tfa = synth.synth_pair(profile, rl, tl, seed)
        with lock:
            host[name] = (rfa, tfa)

    ths = [threading.Thread(target=gen, args=(j,)) for j in jobs]
    for b in range(0, len(ths), 8):
        for t in ths[b:b + 8]:
            t.start()
        for t in ths[b:b + 8]:
            t.join()
    pairs = {}
    for name, _, _, _ in jobs:
        rfa, tfa = host[name]
        pairs[name] = (torch.frombuffer(bytearray(rfa), dtype=torch.uint8).to(dev), len(rfa),
                       torch.frombuffer(bytearray(tfa), dtype=torch.uint8).to(dev), len(tfa))
    rb = sum(len(v[0]) for v in host.values())
    tb = sum(len(v[1]) for v in host.values())
    kept = {n: host[n] for n in keep_host if n in host}
    host.clear()
    return pairs, kept, rb, tb


def device_job(pairs: dict, results: dict, dev):
    """The pair job of a step: compress the HBM-resident pair on the lane and keep its record text."""
    import torch

    def job(lane, name):
        dr, rn, dt_, tn = pairs[name]
        n = lane.ctx.compress_device(dr.data_ptr(), rn, dt_.data_ptr(), tn, lane.out.data_ptr(), lane.cap,
                                     lane.stream.cuda_stream)
        st = lane.ctx.stats()
        prev = results.get(name)
        with torch.cuda.stream(lane.stream):
            buf = prev[0] if prev is not None and prev[0].numel() == n else torch.empty(n, dtype=torch.uint8, device=dev)
            buf.copy_(lane.out[:n])   # the pair's record stream, kept for the gather (the step syncs)
        results[name] = (buf, st)
    return job


def standalone_costs(lane: Lane, pairs: dict, order: list) -> dict:
    """Each pair alone on one lane, one after the other (an untimed pass after the timed steps): its
    compress call's wall time in ms, device-resident inputs -- the per-pair cost a multi-GPU shard
    plan needs (a T2T-like pair's cost is not proportional to its length)."""
    import torch
    out = {}
    if order:   # (the lane's buffers sized for the largest pair first: a pair this lane never took in
        dr, rn, dt_, tn = pairs[order[0]]   # the steps would otherwise pay its reallocations here)
        lane.ctx.compress_device(dr.data_ptr(), rn, dt_.data_ptr(), tn, lane.out.data_ptr(), lane.cap,
                                 lane.stream.cuda_stream)
        lane.stream.synchronize()
    for n in order:
        dr, rn, dt_, tn = pairs[n]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lane.ctx.compress_device(dr.data_ptr(), rn, dt_.data_ptr(), tn, lane.out.data_ptr(), lane.cap,
                                 lane.stream.cuda_stream)
        lane.stream.synchronize()
        out[n] = round((time.perf_counter() - t0) * 1e3, 3)
    return out


def predicted_makespans(cost: dict, sizes: dict, step_ms: float, worlds=(1, 2, 4, 8)) -> dict:
    """The N-GPU job time predicted from one GPU's measurements: per-pair standalone costs, LPT-sharded
    over N GPUs (by measured cost, and by target size as bench.py / genome.py shard by default), each
    GPU's load divided by the overlap its lanes gain on one GPU (sum of standalone costs / measured
    step), and never below the costliest single pair (a pair is one GPU's work unless its walk is
    split, multigpu.split_walk)."""
    import multigpu
    names = sorted(cost)
    gain = sum(cost.values()) / step_ms if step_ms > 0 else 1.0
    out = {"lane_overlap_gain": round(gain, 3), "costliest_pair": max(names, key=lambda n: cost[n]),
           "costliest_pair_ms": max(cost.values())}
    for key, w8 in (("lpt_by_cost", [cost[n] for n in names]), ("lpt_by_size", [sizes[n] for n in names])):
        e = {}
        for w in worlds:
            loads = [sum(cost[names[i]] for i in part) for part in multigpu.lpt_shard(w8, w)]
            e[str(w)] = round(max(max(loads) / gain, max(cost.values())), 3)
        out[key + "_ms"] = e
    return out


def t2t_genome(pool: LanePool, jobs: list, world: int, rank: int, dev, steps: int) -> dict:
    """BASELINE configs[4]'s shape: the same 24 UCSC length pairs with the T2T-like profile (the
    stuck, literal-heavy walk of compression.cpp:83-101), each rank its LPT shard; one warm pass,
    then `steps` timed passes (max over ranks); record sha256 against the reference's pins
    (t2t_<chrom> in tests/golden/genome_manifest.json, tests/golden/pin_genome.py)."""
    import torch
    import multigpu
    import torch.distributed as dist
    t0 = time.perf_counter()
    tj = [(f"t2t_{n}", rl, tl, seed) for n, rl, tl, seed in jobs]
    pairs, _, _, _ = gen_pairs(tj, "t2t", dev, set())
    gen_s = time.perf_counter() - t0
    order = sorted(pairs, key=lambda n: -pairs[n][3])
    results: dict = {}
    job = device_job(pairs, results, dev)
    rounds_per_step: list = []
    if order:   # every lane sized for the largest pair before the timed passes (see main)
        dr, rn, dt_, tn = pairs[order[0]]
        for ln in pool.lanes:
            ln.ctx.compress_device(dr.data_ptr(), rn, dt_.data_ptr(), tn, ln.out.data_ptr(), ln.cap, ln.stream.cuda_stream)
            ln.stream.synchronize()

    def step():
        pool.run(order, job)
        pool.sync()
        rounds_per_step.append({n: results[n][1]["walk_rounds"] for n in order})

    dt = timed_region(step, steps, 1, world, torch.cuda.synchronize, dev)
    timed_rounds = rounds_per_step[1:]   # (the warm pass first)
    cost = standalone_costs(pool.lanes[0], pairs, order)
    shas = {n: hashlib.sha256(results[n][0].cpu().numpy().tobytes()).hexdigest() for n in order}
    per = {n: {"rounds": results[n][1]["walk_rounds"], "rounds_per_timed_step": [r[n] for r in timed_rounds],
               "chains": results[n][1]["walk_chains"], "matches": results[n][1]["n_matches"],
               "mode": "global" if results[n][1]["mode_global"] else "local", "ms_alone": cost[n],
               "switch_segment": results[n][1]["switch_segment"], "target_bases": results[n][1]["target_bases"]}
           for n in order}
    nT = sum(results[n][1]["target_bases"] for n in order)
    if world > 1:
        got = [None] * world
        dist.all_gather_object(got, (shas, per, nT))
        shas, per, nT = {}, {}, 0
        for s_, p_, n_ in got:
            shas.update(s_)
            per.update(p_)
            nT += n_
    del pairs, results
    torch.cuda.empty_cache()
    pins = load_manifest()
    checked = [n for n in shas if n in pins]
    bad = [n for n in checked if shas[n] != pins[n]["record_sha256"]]
    ms = dt / steps * 1e3
    worst = max(per, key=lambda n: per[n]["rounds"]) if per else None
    stable = all(len(set(p["rounds_per_timed_step"])) <= 1 for p in per.values())
    return {"workload": "BASELINE configs[4] shape, synthetic: T2T-like profile (tandem arrays, 1e-2 SNPs, >100-bp "
                        "deletions every ~100 kb) at the hg18/hg19 chromosome lengths (not CHM13/GRCh38 lengths: no "
                        "T2T data offline), 24 pairs, seed = chromosome index",
            "target_bases": nT, "ms": ms, "bases_per_s": nT / (ms * 1e-3), "steps": steps, "contexts": len(pool.lanes),
            "pinned_checked": len(checked), "pinned_mismatch": bad,
            "max_rounds": per[worst]["rounds"] if worst else None, "max_rounds_chrom": worst,
            "rounds_same_every_timed_step": stable,
            "generate_s": round(gen_s, 1), "per_chromosome": per,
            "lpt_max_over_mean_8gpu": multigpu.max_over_mean([j[2] for j in jobs], 8),
            "predicted": predicted_makespans({n: per[n]["ms_alone"] for n in per},
                                             {n: per[n]["target_bases"] for n in per}, ms) if world == 1 else None}


def end_to_end_genome(pool: LanePool, host_fa: dict, order: list, pins: dict, reps: int = 2) -> dict:
    """The whole genome from FASTA files to record files (compression.cpp:181-331 per pair, 7z
    excluded), every pair through sccg_compress_files on the lanes (two contexts: one pair's file
    reads and PCIe copies overlap another's kernels), files in the page cache; then once more with
    the reference's `7z a -mx=9` per pair started as soon as that pair's file is closed (genome.py's
    Emitter overlap, compression.cpp:306-318), if 7z is installed on this host."""
    import genome
    d = tempfile.mkdtemp(prefix="sccg_e2eg_")
    try:
        fa_bytes = 0
        for n in order:
            rfa, tfa = host_fa[n]
            os.makedirs(os.path.join(d, "ref"), exist_ok=True)
            os.makedirs(os.path.join(d, "tgt"), exist_ok=True)
            open(os.path.join(d, "ref", n + ".fa"), "wb").write(rfa)
            open(os.path.join(d, "tgt", n + ".fa"), "wb").write(tfa)
            fa_bytes += len(rfa) + len(tfa)
        out = os.path.join(d, "out")
        stats: dict = {}

        def job_with(em):
            def job(lane, name):
                st = genome.compress_pair_files(lane.ctx, os.path.join(d, "ref", name + ".fa"),
                                                os.path.join(d, "tgt", name + ".fa"), out, name, em)
                stats[name] = st
            return job

        pool.run(order, job_with(None))   # warm (staging buffers)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            pool.run(order, job_with(None))
            ts.append(time.perf_counter() - t0)
        bad = [n for n in order if n in pins and hashlib.sha256(
            open(os.path.join(out, n, "compressed_genome.txt"), "rb").read()).hexdigest() != pins[n]["record_sha256"]]
        nT = sum(stats[n]["target_bases"] for n in order)
        res = {"workload": "24 hg19-vs-hg18 pairs: FASTA files (page cache) -> <out>/<chrom>/compressed_genome.txt "
                           "closed, 7z excluded (sccg_compress_files, 2 contexts)",
               "target_bases": nT, "fasta_bytes": fa_bytes, "ms": min(ts) * 1e3, "ms_all": [round(t * 1e3, 1) for t in ts],
               "bases_per_s": nT / min(ts), "host_to_file_GBps": fa_bytes / min(ts) / 1e9,
               "pinned_checked": len([n for n in order if n in pins]), "pinned_mismatch": bad}
        sz = shutil.which("7z")
        if sz:
            em = genome.Emitter(out, True, sz)
            t0 = time.perf_counter()
            pool.run(order, job_with(em))
            t_gpu = time.perf_counter() - t0
            rc = em.wait()
            t_all = time.perf_counter() - t0
            res["with_7z"] = {"ms": t_all * 1e3, "gpu_part_ms": t_gpu * 1e3, "bases_per_s": nT / t_all, "rc": rc,
                              "7z": sz, "archive_bytes": sum(os.path.getsize(os.path.join(out, n, "compressed_genome.txt.7z"))
                                                            for n in order if os.path.exists(os.path.join(out, n, "compressed_genome.txt.7z")))}
        else:
            res["with_7z"] = "7z is not installed on this host (no package index: it cannot be added); the 7z step "\
                             "is the reference's `7z a -mx=9` and runs unchanged where 7z exists (genome.py Emitter)"
        return res
    finally:
        shutil.rmtree(d, ignore_errors=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--contexts", type=int, default=2, help="library contexts (host threads) per GPU")
    ap.add_argument("--workload", choices=["genome", "chr1"], default="genome",
                    help="genome: BASELINE configs[2] (default); chr1: one chr1-sized pair per rank (configs[1] shape)")
    ap.add_argument("--names", default="", help="comma-separated subset of chromosomes (diagnostics)")
    ap.add_argument("--cpu-timeout", type=int, default=300)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the pinned sha256 checks")
    ap.add_argument("--no-decomp", action="store_true", help="skip the configs[3] reconstruction")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (files) measurements")
    ap.add_argument("--no-t2t", action="store_true", help="skip the T2T-like genome (configs[4] shape)")
    ap.add_argument("--t2t-steps", type=int, default=2)
    ap.add_argument("--t2t-contexts", type=int, default=4,
                    help="library contexts for the T2T-like leg (its pairs are round-latency-bound: 2 / 3 / 4 / 6 "
                         "contexts measured 318 / 289 / 235 / 238 ms, the hg genome unchanged, profiles/r06/ab/r06y)")
    ap.add_argument("--no-prof", action="store_true", help="no per-kernel HIP events in the timed region")
    ap.add_argument("--no-k21", action="store_true", help="skip the configs[1] leg (chr1 at k = 21)")
    ap.add_argument("--only-steps", action="store_true",
                    help="the timed steps and the line only (traces): no per-pair costs, decompress, k=21, e2e, T2T")
    args = ap.parse_args()
    if args.only_steps:
        args.no_decomp = args.no_e2e = args.no_t2t = args.no_k21 = args.no_prof = args.no_cpu_baseline = True

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

    # ---- inputs: generated on the host, then resident in HBM
    t0 = time.perf_counter()
    want_e2e_genome = args.workload == "genome" and not args.no_e2e
    keep = {n for n, _, _, _ in mine} if want_e2e_genome else {"chr1", f"chr1_r{rank}"}
    pairs, host_fa, ref_fa_bytes, tgt_fa_bytes = gen_pairs(mine, "hg", dev, keep)
    keep_chr1 = host_fa.get("chr1") or host_fa.get(f"chr1_r{rank}")
    torch.cuda.synchronize()
    log(f"[rank {rank}] {len(mine)} pairs generated and resident in {time.perf_counter() - t0:.1f} s "
        f"({ref_fa_bytes + tgt_fa_bytes:,} FASTA bytes)")

    n_lanes = max(1, min(args.contexts, len(mine)))
    cap = max(sccg.Context.compress_bound_static(p[1], p[3]) for p in pairs.values())
    lanes = [Lane(sccg, torch, dev, cap, local) for _ in range(n_lanes)]
    pool = LanePool(lanes, dev)
    order = sorted(pairs, key=lambda n: -pairs[n][3])   # largest first onto the first free lane
    results: dict = {}      # name -> (device tensor of its record text, stats)
    job = device_job(pairs, results, dev)
    gather = multigpu.StreamGather() if world > 1 else None
    step = make_step(pool, order, job, results, gather)
    # every lane sized for the largest pair once, before any step: the lanes take pairs from a shared
    # queue, and a lane meeting a larger pair than before in a timed step would grow its buffers there
    # (hipMalloc, the anchor table's first clear)
    if order:
        dr, rn, dt_, tn = pairs[order[0]]
        for ln in lanes:
            ln.ctx.compress_device(dr.data_ptr(), rn, dt_.data_ptr(), tn, ln.out.data_ptr(), ln.cap, ln.stream.cuda_stream)
            ln.stream.synchronize()

    for _ in range(max(args.warmup, 1 if world > 1 else 0)):   # (N > 1: the gather's plan is made here)
        step()
    # HIP events inside the timed region bracket the dominant kernel's launches only (k_walk; events
    # around every family cost ~1 ms of a ~23 ms step); one more, untimed step brackets every family
    # for the per-kernel table and the other kernels' rooflines
    lanes[0].ctx.profile(not args.no_prof, families=[DOMINANT])
    dt = timed_region(step, args.steps, 0, world, torch.cuda.synchronize, dev)
    prof_dom = lanes[0].ctx.profile_get()
    lanes[0].ctx.profile(False)
    prof_all = {}
    if not args.no_prof:
        lanes[0].ctx.profile(True)
        step()
        torch.cuda.synchronize()
        prof_all = lanes[0].ctx.profile_get()
        lanes[0].ctx.profile(False)

    # ---- per-pair standalone costs (untimed) and the N-GPU makespans they predict (N = 1 lines)
    hg_cost = standalone_costs(lanes[0], pairs, order) if world == 1 and not args.only_steps else {}
    hg_sizes = {n: pairs[n][3] for n in hg_cost}   # (the pairs leave HBM before the T2T-like leg)

    # ---- per-rank totals (all ranks' target bases make up the whole job)
    tot = {"target_bases": sum(results[n][1]["target_bases"] for n in order),
           "reference_bases": sum(results[n][1]["reference_bases"] for n in order),
           "walk_reference_bases": sum(results[n][1]["walk_reference_bases"] for n in order),
           "record_bytes": sum(int(results[n][0].numel()) for n in order),
           "tgt_fa": tgt_fa_bytes, "ref_fa": ref_fa_bytes,
           "strip_out_bytes": sum((results[n][1]["target_bases"] + results[n][1]["walk_reference_bases"])
                                  if results[n][1]["mode_global"] else
                                  2 * (results[n][1]["target_bases"] + results[n][1]["reference_bases"]) for n in order),
           "design_bytes": sum(design_alg_bytes(pairs[n][3], pairs[n][1], results[n][1]["target_bases"],
                                                results[n][1]["reference_bases"], results[n][1]["walk_reference_bases"],
                                                int(results[n][0].numel()), bool(results[n][1]["mode_global"]))
                               for n in order),
           "survey_bytes": sum(survey_alg_bytes(results[n][1]["target_bases"], results[n][1]["reference_bases"],
                                                results[n][1]["walk_reference_bases"], int(results[n][0].numel()))
                               for n in order)}
    job_tot, _ = job_totals(tot, world)

    # ---- parity: every chromosome's record stream against the reference's pinned sha256
    parity = None
    if not args.no_check:
        torch.cuda.synchronize()
        if world > 1:
            got = gather.result()
            streams = {n: t.cpu().numpy().tobytes() for n, t in got.items()} if got is not None else None
        else:
            streams = gather_streams(results, order, 1, dev)
        if rank == 0:
            pins = load_manifest() if args.workload == "genome" else {}
            parity = check_pins(streams, pins)
            if args.workload == "chr1":
                parity["record_sha256"] = hashlib.sha256(next(iter(streams.values()))).hexdigest()
            if parity["pinned_mismatch"]:
                raise SystemExit(f"bench: record streams differ from the reference for {parity['pinned_mismatch']}")

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
        ks = max(20, args.steps)   # (a 0.7 ms call: 20 back to back, after 3 warm-up calls)
        for _ in range(3):
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
                                   "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": b_dec / ddt / 1e9 / HBM_PEAK_GBS,
                                   "model": "SURVEY §8(d) B_decomp = |rec| + |R| + |T_fa| + |T_matched|"},
                  "kernels": {k: {"ms_per_call": v[0] / ks, "launches_per_call": v[1] / ks} for k, v in dprof.items()}}
        del d_fa
        if not exact:
            raise SystemExit("bench: chr1 reconstruction differs from the target FASTA")

    # ---- configs[1] as named: chr1 at k = 21 through the global walk (non-parity: the reference
    #      hard-codes k = 14, compression.cpp:373; local = 0), round trip checked on the GPU
    k21 = None
    if rank == 0 and not args.no_k21 and keep_chr1 is not None:
        name = "chr1" if "chr1" in pairs else f"chr1_r{rank}"
        k21 = chr1_k21(lanes[0], pairs[name], keep_chr1[1], dev)
        if not k21["roundtrip_exact"]:
            raise SystemExit("bench: chr1 k=21 record stream does not reconstruct the target FASTA")

    e2e = None
    if rank == 0 and not args.no_e2e and keep_chr1 is not None:
        pin = load_manifest().get("chr1", {}).get("record_sha256") if args.workload == "genome" else None
        e2e = end_to_end(lanes[0].ctx, keep_chr1[0], keep_chr1[1], pin)
    e2e_genome = None
    if want_e2e_genome and world == 1 and not args.names:
        e2e_genome = end_to_end_genome(pool, host_fa, order, load_manifest() if not args.no_check else {})
    host_fa.clear()

    t2t = None
    if args.workload == "genome" and not args.no_t2t and not args.names:
        # the hg pairs' HBM is not needed any more
        for n in list(pairs):
            del pairs[n]
        torch.cuda.empty_cache()
        # more lanes than the hg genome's: a T2T-like pair spends its time in short walk rounds with
        # a host readback each, which other pairs' rounds fill
        t2t_pool = pool
        if args.t2t_contexts > len(lanes):
            pool.close()
            lanes += [Lane(sccg, torch, dev, cap, local) for _ in range(args.t2t_contexts - len(lanes))]
            t2t_pool = pool = LanePool(lanes, dev)
        t2t = t2t_genome(t2t_pool, jobs, world, rank, dev, max(1, args.t2t_steps))
        if rank == 0 and t2t["pinned_mismatch"]:
            raise SystemExit(f"bench: T2T-like record streams differ from the reference for {t2t['pinned_mismatch']}")

    if rank == 0:
        value = job_tot["target_bases"] * args.steps / dt
        ms_step = dt * 1e3 / args.steps
        # (one untimed step with every family bracketed)
        kernels = {k: {"ms_per_step": v[0], "launches_per_step": v[1], "avg_launch_ms": v[0] / v[1]}
                   for k, v in prof_all.items()}
        if prof_all and max(prof_all, key=lambda k: prof_all[k][0]) != DOMINANT:
            log(f"bench: {max(prof_all, key=lambda k: prof_all[k][0])} took more kernel time than {DOMINANT}")
        prof = prof_dom
        roof = None
        if prof:
            dom = DOMINANT
            alg_step = kernel_alg_bytes(dom, tot)
            if alg_step is not None and dom in prof:
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
        # other kernels' achieved rates against the same models (HIP events) and their PMC bytes
        kroof = {}
        for k in ("fasta_strip", "first_sweep_anchors", "run_extract"):
            if k in prof_all and prof_all[k][1]:
                ab = kernel_alg_bytes(k, tot) / prof_all[k][1]
                am = prof_all[k][0] / prof_all[k][1]
                e = {"alg_bytes_per_launch": ab, "avg_launch_ms": am, "achieved_GBps": ab / (am * 1e-3) / 1e9,
                     "frac": ab / (am * 1e-3) / 1e9 / HBM_PEAK_GBS}
                pmc = load_pmc(k) or load_pmc({"first_sweep_anchors": "k_sweep_early"}.get(k, k))   # (family, or round-4 kernel name)
                if pmc:
                    e["traffic_per_launch"] = pmc["hbm_bytes_per_launch"]
                kroof[k] = e
        per_s = ms_step * 1e-3
        roof_job = {"bound": "hbm", "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                    "alg_bytes_per_step": job_tot["design_bytes"],
                    "achieved": job_tot["design_bytes"] / per_s / 1e9,
                    "frac": job_tot["design_bytes"] / per_s / 1e9 / (HBM_PEAK_GBS * world),
                    "model": "design (DESIGN.md §4, bench.design_alg_bytes): per pair both FASTA read + T', R' (+ T, R for a local pair) "
                             "written once (ingest; run lines from the target strip) + R' once (first-step sweep) + 0.5 B per "
                             "target base (walk, SURVEY §8(d)) + the record text; a pair that stays local: its segments "
                             "once instead of the sweep and walk.  |R'| measured per pair.",
                    "survey_model": {"alg_bytes_per_step": job_tot["survey_bytes"],
                                     "frac": job_tot["survey_bytes"] / per_s / 1e9 / (HBM_PEAK_GBS * world),
                                     "model": "SURVEY §8(d) B_global = 1.25(|T|+|R|) + 0.25|R| + 4|R'| + 0.5|T| + |out| "
                                              "with measured |R'|; its 4|R'| CSR index is not built by this design"}}
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_timeout)
        else:
            cpu = cpu_baseline_pointer()
        per = {n: {"mode": "global" if results[n][1]["mode_global"] else "local",
                   "rounds": results[n][1]["walk_rounds"], "matches": results[n][1]["n_matches"],
                   "switch_segment": results[n][1]["switch_segment"],
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
                       "target_bases": job_tot["target_bases"], "reference_bases": job_tot["reference_bases"],
                       "k": 14, "m": 100, "params": "reference constants (compression.cpp:373-379), local controller on",
                       "contexts_per_gpu": n_lanes, "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                       "parallelism": f"LPT chromosome shard x{world}, RCCL gather of record streams to rank 0",
                       "record_bytes": job_tot["record_bytes"]},
            "roofline": roof,
            "roofline_kernels": kroof,
            "roofline_job": roof_job,
            "cpu_baseline": cpu,
            "cpu_genome_estimate": cpu_genome_estimate(cpu.get("wall_s") if cpu and world == 1 else None),
            "parity": parity,
            "decompress": decomp,
            "end_to_end": e2e,
            "end_to_end_genome": e2e_genome,
            "t2t_genome": t2t,
            "chr1_k21": k21,
            "predicted_multi_gpu": {"hg_genome": predicted_makespans(hg_cost, hg_sizes, ms_step)
                                    if hg_cost else None,
                                    "t2t_genome": (t2t or {}).get("predicted"),
                                    "model": "bench.predicted_makespans: per-pair standalone ms, LPT over N GPUs, "
                                             "loads / the lanes' overlap gain on one GPU, floor = costliest pair"},
            "hip_runtime": sccg.hip_runtimes(),
            "kernels": kernels,
            "per_chromosome_rank0": per,
        }
        print(json.dumps(line), flush=True)
    pool.close()
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
        return {"hbm_bytes_per_launch": v, "source": doc.get("_source", "profiles/pmc_summary.json")} if v else None
    except Exception:
        return None


if __name__ == "__main__":
    main()
