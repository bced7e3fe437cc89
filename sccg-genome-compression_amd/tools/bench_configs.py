#!/usr/bin/env python3
"""Secondary measurements (not the bench.py line): device-resident throughput of
  * the whole hg19-vs-hg18 genome on ONE GPU (BASELINE configs[2]: 24 chromosome pairs at their
    UCSC lengths, synthetic, compressed one after another; the 8-GPU job LPT-shards them),
  * decompression of a chr1-sized record stream (BASELINE configs[3]),
  * compression of a T2T-like divergent pair (configs[4] shape, literal-heavy),
  * compression of a pair that stays in local mode (no switch),
  * the chr1-sized pair through the parameter overrides (sccg_params, non-parity): the global walk
    at BASELINE configs[1]'s k = 21 and at the reference's k = 14, without the local controller.

    python bench_configs.py [--scale 1.0] [--steps 3]
Prints one JSON object per workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--only", default="")
    ap.add_argument("--contexts", type=int, default=1,
                    help="genome: contexts (host threads) per GPU compressing chromosomes concurrently")
    ap.add_argument("--genome-profile", default="hg", choices=["hg", "t2t"],
                    help="genome: synthetic profile of the 24 pairs (t2t = BASELINE configs[4]'s shape at UCSC lengths)")
    ap.add_argument("--roundtrip", action="store_true",
                    help="genome: reconstruct every pair on the GPU and compare it with its target FASTA")
    args = ap.parse_args()
    import torch
    import sccg
    import synth

    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ctx = sccg.Context(0)

    def to_dev(b: bytes) -> torch.Tensor:
        return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            r = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps, r

    work = [("chr1_decompress", "hg", 247_249_719, 249_250_621, 1, {}),
            ("t2t_like_compress", "t2t", 100_000_000, 100_000_000, 7, {}),
            ("local_mode_compress", "local", 247_249_719, 247_249_719, 8, {}),
            ("chr1_k21_global_compress", "hg", 247_249_719, 249_250_621, 1, {"k": 21, "local": 0}),
            ("chr1_k14_global_compress", "hg", 247_249_719, 249_250_621, 1, {"local": 0})]
    if not args.only or args.only in "genome":
        genome(ctx, dev, stream, args, to_dev)
    for name, prof, rl, tl, seed, over in work:
        if args.only and args.only not in name:
            continue
        rl, tl = int(rl * args.scale), int(tl * args.scale)
        rfa, tfa = synth.synth_pair(prof, rl, tl, seed)
        d_ref, d_tgt = to_dev(rfa), to_dev(tfa)
        cap = ctx.compress_bound(len(rfa), len(tfa))
        d_rec = torch.empty(cap, dtype=torch.uint8, device=dev)
        n_rec = ctx.compress_device(d_ref.data_ptr(), len(rfa), d_tgt.data_ptr(), len(tfa), d_rec.data_ptr(), cap, stream,
                                    **over)
        st = ctx.stats()
        if name.endswith("decompress"):
            need = ctx.reconstruct_device(d_ref.data_ptr(), len(rfa), d_rec.data_ptr(), n_rec, 0, 0, stream)
            d_fa = torch.empty(need + 64, dtype=torch.uint8, device=dev)
            dt, n_fa = timed(lambda: ctx.reconstruct_device(d_ref.data_ptr(), len(rfa), d_rec.data_ptr(), n_rec,
                                                           d_fa.data_ptr(), need + 64, stream))
            exact = d_fa[:n_fa].cpu().numpy().tobytes() == tfa
            out = {"workload": name, "target_bases": st["target_bases"], "record_bytes": n_rec, "seconds": dt,
                   "bases_per_s": st["target_bases"] / dt, "roundtrip_exact": exact}
        else:
            dt, n = timed(lambda: ctx.compress_device(d_ref.data_ptr(), len(rfa), d_tgt.data_ptr(), len(tfa),
                                                      d_rec.data_ptr(), cap, stream, **over))
            st = ctx.stats()
            out = {"workload": name, "target_bases": st["target_bases"], "record_bytes": n, "seconds": dt,
                   "bases_per_s": st["target_bases"] / dt, "mode": "global" if st["mode_global"] else "local",
                   "switch_segment": st["switch_segment"], "walk_rounds": st["walk_rounds"], "matches": st["n_matches"]}
            if over:
                out["params"] = over
                rec = d_rec[:n].cpu().numpy().tobytes()
                out["roundtrip_exact"] = ctx.reconstruct(rec, rfa) == tfa
        print(json.dumps(out), flush=True)
        del d_ref, d_tgt, d_rec
        torch.cuda.empty_cache()


def genome(ctx, dev, stream, args, to_dev) -> None:
    """BASELINE configs[2] on one GPU: every chromosome pair resident in HBM, compressed in turn."""
    import torch
    import multigpu
    import sccg
    import synth
    t0 = time.perf_counter()
    pairs = []
    for i, (rl, tl) in enumerate(zip(multigpu.HG18, multigpu.HG19)):
        rfa, tfa = synth.synth_pair(args.genome_profile, int(rl * args.scale), int(tl * args.scale), i + 1)
        pairs.append((to_dev(rfa), len(rfa), to_dev(tfa), len(tfa)))
        print(f"[genome] pair {i + 1}/24 generated ({time.perf_counter() - t0:.1f} s)", file=sys.stderr, flush=True)
        del rfa, tfa
    gen_s = time.perf_counter() - t0
    cap = max(ctx.compress_bound(r, t) for _, r, _, t in pairs)
    d_rec = torch.empty(cap, dtype=torch.uint8, device=dev)
    ctx.compress_device(pairs[20][0].data_ptr(), pairs[20][1], pairs[20][2].data_ptr(), pairs[20][3],
                        d_rec.data_ptr(), cap, stream)   # warm-up (chr21)
    # several contexts on the one GPU, each driven by its own host thread (ctypes drops the GIL):
    # one chromosome's host round trips and serial phases overlap another's kernels
    import queue
    import threading
    ctxs = [ctx] + [sccg.Context(0) for _ in range(max(0, args.contexts - 1))]
    outs = [d_rec] + [torch.empty(cap, dtype=torch.uint8, device=dev) for _ in ctxs[1:]]
    streams = [torch.cuda.Stream(dev) for _ in ctxs]
    order = sorted(range(len(pairs)), key=lambda i: -pairs[i][3])   # largest first

    def run_all():
        q = queue.Queue()
        for i in order:
            q.put(i)
        res = {}

        def worker(c, o, sm):
            torch.cuda.set_device(dev)
            while True:
                try:
                    i = q.get_nowait()
                except queue.Empty:
                    return
                dr, rn, dt_, tn = pairs[i]
                n = c.compress_device(dr.data_ptr(), rn, dt_.data_ptr(), tn, o.data_ptr(), cap, sm.cuda_stream)
                res[i] = (c.stats()["target_bases"], n)

        th = [threading.Thread(target=worker, args=(c, o, sm)) for c, o, sm in zip(ctxs, outs, streams)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        return res

    best = None
    for _ in range(args.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = run_all()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None or dt < best else best
        bases = sum(v[0] for v in res.values())
        rec_bytes = sum(v[1] for v in res.values())
        per = [res[i][0] for i in range(len(pairs))]
    # per chromosome (synchronised individually; diagnostics)
    per_s = []
    for dr, rn, dt_, tn in pairs:
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ctx.compress_device(dr.data_ptr(), rn, dt_.data_ptr(), tn, d_rec.data_ptr(), cap, stream)
        st = ctx.stats()
        per_s.append({"ms": round((time.perf_counter() - t1) * 1e3, 2), "rounds": st["walk_rounds"],
                      "switch": st["switch_segment"], "matches": st["n_matches"]})
        if args.roundtrip:   # record -> FASTA on the GPU, compared with the target on the device
            n_rec = ctx.compress_device(dr.data_ptr(), rn, dt_.data_ptr(), tn, d_rec.data_ptr(), cap, stream)
            need = ctx.reconstruct_device(dr.data_ptr(), rn, d_rec.data_ptr(), n_rec, 0, 0, stream)
            d_fa = torch.empty(need + 64, dtype=torch.uint8, device=dev)
            n_fa = ctx.reconstruct_device(dr.data_ptr(), rn, d_rec.data_ptr(), n_rec, d_fa.data_ptr(), need + 64, stream)
            per_s[-1]["roundtrip_exact"] = bool(n_fa == tn and torch.equal(d_fa[:n_fa], dt_))
            del d_fa
    for c in ctxs[1:]:
        c.close()
    wl = "hg19_vs_hg18_genome_1gpu" if args.genome_profile == "hg" else "t2t_like_genome_1gpu"
    print(json.dumps({"workload": wl, "roundtrip_all_exact": all(p.get("roundtrip_exact", False) for p in per_s) if args.roundtrip else None, "contexts": len(ctxs), "chromosomes": len(pairs), "target_bases": bases,
                      "record_bytes": rec_bytes, "seconds": best, "bases_per_s": bases / best,
                      "lpt_max_over_mean_8gpu": multigpu.max_over_mean(per, 8), "generate_seconds": gen_s,
                      "per_chromosome": dict(zip(multigpu.CHROMS, per_s))}),
          flush=True)
    del pairs, d_rec
    torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
