#!/usr/bin/env python3
"""Secondary measurements (not the bench.py line): device-resident throughput of
  * decompression of a chr1-sized record stream (BASELINE configs[3]),
  * compression of a T2T-like divergent pair (configs[4] shape, literal-heavy),
  * compression of a pair that stays in local mode (no switch).

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

    work = [("chr1_decompress", "hg", 247_249_719, 249_250_621, 1),
            ("t2t_like_compress", "t2t", 100_000_000, 100_000_000, 7),
            ("local_mode_compress", "local", 247_249_719, 247_249_719, 8)]
    for name, prof, rl, tl, seed in work:
        if args.only and args.only not in name:
            continue
        rl, tl = int(rl * args.scale), int(tl * args.scale)
        rfa, tfa = synth.synth_pair(prof, rl, tl, seed)
        d_ref, d_tgt = to_dev(rfa), to_dev(tfa)
        cap = ctx.compress_bound(len(rfa), len(tfa))
        d_rec = torch.empty(cap, dtype=torch.uint8, device=dev)
        n_rec = ctx.compress_device(d_ref.data_ptr(), len(rfa), d_tgt.data_ptr(), len(tfa), d_rec.data_ptr(), cap, stream)
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
                                                      d_rec.data_ptr(), cap, stream))
            st = ctx.stats()
            out = {"workload": name, "target_bases": st["target_bases"], "record_bytes": n, "seconds": dt,
                   "bases_per_s": st["target_bases"] / dt, "mode": "global" if st["mode_global"] else "local",
                   "switch_segment": st["switch_segment"], "walk_rounds": st["walk_rounds"], "matches": st["n_matches"]}
        print(json.dumps(out), flush=True)
        del d_ref, d_tgt, d_rec
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
