#!/usr/bin/env python3
"""Device-resident reconstruction time of one synthetic pair's record stream (diagnostics / A/B).

    python bench_decomp.py <profile> <ref_len> <tgt_len> <seed> [--steps 10] [--prof]
Compresses the pair once, then times sccg_reconstruct_device; prints one JSON line (median / min ms,
round trip exact, per-kernel HIP-event ms per call with --prof)."""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("profile")
    ap.add_argument("ref_len", type=int)
    ap.add_argument("tgt_len", type=int)
    ap.add_argument("seed", type=int)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--prof", action="store_true")
    a = ap.parse_args()
    import torch
    import sccg
    import synth
    dev = torch.device("cuda", 0)
    rfa, tfa = synth.synth_pair(a.profile, a.ref_len, a.tgt_len, a.seed)
    ctx = sccg.Context(0)
    rec_h = ctx.compress(rfa, tfa)
    d_ref = torch.frombuffer(bytearray(rfa), dtype=torch.uint8).to(dev)
    d_rec = torch.frombuffer(bytearray(rec_h), dtype=torch.uint8).to(dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    need = ctx.reconstruct_device(d_ref.data_ptr(), len(rfa), d_rec.data_ptr(), len(rec_h), 0, 0, s)
    d_fa = torch.empty(need + 64, dtype=torch.uint8, device=dev)
    ts, extra = [], {}
    for i in range(a.steps + 1):
        if a.prof and i == 1:
            ctx.profile(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = ctx.reconstruct_device(d_ref.data_ptr(), len(rfa), d_rec.data_ptr(), len(rec_h), d_fa.data_ptr(), need + 64, s)
        torch.cuda.synchronize()
        if i:
            ts.append((time.perf_counter() - t0) * 1e3)
    if a.prof:
        extra["kernels_ms"] = {k: round(v[0] / a.steps, 4) for k, v in ctx.profile_get().items() if v[1]}
        ctx.profile(False)
    exact = d_fa[:n].cpu().numpy().tobytes() == tfa
    print(json.dumps({**extra, "pair": f"{a.profile}-{a.ref_len}-{a.tgt_len}-{a.seed}", "ms_median": round(statistics.median(ts), 3),
                      "ms_min": round(min(ts), 3), "exact": exact,
                      "env": {k: v for k, v in os.environ.items() if k.startswith("SCCG_")}}))


if __name__ == "__main__":
    main()
