#!/usr/bin/env python3
"""Device-resident compress time of one synthetic pair (diagnostics / A/B of tuning knobs).

    python bench_pair.py <profile> <ref_len> <tgt_len> <seed> [--steps 5]
Prints one JSON line: median and min ms per compress, walk rounds, chains."""
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
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--sha", action="store_true", help="also print the record's sha256")
    ap.add_argument("--prof", action="store_true", help="per-kernel HIP-event totals per call (timed steps)")
    a = ap.parse_args()
    import torch
    import sccg
    import synth
    dev = torch.device("cuda", 0)
    rfa, tfa = synth.synth_pair(a.profile, a.ref_len, a.tgt_len, a.seed)
    d_ref = torch.frombuffer(bytearray(rfa), dtype=torch.uint8).to(dev)
    d_tgt = torch.frombuffer(bytearray(tfa), dtype=torch.uint8).to(dev)
    ctx = sccg.Context(0)
    cap = ctx.compress_bound(len(rfa), len(tfa))
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ts = []
    for i in range(a.steps + 1):
        if a.prof and i == 1:
            ctx.profile(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.compress_device(d_ref.data_ptr(), len(rfa), d_tgt.data_ptr(), len(tfa), d_out.data_ptr(), cap, stream)
        torch.cuda.synchronize()
        if i:
            ts.append((time.perf_counter() - t0) * 1e3)
    st = ctx.stats()
    extra = {}
    if a.prof:
        extra["kernels_ms"] = {k: round(v[0] / a.steps, 4) for k, v in ctx.profile_get().items() if v[1]}
        ctx.profile(False)
    if a.sha:
        import hashlib
        extra["record_sha256"] = hashlib.sha256(d_out[:st["record_bytes"]].cpu().numpy().tobytes()).hexdigest()
    print(json.dumps({**extra, "pair": f"{a.profile}-{a.ref_len}-{a.tgt_len}-{a.seed}", "ms_median": round(statistics.median(ts), 3),
                      "ms_min": round(min(ts), 3), "rounds": st["walk_rounds"], "chains": st["walk_chains"],
                      "env": {k: v for k, v in os.environ.items() if k.startswith("SCCG_")}}))


if __name__ == "__main__":
    main()
