"""Diagnostics: one compression of a synthetic pair with SCCG_DEBUG traces of the global walk.

    SCCG_DEBUG=1 python sccg-genome-compression_amd/tools/dbg_walk.py [profile] [ref_len] [tgt_len] [seed]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sccg  # noqa: E402
import synth  # noqa: E402

prof = sys.argv[1] if len(sys.argv) > 1 else "hg"
rl = int(sys.argv[2]) if len(sys.argv) > 2 else 4_000_000
tl = int(sys.argv[3]) if len(sys.argv) > 3 else rl + rl // 400
seed = int(sys.argv[4]) if len(sys.argv) > 4 else 5
rfa, tfa = synth.synth_pair(prof, rl, tl, seed)
with sccg.Context(0) as c:
    for i in range(2):
        t0 = time.perf_counter()
        rec = c.compress(rfa, tfa)
        print(f"compress {i}: {time.perf_counter() - t0:.3f} s", c.stats(), file=sys.stderr)
