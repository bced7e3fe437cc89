"""Diagnostics: one fuzz case through the GPU with SCCG_DEBUG phases (run under a timeout)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sccg-genome-compression_amd"))
import fuzzgen, oraclelib, sccg
kind, seed = sys.argv[1], int(sys.argv[2])
rfa, tfa = (fuzzgen.local_case if kind == "local" else fuzzgen.global_case)(seed)
print("sizes", len(rfa), len(tfa), flush=True)
want = oraclelib.compress(rfa, tfa)
print("oracle", len(want), want[:200], flush=True)
with sccg.Context(0) as c:
    t0 = time.time()
    got = c.compress(rfa, tfa)
    print("gpu", len(got), got == want, time.time() - t0, c.stats(), flush=True)
