import sys, os
sys.path.insert(0, "tests"); sys.path.insert(0, "sccg-genome-compression_amd")
import sccg, synth
rfa, tfa = synth.synth_pair("hg", 4_000_000, 4_010_000, 5)
with sccg.Context(0) as c:
    rec = c.compress(rfa, tfa)
    print(c.stats(), file=sys.stderr)
