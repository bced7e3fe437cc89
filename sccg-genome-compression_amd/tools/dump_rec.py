import sys, os
sys.path.insert(0, 'sccg-genome-compression_amd')
import sccg, synth
rfa, tfa = synth.synth_pair("hg", 247_249_719, 249_250_621, 1)
with sccg.Context(0) as c:
    rec = c.compress(rfa, tfa)
os.makedirs("gpurun_out", exist_ok=True)
open("gpurun_out/chr1.rec", "wb").write(rec)
print(len(rec))
