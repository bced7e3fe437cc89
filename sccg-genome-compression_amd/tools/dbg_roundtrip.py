"""Diagnostics: compress + reconstruct one small synthetic pair in-process (faulthandler dumps the
stack if it hangs).  SCCG_DBG_ONLY_RECON=1 reconstructs the oracle's record instead of compressing."""
import faulthandler
import os
import sys

faulthandler.dump_traceback_later(int(os.environ.get("DBG_TIMEOUT", "40")), exit=True)
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "sccg-genome-compression_amd"))
import oraclelib  # noqa: E402
import sccg  # noqa: E402
import synthlib  # noqa: E402

rfa, tfa = synthlib.synth_pair("hg", 600_000, 601_500, 31)
rec = oraclelib.compress(rfa, tfa)
print("oracle record", len(rec), flush=True)
with sccg.Context(0) as ctx:
    fa = ctx.reconstruct(rec, rfa)
    print("reconstructed", fa == tfa, flush=True)
