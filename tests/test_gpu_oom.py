"""Optional-allocation fallbacks after a real hipMalloc failure (GPU).

Two device allocations are optional: the target strip's run-event slots (without them the run
lines of compression.cpp:341-368 / :527-555 come from separate passes over T) and the
reconstruction's speculative token-fill buffer (without it the fill waits for the decoded length,
decompression.cpp:210-236).  SCCG_TEST_OOM=<slot>,... makes the first allocation of each listed
context slot ask for 2^62 bytes, so hipMalloc really fails and HIP records the error; the call must
then take its fallback and stay exact (the library clears HIP's last error after a failed
allocation -- before the fix the next launch check reported the out-of-memory and the call failed).
Slot numbers: B_RSLOT = 62, B_D_DEC = 43 (static_assert in sccg_api.cpp).  The knob is read once
per process, so the checks run in a child process.
"""
import json
import os
import subprocess
import sys

import pytest

import oraclelib
import synthlib

HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = pytest.mark.gpu

PAIRS = (("hg", 300_000, 302_000, 11), ("t2t", 200_000, 200_000, 12))

CHILD = r"""
import hashlib, json, sys
sys.path.insert(0, HERE)
import torch
torch.zeros(1, device=torch.device("cuda", 0))   # torch's HIP runtime before the library context
import synthlib
from pkg import sccg
out = []
with sccg.Context(0) as ctx:
    for prof, rl, tl, seed in PAIRS:
        rfa, tfa = synthlib.synth_pair(prof, rl, tl, seed)
        rec = ctx.compress(rfa, tfa)
        back = ctx.reconstruct(rec, rfa)
        out.append([hashlib.sha256(rec).hexdigest(), back == tfa])
print(json.dumps(out))
"""


@pytest.mark.parametrize("slots", ["62", "43", "62,43"], ids=["run_slots", "spec_fill", "both"])
def test_alloc_fallbacks_exact(slots):
    import hashlib
    want = []
    for prof, rl, tl, seed in PAIRS:
        rfa, tfa = synthlib.synth_pair(prof, rl, tl, seed)
        want.append([hashlib.sha256(oraclelib.compress(rfa, tfa)).hexdigest(), True])
    env = dict(os.environ, SCCG_TEST_OOM=slots)
    p = subprocess.run([sys.executable, "-c", f"HERE = {HERE!r}\nPAIRS = {PAIRS!r}\n" + CHILD], env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    assert json.loads(p.stdout.strip().splitlines()[-1]) == want
