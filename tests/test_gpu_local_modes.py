"""The local pass with and without its class-0 proof, against the oracle (GPU).

SCCG_LOCAL_PROVE selects how the local controller of compression.cpp:372-481 finds the first
switch (:462-473): 1 (the default) proves each segment class 0 before walking it, and walks it only
when the proof fails; a proved segment has no records yet, so a pair that stays local computes
them afterwards.  0 walks every segment.  The gap cases put long unproved runs without a switch
(half-copied segments, all-N segments) before a planted switch, a switch inside such a run, and
switches around segment 263 (where 64 unproved segments in a row end).  The knob is read once per
process: each mode runs in a child, and the parent compares record bytes, mode and
switch segment with the oracle's.
"""
import hashlib
import json
import os
import subprocess
import sys

import pytest

import oraclelib
from test_gpu_parity import _switch_case

HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = pytest.mark.gpu

# (seed, nseg, plant): planted switch windows near the start, deep, at the last segment, and
# pairs that stay local
CASES = [(0, 2400, None, None), (1, 2400, 4, None), (3, 2400, 9, None), (7, 2400, 1000, None), (9, 2400, 2399, None),
         (700, 17000, 16386, None), (701, 17000, None, None),
         # long unproved runs that never switch (class 1 / class 3), then a switch or none
         (11, 2400, 1500, (200, 150, (2,))), (20, 2400, None, (300, 200, (3,))), (13, 3000, 2990, (100, 70, (2, 3))),
         (14, 2400, 64, (0, 80, (2,))),
         # a switch inside a long unproved run, and one right where the run reaches 64
         (15, 2400, 230, (200, 200, (1, 2, 4))), (16, 2400, 263, (200, 100, (2,))),
         # switches at and just past segment 263
         (20, 2400, 266, (200, 62, (2,))), (21, 2400, 266, (200, 62, (2,))), (24, 2400, 266, (200, 62, (2,))),
         (17, 2400, 266, (200, 62, (2,)))]

CHILD = r"""
import hashlib, json, sys
sys.path.insert(0, HERE)
import torch
torch.zeros(1, device=torch.device("cuda", 0))   # torch's HIP runtime before the library context
from pkg import sccg
from test_gpu_parity import _switch_case
out = []
with sccg.Context(0) as ctx:
    ctx.exact_switch(EXACT)
    for seed, nseg, plant, gap in CASES:
        rfa, tfa = _switch_case(seed, nseg=nseg, plant_at=plant, gap=gap)
        rec = ctx.compress(rfa, tfa)
        st = ctx.stats()
        out.append([hashlib.sha256(rec).hexdigest(), int(st["mode_global"]), int(st["switch_segment"])])
print(json.dumps(out))
"""


@pytest.fixture(scope="module")
def want():
    res = []
    for seed, nseg, plant, gap in CASES:
        rfa, tfa = _switch_case(seed, nseg=nseg, plant_at=plant, gap=gap)
        rec = oraclelib.compress(rfa, tfa)
        mode_global, sw = oraclelib.last_mode()
        res.append([hashlib.sha256(rec).hexdigest(), int(mode_global), sw if mode_global else -1])
    return res


@pytest.mark.parametrize("mode,exact", [("0", True), ("1", True), ("1", False)],
                         ids=["walk_every_segment", "prove_first", "prove_first_probe"])
def test_local_modes_vs_oracle(want, mode, exact):
    env = dict(os.environ, SCCG_LOCAL_PROVE=mode)
    p = subprocess.run([sys.executable, "-c", f"HERE = {HERE!r}\nCASES = {CASES!r}\nEXACT = {exact!r}\n" + CHILD],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    got = json.loads(p.stdout.strip().splitlines()[-1])
    if exact:
        assert got == want
    else:   # the mode probe: same bytes and mode, a switch window at or after the first
        assert [g[:2] for g in got] == [w[:2] for w in want]
        assert all(g[2] == w[2] if w[2] < 0 else g[2] >= w[2] for g, w in zip(got, want))
