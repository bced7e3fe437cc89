"""Opt-in reconstruction paths and the profiler's family mask (GPU).

* The token fill (decompression.cpp:210-236) is queued before the host knows the decoded length,
  into a buffer of the output's capacity, beside the readback (the default, exercised by every
  other reconstruction test); SCCG_DC_SPEC=0 queues it after the host read the length.  Both must
  stay exact: round trips against the target FASTA, a too-small output buffer (SCCG_E_NOMEM, also
  below the decoded length itself), a far larger one, and tokens beyond the reference (:223-229,
  SCCG_E_RANGE).  The knob is read once per process, so the
  checks run in a child process.
* The same child with the round-5 orders and passes: SCCG_STRIP_KC=0 (the strips' write pass
  classifies every tile again instead of taking plain tiles' masks from the summary) and
  SCCG_DC_RUNS_FIRST=0 (the record line's parse chain issued before the run lines'); the record
  streams are checked against the oracle there too.
* sccg_profile with a family mask brackets only those families (bench.py's timed region).
"""
import json
import os
import subprocess
import sys

import pytest

from pkg import sccg

HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = sccg.Context(0)
    yield c
    c.close()


CHILD = r"""
import json, sys
sys.path.insert(0, HERE)
import torch
import synthlib
import oraclelib
from pkg import sccg
dev = torch.device("cuda", 0)
torch.zeros(1, device=dev)   # torch's HIP runtime before the library context
ctx = sccg.Context(0)
out = {"round_trips": [], "nomem": None, "range": [], "oracle": []}

def dev_bytes(b):
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)

def run(rfa, rec, cap):
    d_r, d_c = dev_bytes(rfa), dev_bytes(rec)
    d_o = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
    n = ctx.reconstruct_device(d_r.data_ptr(), len(rfa), d_c.data_ptr(), len(rec), d_o.data_ptr(), cap)
    torch.cuda.synchronize()
    return d_o[:n].cpu().numpy().tobytes()

for prof, rl, tl, seed in (("hg", 200_000, 201_000, 3), ("hg", 1_000_000, 1_003_000, 4), ("t2t", 300_000, 300_000, 5)):
    rfa, tfa = synthlib.synth_pair(prof, rl, tl, seed)
    rec = ctx.compress(rfa, tfa)
    out["oracle"].append(rec == oraclelib.compress(rfa, tfa))
    need = ctx.reconstruct_device(dev_bytes(rfa).data_ptr(), len(rfa), dev_bytes(rec).data_ptr(), len(rec), 0, 0)
    got = run(rfa, rec, need + 64)
    out["round_trips"].append(got == tfa)
    if seed == 3:
        try:
            run(rfa, rec, need - 1)
            out["nomem"] = 0
        except sccg.SccgError as e:
            out["nomem"] = e.rc
        # a capacity below the decoded length D itself: the speculative fill's clamp is what keeps
        # its writes inside the buffer (ADVICE r4)
        try:
            run(rfa, rec, len(tfa) // 3)
            out["nomem_below_d"] = 0
        except sccg.SccgError as e:
            out["nomem_below_d"] = e.rc
        # a far larger capacity than the record can need: the non-speculative path, still exact
        out["big_cap"] = run(rfa, rec, need + (160 << 20)) == tfa
rfa = b">r\n" + b"ACGT" * 50 + b"\n"
for rec in (b"\n,\n(0,20)(500,30)", b">h\n\n(3,2)\n(0,20)(500,30)", b"\n,\nAC(190,20)"):
    try:
        run(rfa, rec, 1 << 16)
        out["range"].append(0)
    except sccg.SccgError as e:
        out["range"].append(e.rc)
ctx.close()
print(json.dumps(out))
"""


@pytest.mark.parametrize("knobs", [{"SCCG_DC_SPEC": "0"}, {}, {"SCCG_STRIP_KC": "0", "SCCG_DC_RUNS_FIRST": "0"}],
                         ids=["fill_after_readback", "speculative_fill", "round5_strip_and_order"])
def test_fill_round_trips_and_errors(knobs):
    env = dict(os.environ)
    for k in ("SCCG_DC_SPEC", "SCCG_STRIP_KC", "SCCG_DC_RUNS_FIRST"):
        env.pop(k, None)
    env.update(knobs)
    p = subprocess.run([sys.executable, "-c", f"HERE = {HERE!r}\n" + CHILD], env=env, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["round_trips"] == [True, True, True], d
    assert d["oracle"] == [True, True, True], d
    assert d["nomem"] == sccg.ERR_CODES["SCCG_E_NOMEM"], d
    assert d["nomem_below_d"] == sccg.ERR_CODES["SCCG_E_NOMEM"], d
    assert d["big_cap"] is True, d
    assert d["range"] == [sccg.ERR_CODES["SCCG_E_RANGE"]] * 3, d


def test_profile_family_mask(ctx):
    import synthlib
    rfa, tfa = synthlib.synth_pair("hg", 2_000_000, 2_010_000, 6)
    ctx.profile(True, families=["walk"])
    ctx.compress(rfa, tfa)
    only = ctx.profile_get()
    ctx.profile(True)
    ctx.compress(rfa, tfa)
    every = ctx.profile_get()
    ctx.profile(False)
    assert set(only) <= {"walk"}, only
    assert "walk" in every and len(every) > 1, every
    # family 0 alone (its mask is 1, which sccg_profile(ctx, 1) reads as "every family")
    first = sccg.load_library().sccg_profile_name(0).decode()
    ctx.profile(True, families=[first])
    ctx.compress(rfa, tfa)
    zero = ctx.profile_get()
    ctx.profile(False)
    assert set(zero) == {first}, zero
    with pytest.raises(ValueError):
        ctx.profile(True, families=["no_such_family"])
