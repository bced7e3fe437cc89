"""The CPU restatement (oracle/, the on-box parity checker) under AddressSanitizer + UBSan.

SURVEY.md §5: the reference's sanitizer toggles are off (.vscode/settings.json:53-55); the oracle
gets them instead.  `make -C oracle sanitize` builds oracle/_san/sccg_oracle with
-fsanitize=address,undefined -fno-sanitize-recover=all; every golden fixture (outputs of the compiled
reference) runs through it -- compression and decompression -- and must give the reference's bytes
and exit code with no sanitizer report.
"""
import fcntl
import os
import subprocess

import pytest

import fuzzgen

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(REPO, "oracle", "_san", "sccg_oracle")


@pytest.fixture(scope="module")
def san_bin():
    # pytest-xdist workers each build the fixture: serialise the make so none runs the binary while
    # another relinks it
    with open(os.path.join(REPO, "oracle", ".san.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "sanitize"], capture_output=True, text=True)
    if r.returncode != 0 or not os.path.exists(SAN):
        pytest.skip("sanitizer build unavailable: " + r.stderr[-300:])
    return SAN


def _run(san, mode, a, b, tmp):
    pa, pb, po = os.path.join(tmp, "a"), os.path.join(tmp, "b"), os.path.join(tmp, "o")
    open(pa, "wb").write(a)
    open(pb, "wb").write(b)
    if os.path.exists(po):
        os.remove(po)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=99:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98")
    p = subprocess.run([san, mode, pa, pb, po], capture_output=True, env=env, timeout=120)
    err = p.stderr.decode(errors="replace")
    assert "Sanitizer" not in err and "runtime error" not in err, err[-2000:]
    assert p.returncode in (0, 1), (p.returncode, err[-2000:])
    out = open(po, "rb").read() if os.path.exists(po) else None
    return p.returncode, out


def test_golden_cases_under_sanitizers(san_bin, golden_cases, tmp_path):
    bad = []
    for c in golden_cases:
        rc, rec = _run(san_bin, "compress", c["ref_fa"], c["tgt_fa"], str(tmp_path))
        if rc != c["compress_rc"] or rec != c["record"]:
            bad.append(("compress", c["name"]))
        if c["decompress_rc"] is not None:
            rc, fa = _run(san_bin, "decompress", c["record"], c["ref_fa"], str(tmp_path))
            if rc != c["decompress_rc"] or (rc == 0 and fa != c["fasta"]):
                bad.append(("decompress", c["name"]))
    assert not bad, bad


@pytest.mark.parametrize("kind,seed", [("local", s) for s in range(5)] + [("global", s) for s in range(5)])
def test_fuzz_under_sanitizers(san_bin, kind, seed, tmp_path):
    rfa, tfa = (fuzzgen.local_case if kind == "local" else fuzzgen.global_case)(500 + seed)
    rc, rec = _run(san_bin, "compress", rfa, tfa, str(tmp_path))
    assert rc == 0 and rec
    _run(san_bin, "decompress", rec, rfa, str(tmp_path))
