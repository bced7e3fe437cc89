"""ctypes binding of the CPU restatement (oracle/sccg_oracle.c) -- the parity CHECKER.

Test infrastructure only: never imported by the product package."""
from __future__ import annotations

import ctypes
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(REPO, "oracle", "libsccg_oracle.so")
_lib = None


class OracleError(RuntimeError):
    def __init__(self, rc: int, partial: bytes | None = None):
        super().__init__(f"oracle rc={rc}")
        self.rc = rc
        self.partial = partial


class OrcParams(ctypes.Structure):
    """orc_params (oracle/sccg_oracle.h): compression.cpp:373-379's constants."""
    _fields_ = [("k", ctypes.c_int), ("k2", ctypes.c_int), ("L", ctypes.c_int), ("m", ctypes.c_int),
                ("T1", ctypes.c_float), ("T2", ctypes.c_int), ("local", ctypes.c_int)]


class OrcRec(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("p", ctypes.c_int32), ("l", ctypes.c_int32),
                ("t", ctypes.c_int64)]


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle`")
        lib = ctypes.CDLL(LIB_PATH)
        pp, psz = ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)
        lib.orc_compress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, pp, psz]
        lib.orc_decompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, pp, psz]
        lib.orc_match.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_int64, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                  ctypes.POINTER(ctypes.POINTER(OrcRec)), ctypes.POINTER(ctypes.c_int64)]
        lib.orc_compress_params.argtypes = [ctypes.POINTER(OrcParams), ctypes.c_char_p, ctypes.c_size_t,
                                            ctypes.c_char_p, ctypes.c_size_t, pp, psz]
        lib.orc_params_default.argtypes = [ctypes.POINTER(OrcParams)]
        lib.orc_free.argtypes = [ctypes.c_void_p]
        lib.orc_last_mode_global.restype = ctypes.c_int
        lib.orc_last_switch_segment.restype = ctypes.c_int64
        _lib = lib
    return _lib


def _call(fn, a: bytes, b: bytes) -> bytes:
    lib = _load()
    out, n = ctypes.c_void_p(), ctypes.c_size_t()
    rc = fn(a, len(a), b, len(b), ctypes.byref(out), ctypes.byref(n))
    data = ctypes.string_at(out, n.value) if out.value else None
    if out.value:
        lib.orc_free(out)
    if rc:
        raise OracleError(rc, data)
    return data


def compress(ref_fa: bytes, tgt_fa: bytes) -> bytes:
    """compressed_genome.txt bytes (compression.cpp:320-580, without 7z)."""
    return _call(_load().orc_compress, ref_fa, tgt_fa)


def compress_params(ref_fa: bytes, tgt_fa: bytes, **overrides) -> bytes:
    """compress() with compression.cpp:373-379's constants overridden (k, k2, L, m, T1, T2, local)."""
    lib = _load()
    prm = OrcParams()
    lib.orc_params_default(ctypes.byref(prm))
    for name, v in overrides.items():
        setattr(prm, name, v)
    return _call(lambda a, na, b, nb, o, n: lib.orc_compress_params(ctypes.byref(prm), a, na, b, nb, o, n),
                 ref_fa, tgt_fa)


def last_mode() -> tuple[bool, int]:
    lib = _load()
    return bool(lib.orc_last_mode_global()), int(lib.orc_last_switch_segment())


def decompress(record: bytes, ref_fa: bytes) -> bytes:
    """reconstructed_genome.fa bytes (decompression.cpp, after 7z)."""
    return _call(_load().orc_decompress, record, ref_fa)


def match(sr: bytes, st: bytes, k: int, m: int, glob: bool, offset: int = 0):
    """compression.cpp:36 match_sequences -> [(kind, p, l, t)]"""
    lib = _load()
    recs, n = ctypes.POINTER(OrcRec)(), ctypes.c_int64()
    rc = lib.orc_match(sr, len(sr), st, len(st), k, m, int(glob), offset, ctypes.byref(recs), ctypes.byref(n))
    if rc:
        raise OracleError(rc)
    out = [(recs[i].kind, recs[i].p, recs[i].l, recs[i].t) for i in range(n.value)]
    lib.orc_free(recs)
    return out


def walk_range(sr: bytes, st: bytes, k: int, m: int, x0: int, p0: int, x_end: int):
    """The global walk from state (x0, P0) until index >= x_end (orc_walk_range): ([(t, p, l)], (x, P))."""
    lib = _load()
    fn = lib.orc_walk_range
    fn.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                   ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(ctypes.POINTER(OrcRec)),
                   ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    recs, n, ex, ep = ctypes.POINTER(OrcRec)(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    rc = fn(sr, len(sr), st, len(st), k, m, x0, p0, x_end, ctypes.byref(recs), ctypes.byref(n), ctypes.byref(ex),
            ctypes.byref(ep))
    if rc:
        raise OracleError(rc)
    out = [(recs[i].t, recs[i].p, recs[i].l) for i in range(n.value)]
    lib.orc_free(recs)
    return out, (ex.value, ep.value)


def global_sequences(ref_fa: bytes, tgt_fa: bytes) -> tuple[bytes, bytes]:
    """R', T' of the global pass: FASTA ingest (compression.cpp:181-220), toupper, N erase (:556-557)."""
    def seq(fa: bytes, target: bool) -> bytes:
        out, seen_hdr = [], False
        for line in fa.split(b"\n"):
            if target:
                if not line:
                    continue
                if not seen_hdr and line[:1] == b">":
                    seen_hdr = True
                    continue
            elif not line or line[:1] == b">":
                continue
            out.append(line)
        s = b"".join(out)
        s = bytes(c for c in s if c not in b" \t\n\v\f\r") if any(c in s for c in b" \t\v\f\r") else s
        return s.upper().replace(b"N", b"")
    return seq(ref_fa, False), seq(tgt_fa, True)
