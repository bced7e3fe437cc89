"""ctypes binding of the synthetic-pair generator (tools/synth.c; SURVEY.md §8(d) shapes)."""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "tools", "libsccg_synth.so")
PROFILES = {"hg": 0, "local": 1, "t2t": 2}
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make` (or __graft_entry__.build())")
        lib = ctypes.CDLL(LIB_PATH)
        lib.synth_pair.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64,
                                   ctypes.c_char_p, ctypes.c_char_p,
                                   ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                   ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]
        lib.synth_pair.restype = ctypes.c_int
        lib.synth_free.argtypes = [ctypes.c_void_p]
        _lib = lib
    return _lib


def synth_pair(profile: str, ref_len: int, tgt_len: int, seed: int,
               ref_name: str = "chrR", tgt_name: str = "chrT") -> tuple[bytes, bytes]:
    lib = _load()
    a, b = ctypes.c_void_p(), ctypes.c_void_p()
    na, nb = ctypes.c_size_t(), ctypes.c_size_t()
    rc = lib.synth_pair(PROFILES[profile], ref_len, tgt_len, seed, ref_name.encode(), tgt_name.encode(),
                        ctypes.byref(a), ctypes.byref(na), ctypes.byref(b), ctypes.byref(nb))
    if rc:
        raise RuntimeError("synth_pair failed")
    try:
        return ctypes.string_at(a, na.value), ctypes.string_at(b, nb.value)
    finally:
        lib.synth_free(a)
        lib.synth_free(b)
