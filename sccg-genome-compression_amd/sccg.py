"""ctypes binding of libsccg.so (include/sccg.h) -- the MI355X SCCG hot path.

Mirrors the reference's two entry points (compression.cpp:320 compress_genome up to 7z,
decompression.cpp:117 reconstruct_genome + file body) and the match_sequences seam
(compression.cpp:36).  There is no CPU fallback: if the HIP library or a GPU is missing,
construction raises.
"""
from __future__ import annotations

import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
# SCCG_LIB_PATH: an alternative build of the same library (tuning runs compare variants)
LIB_PATH = os.environ.get("SCCG_LIB_PATH") or os.path.join(HERE, "lib", "libsccg.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "sccg.h")

SCCG_OK = 0
SCCG_E_DELTA_STOI = 4
OPT_EXACT_SWITCH = 1   # sccg_ctx_set_option (include/sccg.h)
ERRORS = {1: "SCCG_E_INVALID", 2: "SCCG_E_HIP", 3: "SCCG_E_NOMEM", 4: "SCCG_E_DELTA_STOI",
          5: "SCCG_E_FORMAT", 6: "SCCG_E_RANGE", 7: "SCCG_E_PARSE", 8: "SCCG_E_UNSUPPORTED",
          9: "SCCG_E_INTERNAL", 10: "SCCG_E_OPEN_REF", 11: "SCCG_E_OPEN_TGT", 12: "SCCG_E_WRITE"}
ERR_CODES = {v: k for k, v in ERRORS.items()}


class SccgError(RuntimeError):
    def __init__(self, rc: int, msg: str = ""):
        super().__init__(f"{ERRORS.get(rc, rc)}: {msg}")
        self.rc = rc


class Buf(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_size_t)]


class Records(ctypes.Structure):
    _fields_ = [("kind", ctypes.POINTER(ctypes.c_uint8)), ("pos", ctypes.POINTER(ctypes.c_int32)),
                ("len", ctypes.POINTER(ctypes.c_int32)), ("t", ctypes.POINTER(ctypes.c_int64)),
                ("n", ctypes.c_int64)]


class Stats(ctypes.Structure):
    _fields_ = [("mode_global", ctypes.c_int), ("switch_segment", ctypes.c_int64),
                ("target_bases", ctypes.c_int64), ("reference_bases", ctypes.c_int64),
                ("n_matches", ctypes.c_int64), ("literal_bases", ctypes.c_int64),
                ("walk_rounds", ctypes.c_int64), ("walk_chunks", ctypes.c_int64),
                ("record_bytes", ctypes.c_int64), ("walk_chains", ctypes.c_int64),
                ("walk_reference_bases", ctypes.c_int64)]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class Params(ctypes.Structure):
    """sccg_params (include/sccg.h): compression.cpp:373-379's constants; other values than the
    defaults are non-parity overrides (local=1 takes only m; local=0 takes 1 <= k <= 32, m)."""
    _fields_ = [("k", ctypes.c_int32), ("k2", ctypes.c_int32), ("L", ctypes.c_int32), ("m", ctypes.c_int32),
                ("T1", ctypes.c_float), ("T2", ctypes.c_int32), ("local", ctypes.c_int32)]


_lib = None


def hip_runtimes() -> list[str]:
    """The distinct libamdhip64 files mapped into this process (/proc/self/maps)."""
    try:
        with open("/proc/self/maps") as f:
            return sorted({ln.split()[-1] for ln in f if "libamdhip64" in ln and "/" in ln})
    except OSError:
        return []


def load_library():
    """Load libsccg.so (raises if it was not built: no silent fallback).

    One HIP runtime per process: torch ships its own libamdhip64 (SONAME libamdhip64.so.7, the same
    as /opt/rocm's that libsccg links), and whichever is loaded first serves every later user of
    that SONAME -- but torch's libraries name the file (libamdhip64.so, RPATH $ORIGIN), so loading
    libsccg before torch maps BOTH runtimes, and torch then sees no GPU.  So torch (when installed)
    is imported first and its runtime serves libsccg too; a process that still ends up with two
    runtimes mapped is refused with a clear message instead of failing later in a HIP call.  The
    C CLIs (no torch) run on /opt/rocm's runtime."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run `make` or __graft_entry__.build()")
    try:
        import torch  # noqa: F401  (its HIP runtime first: see above)
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    rts = hip_runtimes()
    if len({os.path.realpath(r) for r in rts}) > 1:
        raise RuntimeError("two HIP runtimes are mapped into this process (" + ", ".join(rts) + "): libsccg was "
                           "loaded before torch; import torch (or sccg) before loading libsccg.so yourself")
    vp, sz, c, i64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_int64
    lib.sccg_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    lib.sccg_ctx_destroy.argtypes = [vp]
    lib.sccg_last_error.argtypes = [vp]
    lib.sccg_last_error.restype = ctypes.c_char_p
    lib.sccg_last_stats.argtypes = [vp, ctypes.POINTER(Stats)]
    lib.sccg_ctx_set_option.argtypes = [vp, ctypes.c_int, i64]
    lib.sccg_compress.argtypes = [vp, c, sz, c, sz, ctypes.POINTER(Buf)]
    lib.sccg_compress_device.argtypes = [vp, vp, sz, vp, sz, vp, sz, ctypes.POINTER(sz), vp]
    if hasattr(lib, "sccg_params_default"):   # (absent from builds older than the overrides: A/B runs)
        lib.sccg_params_default.argtypes = [ctypes.POINTER(Params)]
        lib.sccg_compress_ex.argtypes = [vp, ctypes.POINTER(Params), c, sz, c, sz, ctypes.POINTER(Buf)]
        lib.sccg_compress_device_ex.argtypes = [vp, ctypes.POINTER(Params), vp, sz, vp, sz, vp, sz, ctypes.POINTER(sz), vp]
    if hasattr(lib, "sccg_compress_files"):
        lib.sccg_compress_files.argtypes = [vp, ctypes.POINTER(Params), c, c, c, ctypes.POINTER(sz)]
    lib.sccg_compress_bound.argtypes = [sz, sz]
    lib.sccg_compress_bound.restype = sz
    lib.sccg_match.argtypes = [vp, c, sz, c, sz, ctypes.c_int, ctypes.c_int, ctypes.c_int, i64,
                               ctypes.POINTER(Records)]
    lib.sccg_records_free.argtypes = [ctypes.POINTER(Records)]
    if hasattr(lib, "sccg_walk_range"):
        lib.sccg_walk_range.argtypes = [vp, c, sz, c, sz, ctypes.c_int, ctypes.c_int, i64, i64, i64,
                                        ctypes.POINTER(Records), ctypes.POINTER(i64)]
        lib.sccg_walk_range_device.argtypes = [vp, vp, sz, vp, sz, ctypes.c_int, ctypes.c_int, i64, i64, i64,
                                               ctypes.POINTER(Records), ctypes.POINTER(i64), vp]
    lib.sccg_reconstruct.argtypes = [vp, c, sz, c, sz, ctypes.POINTER(Buf)]
    lib.sccg_reconstruct_device.argtypes = [vp, vp, sz, vp, sz, vp, sz, ctypes.POINTER(sz), vp]
    lib.sccg_buf_free.argtypes = [ctypes.POINTER(Buf)]
    lib.sccg_profile.argtypes = [vp, ctypes.c_int]
    lib.sccg_profile_mask.argtypes = [vp, ctypes.c_uint32]
    lib.sccg_profile_get.argtypes = [vp, c, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i64)]
    lib.sccg_profile_name.argtypes = [ctypes.c_int]
    lib.sccg_profile_name.restype = ctypes.c_char_p
    _lib = lib
    return lib


def header_functions() -> list[str]:
    """Every function the C ABI header declares."""
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|size_t|const char\*)\s+(sccg_\w+)\s*\(", text, re.M)))


class Context:
    """One GPU context (sccg_ctx).  Not re-entrant; one per device."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        self.ptr = ctypes.c_void_p()
        rc = self.lib.sccg_ctx_create(device, ctypes.byref(self.ptr))
        if rc:
            raise SccgError(rc, f"sccg_ctx_create(device={device}) failed: no usable GPU")

    def close(self):
        if self.ptr:
            self.lib.sccg_ctx_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self, rc: int):
        raise SccgError(rc, self.lib.sccg_last_error(self.ptr).decode(errors="replace"))

    def set_option(self, option: int, value: int) -> None:
        """sccg_ctx_set_option (include/sccg.h), e.g. OPT_EXACT_SWITCH."""
        rc = self.lib.sccg_ctx_set_option(self.ptr, option, value)
        if rc:
            self._err(rc)

    def exact_switch(self, on: bool = True) -> None:
        """stats()['switch_segment'] = the reference's first switch (the in-order local pass)
        instead of any switch window (the default mode probe); the record bytes are the same."""
        self.set_option(OPT_EXACT_SWITCH, int(on))

    def stats(self) -> dict:
        st = Stats()
        self.lib.sccg_last_stats(self.ptr, ctypes.byref(st))
        return st.as_dict()

    def _take(self, buf: Buf) -> bytes:
        data = ctypes.string_at(buf.data, buf.len) if buf.data else b""
        self.lib.sccg_buf_free(ctypes.byref(buf))
        return data

    def params(self, **overrides) -> Params:
        """sccg_params: the reference's constants (compression.cpp:373-379) with `overrides` applied."""
        prm = Params()
        self.lib.sccg_params_default(ctypes.byref(prm))
        for name, v in overrides.items():
            if name not in dict(Params._fields_):
                raise TypeError(f"unknown parameter {name!r}")
            setattr(prm, name, v)
        return prm

    def compress(self, ref_fa: bytes, tgt_fa: bytes, **overrides) -> bytes:
        """Bytes of compressed_genome.txt (compression.cpp:320-580, without 7z).  Keyword overrides
        (k, k2, L, m, T1, T2, local) go through sccg_compress_ex as non-parity parameters."""
        buf = Buf()
        if overrides:
            rc = self.lib.sccg_compress_ex(self.ptr, ctypes.byref(self.params(**overrides)), ref_fa, len(ref_fa),
                                           tgt_fa, len(tgt_fa), ctypes.byref(buf))
        else:
            rc = self.lib.sccg_compress(self.ptr, ref_fa, len(ref_fa), tgt_fa, len(tgt_fa), ctypes.byref(buf))
        if rc:
            data = self._take(buf)
            err = SccgError(rc, self.lib.sccg_last_error(self.ptr).decode(errors="replace"))
            err.partial = data
            raise err
        return self._take(buf)

    def compress_files(self, ref_path: str, tgt_path: str, out_path: str, **overrides) -> int:
        """FASTA files -> record file out_path (sccg_compress_files: compression.cpp:181-220, :320-331,
        without 7z); returns the bytes written.  SCCG_E_DELTA_STOI raises after writing the file."""
        n = ctypes.c_size_t()
        prm = ctypes.byref(self.params(**overrides)) if overrides else None
        rc = self.lib.sccg_compress_files(self.ptr, prm, os.fsencode(ref_path), os.fsencode(tgt_path),
                                          os.fsencode(out_path), ctypes.byref(n))
        if rc:
            self._err(rc)
        return n.value

    def reconstruct(self, record: bytes, ref_fa: bytes) -> bytes:
        """Bytes of reconstructed_genome.fa (decompression.cpp after 7z)."""
        buf = Buf()
        rc = self.lib.sccg_reconstruct(self.ptr, ref_fa, len(ref_fa), record, len(record), ctypes.byref(buf))
        if rc:
            self._err(rc)
        return self._take(buf)

    def compress_device(self, d_ref: int, ref_len: int, d_tgt: int, tgt_len: int, d_out: int, out_cap: int,
                        stream: int = 0, **overrides) -> int:
        """HBM-resident compress: device pointers in, record text written to d_out; returns length."""
        n = ctypes.c_size_t()
        if overrides:
            rc = self.lib.sccg_compress_device_ex(self.ptr, ctypes.byref(self.params(**overrides)), d_ref, ref_len,
                                                  d_tgt, tgt_len, d_out, out_cap, ctypes.byref(n), stream or None)
        else:
            rc = self.lib.sccg_compress_device(self.ptr, d_ref, ref_len, d_tgt, tgt_len, d_out, out_cap,
                                               ctypes.byref(n), stream or None)
        if rc:
            self._err(rc)
        return n.value

    def reconstruct_device(self, d_ref: int, ref_len: int, d_rec: int, rec_len: int, d_out: int, out_cap: int,
                           stream: int = 0) -> int:
        n = ctypes.c_size_t()
        rc = self.lib.sccg_reconstruct_device(self.ptr, d_ref, ref_len, d_rec, rec_len, d_out, out_cap,
                                              ctypes.byref(n), stream or None)
        if rc:
            self._err(rc)
        return n.value

    def profile(self, enable: bool = True, families: list | None = None) -> None:
        """Reset and enable (or disable) per-kernel HIP-event timing; `families` (names from
        sccg_profile_name) limits the bracketed launches to those families."""
        if enable and families:
            mask, i = 0, 0
            while True:
                name = self.lib.sccg_profile_name(i)
                if not name:
                    break
                if name.decode() in families:
                    mask |= 1 << i
                i += 1
            if not mask:
                raise ValueError(f"profile: unknown kernel families {families}")
            self.lib.sccg_profile_mask(self.ptr, mask)
            return
        self.lib.sccg_profile(self.ptr, int(enable))

    def profile_get(self) -> dict:
        """{kernel family: (total_ms, launches)} since the last profile() call."""
        out, i = {}, 0
        while True:
            name = self.lib.sccg_profile_name(i)
            if not name:
                return out
            ms, n = ctypes.c_double(), ctypes.c_int64()
            self.lib.sccg_profile_get(self.ptr, name, ctypes.byref(ms), ctypes.byref(n))
            if n.value:
                out[name.decode()] = (ms.value, n.value)
            i += 1

    def compress_bound(self, ref_len: int, tgt_len: int) -> int:
        return self.lib.sccg_compress_bound(ref_len, tgt_len)

    @staticmethod
    def compress_bound_static(ref_len: int, tgt_len: int) -> int:
        """sccg_compress_bound without a context (it needs no device)."""
        return load_library().sccg_compress_bound(ref_len, tgt_len)

    def _walk_out(self, rc: int, recs: Records, ex) -> tuple[list, tuple[int, int]]:
        try:
            if rc:
                self._err(rc)
            out = [(recs.t[i], recs.pos[i], recs.len[i]) for i in range(recs.n)]
        finally:   # (the library frees on its own error paths too; freeing zeroed records is a no-op)
            self.lib.sccg_records_free(ctypes.byref(recs))
        return out, (ex[0], ex[1])

    def walk_range(self, sr: bytes, st: bytes, k: int, m: int, x0: int, p0: int, x_end: int):
        """The global walk (compression.cpp:64-161) from state (x0, P0) until index >= x_end on the
        N-erased uppercase R', T' (sccg_walk_range): ([(t, p, l)], (exit index, exit P))."""
        recs, ex = Records(), (ctypes.c_int64 * 2)()
        rc = self.lib.sccg_walk_range(self.ptr, sr, len(sr), st, len(st), k, m, x0, p0, x_end, ctypes.byref(recs), ex)
        return self._walk_out(rc, recs, ex)

    def walk_range_device(self, d_r: int, nr: int, d_t: int, nt: int, k: int, m: int, x0: int, p0: int, x_end: int,
                          stream: int = 0):
        """walk_range on device-resident R', T' (sccg_walk_range_device)."""
        recs, ex = Records(), (ctypes.c_int64 * 2)()
        rc = self.lib.sccg_walk_range_device(self.ptr, d_r, nr, d_t, nt, k, m, x0, p0, x_end, ctypes.byref(recs), ex,
                                             stream or None)
        return self._walk_out(rc, recs, ex)

    def match(self, sr: bytes, st: bytes, k: int, m: int, glob: bool, offset: int = 0):
        """match_sequences (compression.cpp:36) -> [(kind, p, l, t)] like the oracle's records."""
        recs = Records()
        rc = self.lib.sccg_match(self.ptr, sr, len(sr), st, len(st), k, m, int(glob), offset, ctypes.byref(recs))
        if rc:
            self._err(rc)
        out = [(recs.kind[i], recs.pos[i] if recs.kind[i] else 0, recs.len[i], recs.t[i]) for i in range(recs.n)]
        self.lib.sccg_records_free(ctypes.byref(recs))
        return out
