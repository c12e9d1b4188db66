"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper around ``liborc.so`` (built from ``cutadapt_oracle.c`` by ``oracle/Makefile``),
the C restatement of cutadapt 4.9's alignment / best-match / --rc / two-round / linked
semantics (see that file's header for reference citations).  PARITY UNPINNED.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this
module, and only as the checker or the timed CPU baseline; the product path never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORC_LIBDIR: a sanitizer build of the same library (tools/sanitize.sh)
LIB_PATH = os.path.join(os.environ.get("ORC_LIBDIR") or HERE, "liborc.so")

FRONT, BACK = 11, 14

# Same layout as dmx_result (include/dmx.h).
RESULT_DTYPE = np.dtype([
    ("bin1", "<i2"), ("bin2", "<i2"), ("rc1", "u1"), ("rc2", "u1"), ("flags", "u1"), ("pad", "u1"),
    ("m1_rstart", "<i4"), ("m1_rstop", "<i4"), ("m1_astart", "<i2"), ("m1_astop", "<i2"),
    ("m1_score", "<i2"), ("m1_errors", "<i2"),
    ("m2_rstart", "<i4"), ("m2_rstop", "<i4"), ("m2_astart", "<i2"), ("m2_astop", "<i2"),
    ("m2_score", "<i2"), ("m2_errors", "<i2"),
])
assert RESULT_DTYPE.itemsize == 40

_lib = None


def build() -> str:
    """Compile liborc.so (gcc, seconds).  Used by __graft_entry__.build() and tests."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_locate.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                 ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.orc_panel_new.restype = ctypes.c_void_p
        L.orc_panel_new.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                    ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                    ctypes.c_double, ctypes.c_int]
        L.orc_panel_free.argtypes = [ctypes.c_void_p]
        L.orc_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                ctypes.c_void_p, ctypes.c_int]
        _lib = L
    return _lib


def locate(ref: str, query: str, max_error_rate: float, flags: int, min_overlap: int = 3):
    """Aligner.locate -> (ref_start, ref_stop, query_start, query_stop, score, errors) or None."""
    wild = 0 if set(ref) <= set("ACGT") else 1
    out = (ctypes.c_int * 6)()
    r = lib().orc_locate(ref.encode(), len(ref), query.encode(), len(query), max_error_rate,
                         flags, wild, 0, min_overlap, out)
    if r < 0:
        raise ValueError("bad adapter")
    return tuple(out) if r == 1 else None


class Panel:
    def __init__(self, seqs, where, max_errors=0.1, min_overlap=3):
        if isinstance(where, int):
            where = [where] * len(seqs)
        self.seqs = [s.upper().replace("U", "T") for s in seqs]
        arr = (ctypes.c_char_p * len(seqs))(*[s.encode() for s in self.seqs])
        lens = (ctypes.c_int * len(seqs))(*[len(s) for s in self.seqs])
        wh = (ctypes.c_int * len(seqs))(*where)
        self._p = lib().orc_panel_new(len(seqs), arr, lens, wh, float(max_errors), min_overlap)
        if not self._p:
            raise ValueError("bad panel")

    def __del__(self):
        if getattr(self, "_p", None):
            lib().orc_panel_free(self._p)
            self._p = None


def run_batch(p1: Panel, p2: Panel | None, seqs_blob: np.ndarray, offsets: np.ndarray,
              lengths: np.ndarray, mode: int, use_rc: bool = True, threads: int = 1) -> np.ndarray:
    """mode 0 single round, 1 two rounds, 2 linked.  seqs_blob: uint8 ASCII concatenation."""
    n = len(lengths)
    res = np.zeros(n, dtype=RESULT_DTYPE)
    blob = np.ascontiguousarray(seqs_blob, dtype=np.uint8)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = np.ascontiguousarray(lengths, dtype=np.uint32)
    lib().orc_batch(p1._p, p2._p if p2 is not None else None, mode, int(use_rc),
                    blob.ctypes.data, offs.ctypes.data, lens.ctypes.data, n, res.ctypes.data,
                    threads)
    return res


def pack_ascii(seqs):
    """list[str] -> (blob uint8, offsets u64, lengths u32) for run_batch."""
    lens = np.array([len(s) for s in seqs], dtype=np.uint32)
    offs = np.zeros(len(seqs), dtype=np.uint64)
    if len(seqs) > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    blob = np.frombuffer("".join(seqs).encode("ascii"), dtype=np.uint8)
    return blob, offs, lens
