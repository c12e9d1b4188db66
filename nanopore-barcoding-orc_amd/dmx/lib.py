"""ctypes binding of libdmx.so (the C-ABI declared in include/dmx.h).

The product path has exactly one compute backend: the HIP kernels in libdmx.so.  If the
library is missing or no GPU is visible, the calls raise — there is no CPU fallback.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# DMX_LIBDMX: an alternative in-tree build of the same library (A/B kernel variants)
# DMX_LIBDIR: a directory with another build of every library (host sanitizer builds)
# DMX_DEBUG_BOUNDS=1: the bounds-checking build (every gather and slot access checked; a
#   violation fails the call naming the kernel), dmx/libdmx_bounds.so
BOUNDS = os.environ.get("DMX_DEBUG_BOUNDS", "") not in ("", "0")
LIB_PATH = os.environ.get("DMX_LIBDMX") or os.path.join(
    os.environ.get("DMX_LIBDIR") or HERE, "libdmx_bounds.so" if BOUNDS else "libdmx.so")

DMX_FRONT, DMX_BACK, DMX_RC = 0x01, 0x02, 0x10
MODE_SINGLE, MODE_TWO_ROUND, MODE_LINKED = 0, 1, 2
PACK_PAD = 64

MATCH_FIELDS = [("rstart", "<i4"), ("rstop", "<i4"), ("astart", "<i2"), ("astop", "<i2"),
                ("score", "<i2"), ("errors", "<i2")]
RESULT_DTYPE = np.dtype([("bin1", "<i2"), ("bin2", "<i2"), ("rc1", "u1"), ("rc2", "u1"),
                         ("flags", "u1"), ("pad", "u1")]
                        + [("m1_" + n, t) for n, t in MATCH_FIELDS]
                        + [("m2_" + n, t) for n, t in MATCH_FIELDS])
assert RESULT_DTYPE.itemsize == 40

EXPORTS = ["dmx_abi_version", "dmx_open", "dmx_close", "dmx_last_error", "dmx_set_panel",
           "dmx_set_panel_mixed", "dmx_set_mode", "dmx_pack_words", "dmx_pack", "dmx_run", "dmx_load", "dmx_exec",
           "dmx_sync", "dmx_fetch", "dmx_counts", "dmx_stats", "dmx_device_count",
           "dmx_run_multi", "dmx_locate", "dmx_chop_set", "dmx_chop_exec", "dmx_chop_fetch",
           "dmx_chop_stats", "dmx_comm_unique_id", "dmx_comm_init_rank", "dmx_comm_init_all",
           "dmx_comm_size", "dmx_allreduce_counts", "dmx_debug_fetch", "dmx_run_sparse",
           "dmx_mask_exceptions", "dmx_host_register", "dmx_host_unregister", "dmx_panel_reach",
           "dmx_debug_bounds_selftest", "dmx_panel_pieces"]
ABI_VERSION = 4
COMM_ID_BYTES = 128

LOC_IGNORE_CASE, LOC_ONLY_POSITIVE = 0x1, 0x2
HIT_DTYPE = np.dtype([("seq", "<u8"), ("pattern", "<i4"), ("strand", "<i4"), ("start", "<i4"),
                      ("end", "<i4")])
assert HIT_DTYPE.itemsize == 24

# include/dmx.h dmx_chop_hit / dmx_chop_seg (pychopper-style reorientation)
CHOP_HIT_DTYPE = np.dtype([("read", "<u4"), ("label", "<i2"), ("dist", "<i2"), ("start", "<i4"),
                           ("stop", "<i4")])
CHOP_SEG_DTYPE = np.dtype([("read", "<u4"), ("start", "<i4"), ("stop", "<i4"),
                           ("strand", "<i2"), ("rule", "<i2")])
assert CHOP_HIT_DTYPE.itemsize == 16 and CHOP_SEG_DTYPE.itemsize == 16


# internal record layouts exposed by dmx_debug_fetch (csrc/dmx_device.h Window / Cand)
WINDOW_DTYPE = np.dtype([("item", "<u4"), ("o", "u1"), ("lastcol", "u1"), ("strand", "u1"),
                         ("bmin", "u1"), ("j1", "<u4"), ("j2", "<u4"), ("n", "<u4"),
                         ("start", "<u4"), ("len", "<u4"), ("info", "<u4"), ("off", "<u8")])
CAND_DTYPE = np.dtype([("item", "<u4"), ("sub", "<u2"), ("iend", "u1"), ("cost", "u1"),
                       ("j", "<u4"), ("n", "<u4"), ("start", "<u4"), ("len", "<u4"),
                       ("strand", "u1"), ("o", "u1"), ("a", "u1"), ("clean", "u1"), ("pad2", "<u4"),
                       ("off", "<u8")])
assert WINDOW_DTYPE.itemsize == 40 and CAND_DTYPE.itemsize == 40
DBG_WINDOWS, DBG_VERIFIED, DBG_TASKS, DBG_CANDS0, DBG_CANDS1, DBG_FLAGS = range(6)


class DmxError(RuntimeError):
    pass


_lib = None


def load() -> ctypes.CDLL:
    """Load libdmx.so (built by `make -C nanopore-barcoding-orc_amd`); raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise DmxError(f"{LIB_PATH} not built: run `make -C nanopore-barcoding-orc_amd` "
                       "(the HIP extension is required; there is no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    P, c_int, c_size, c_u64p = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p
    L.dmx_abi_version.restype = c_int
    L.dmx_open.argtypes = [c_int, ctypes.POINTER(P)]
    L.dmx_close.argtypes = [P]
    L.dmx_close.restype = None
    L.dmx_last_error.argtypes = [P]
    L.dmx_last_error.restype = ctypes.c_char_p
    L.dmx_set_panel.argtypes = [P, c_int, ctypes.POINTER(ctypes.c_char_p),
                                ctypes.POINTER(c_int), c_int, ctypes.c_double, c_int, c_int]
    L.dmx_set_panel_mixed.argtypes = [P, c_int, ctypes.POINTER(ctypes.c_char_p),
                                      ctypes.POINTER(c_int), ctypes.POINTER(c_int), c_int,
                                      ctypes.c_double, c_int, c_int]
    L.dmx_set_mode.argtypes = [P, c_int]
    L.dmx_pack_words.argtypes = [ctypes.c_uint64, c_size]
    L.dmx_pack_words.restype = c_size
    L.dmx_pack.argtypes = [P, c_u64p, P, c_size, P, P, c_u64p]
    L.dmx_run.argtypes = [P, P, P, c_u64p, P, c_size, c_size, P]
    L.dmx_load.argtypes = [P, P, P, c_u64p, P, c_size, c_size]
    L.dmx_exec.argtypes = [P]
    L.dmx_sync.argtypes = [P]
    L.dmx_fetch.argtypes = [P, P]
    L.dmx_counts.argtypes = [P, c_u64p, c_size]
    L.dmx_stats.argtypes = [P, ctypes.POINTER(ctypes.c_float), c_int, c_u64p, c_int,
                            ctypes.POINTER(c_int)]
    L.dmx_device_count.restype = c_int
    L.dmx_run_multi.argtypes = [ctypes.POINTER(P), c_int, P, P, c_u64p, P, c_size, c_size, P, c_u64p, c_size]
    L.dmx_locate.argtypes = [P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(c_int), c_int,
                             c_int, P, c_u64p, P, c_size, P, c_size,
                             ctypes.POINTER(ctypes.c_uint64)]
    L.dmx_chop_set.argtypes = [P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(c_int), c_int,
                               ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                               ctypes.POINTER(c_int), c_int, ctypes.c_double, c_int]
    L.dmx_chop_exec.argtypes = [P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    L.dmx_chop_fetch.argtypes = [P, P, P, P, c_size, P, c_size]
    L.dmx_chop_stats.argtypes = [P, ctypes.POINTER(ctypes.c_float), c_int]
    L.dmx_comm_unique_id.argtypes = [P]
    L.dmx_comm_init_rank.argtypes = [P, P, c_int, c_int]
    L.dmx_comm_init_all.argtypes = [ctypes.POINTER(P), c_int]
    L.dmx_comm_size.argtypes = [P]
    L.dmx_allreduce_counts.argtypes = [P, c_u64p, c_size]
    L.dmx_debug_fetch.argtypes = [P, c_int, c_int, P, c_size]
    L.dmx_run_sparse.argtypes = [P, P, P, P, c_size, c_u64p, P, c_size, c_size, P]
    L.dmx_mask_exceptions.argtypes = [P, c_size, P, P, c_size]
    L.dmx_mask_exceptions.restype = c_size
    L.dmx_host_register.argtypes = [P, c_size]
    L.dmx_host_unregister.argtypes = [P]
    if hasattr(L, "dmx_panel_reach"):
        L.dmx_panel_reach.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(c_int), P,
                                      c_int, ctypes.c_double, c_int, c_int, P, c_int]
        L.dmx_debug_bounds_selftest.argtypes = [P, P]
    if hasattr(L, "dmx_panel_pieces"):
        L.dmx_panel_pieces.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(c_int),
                                       c_int, ctypes.c_double, c_int, c_int, P, c_int, P, c_int]
    # DMX_ALLOW_ABI=1: load an older in-tree build for a regression A/B (tools/replay_sweep.py)
    if L.dmx_abi_version() != ABI_VERSION and os.environ.get("DMX_ALLOW_ABI") != "1":
        raise DmxError("libdmx ABI mismatch")
    _lib = L
    return L


class Packed:
    """A batch of reads in the device layout: 2-bit codes + no-match mask (see include/dmx.h)."""

    def __init__(self, seq2b: np.ndarray, nmask: np.ndarray, offsets: np.ndarray,
                 lengths: np.ndarray):
        self.seq2b, self.nmask, self.offsets, self.lengths = seq2b, nmask, offsets, lengths

    @property
    def n_reads(self) -> int:
        return int(len(self.lengths))

    def exceptions(self):
        """The no-match mask's nonzero words as (indices, values) (dmx_mask_exceptions)."""
        if getattr(self, "_exc", None) is None:
            L = load()
            n = L.dmx_mask_exceptions(self.nmask.ctypes.data, self.n_words, None, None, 0)
            idx = np.empty(max(n, 1), dtype=np.uint32)
            val = np.empty(max(n, 1), dtype=np.uint32)
            L.dmx_mask_exceptions(self.nmask.ctypes.data, self.n_words, idx.ctypes.data,
                                  val.ctypes.data, n)
            self._exc = (idx[:n], val[:n])
        return self._exc

    @property
    def n_words(self) -> int:
        return int(len(self.seq2b))


def pack(ascii_blob: np.ndarray, offsets: np.ndarray, lengths: np.ndarray) -> Packed:
    """Pack ASCII reads (uint8 blob + per-read offset/length) with the library's host packer."""
    L = load()
    blob = np.ascontiguousarray(ascii_blob, dtype=np.uint8)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = np.ascontiguousarray(lengths, dtype=np.uint32)
    n = len(lens)
    words = L.dmx_pack_words(int(lens.sum(dtype=np.uint64)), n)
    seq = np.empty(words, dtype=np.uint32)
    nm = np.empty(words, dtype=np.uint32)
    out_offs = np.empty(n, dtype=np.uint64)
    rc = L.dmx_pack(blob.ctypes.data if len(blob) else None, offs.ctypes.data, lens.ctypes.data,
                    n, seq.ctypes.data, nm.ctypes.data, out_offs.ctypes.data)
    if rc != 0:
        raise DmxError(f"dmx_pack failed ({rc})")
    return Packed(seq, nm, out_offs, lens)


class Context:
    """One device context (include/dmx.h: one per GPU, one host thread per context)."""

    def __init__(self, device: int = 0):
        self._L = load()
        h = ctypes.c_void_p()
        rc = self._L.dmx_open(int(device), ctypes.byref(h))
        if rc != 0:
            raise DmxError(f"dmx_open(device={device}) failed ({rc}): no usable HIP device")
        self._h = h
        self.device = device
        self.panel_sizes = [0, 0]
        self.mode = MODE_SINGLE

    def close(self):
        if getattr(self, "_h", None):
            self._L.dmx_close(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int, what: str) -> int:
        if rc < 0:
            msg = self._L.dmx_last_error(self._h)
            raise DmxError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
        return rc

    def set_panel(self, rnd: int, seqs, flags: int, max_errors: float = 0.1,
                  min_overlap: int = 3):
        arr = (ctypes.c_char_p * len(seqs))(*[s.encode("ascii") for s in seqs])
        lens = (ctypes.c_int * len(seqs))(*[len(s) for s in seqs])
        self._check(self._L.dmx_set_panel(self._h, rnd, arr, lens, len(seqs), float(max_errors),
                                          int(min_overlap), int(flags)), "dmx_set_panel")
        self.panel_sizes[rnd] = len(seqs)

    def set_panel_mixed(self, rnd: int, seqs, wheres, rc: bool, max_errors: float = 0.1,
                        min_overlap: int = 3):
        """Per-adapter DMX_FRONT / DMX_BACK (a cutadapt call mixing -g and -a)."""
        arr = (ctypes.c_char_p * len(seqs))(*[s.encode("ascii") for s in seqs])
        lens = (ctypes.c_int * len(seqs))(*[len(s) for s in seqs])
        wh = (ctypes.c_int * len(seqs))(*wheres)
        self._check(self._L.dmx_set_panel_mixed(self._h, rnd, arr, lens, wh, len(seqs),
                                                float(max_errors), int(min_overlap), int(rc)),
                    "dmx_set_panel_mixed")
        self.panel_sizes[rnd] = len(seqs)

    def bounds_selftest(self):
        """DMX_DEBUG_BOUNDS builds: (return code, message, the kernel's 3 outputs)."""
        out = np.zeros(3, dtype=np.uint32)
        rc = self._L.dmx_debug_bounds_selftest(self._h, out.ctypes.data)
        msg = self._L.dmx_last_error(self._h)
        return rc, (msg.decode() if msg else ""), out

    def set_mode(self, mode: int):
        self._check(self._L.dmx_set_mode(self._h, mode), "dmx_set_mode")
        self.mode = mode

    def run(self, p: Packed) -> np.ndarray:
        out = np.zeros(p.n_reads, dtype=RESULT_DTYPE)
        self._check(self._L.dmx_run(self._h, p.seq2b.ctypes.data, p.nmask.ctypes.data,
                                    p.offsets.ctypes.data, p.lengths.ctypes.data, p.n_words,
                                    p.n_reads, out.ctypes.data), "dmx_run")
        self._n_loaded = p.n_reads
        return out

    def run_sparse(self, p: Packed) -> np.ndarray:
        """dmx_run with the no-match mask uploaded as its exceptions (dmx_run_sparse)."""
        idx, val = p.exceptions()
        out = np.zeros(p.n_reads, dtype=RESULT_DTYPE)
        self._check(self._L.dmx_run_sparse(self._h, p.seq2b.ctypes.data, idx.ctypes.data,
                                           val.ctypes.data, len(idx), p.offsets.ctypes.data,
                                           p.lengths.ctypes.data, p.n_words, p.n_reads,
                                           out.ctypes.data), "dmx_run_sparse")
        self._n_loaded = p.n_reads
        return out

    def load(self, p: Packed):
        self._check(self._L.dmx_load(self._h, p.seq2b.ctypes.data, p.nmask.ctypes.data,
                                     p.offsets.ctypes.data, p.lengths.ctypes.data, p.n_words,
                                     p.n_reads), "dmx_load")
        self._n_loaded = p.n_reads

    def exec(self):
        self._check(self._L.dmx_exec(self._h), "dmx_exec")

    def sync(self):
        self._check(self._L.dmx_sync(self._h), "dmx_sync")

    def fetch(self) -> np.ndarray:
        out = np.zeros(self._n_loaded, dtype=RESULT_DTYPE)
        self._check(self._L.dmx_fetch(self._h, out.ctypes.data), "dmx_fetch")
        return out

    def locate(self, patterns, ascii_blob: np.ndarray, offsets: np.ndarray, lengths: np.ndarray,
               ignore_case: bool = False, only_positive: bool = False) -> np.ndarray:
        """Every exact IUPAC occurrence of every pattern (both strands unless only_positive):
        HIT_DTYPE records sorted as `seqkit locate` prints them — by record, then pattern, '+'
        hits by start, then '-' hits in the order a scan of the reverse complement meets them
        (descending positive-strand end)."""
        pats = [p.encode("ascii") if isinstance(p, str) else bytes(p) for p in patterns]
        arr = (ctypes.c_char_p * max(len(pats), 1))(*pats)
        pl = (ctypes.c_int * max(len(pats), 1))(*[len(p) for p in pats])
        blob = np.ascontiguousarray(ascii_blob, dtype=np.uint8)
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lengths, dtype=np.uint32)
        flags = (LOC_IGNORE_CASE if ignore_case else 0) | (LOC_ONLY_POSITIVE if only_positive
                                                           else 0)
        cap = max(1024, len(lens))
        while True:
            hits = np.zeros(cap, dtype=HIT_DTYPE)
            nh = ctypes.c_uint64()
            self._check(self._L.dmx_locate(self._h, arr, pl, len(pats), flags,
                                           blob.ctypes.data if len(blob) else None,
                                           offs.ctypes.data, lens.ctypes.data, len(lens),
                                           hits.ctypes.data, cap, ctypes.byref(nh)),
                        "dmx_locate")
            if nh.value <= cap:
                hits = hits[:nh.value]
                break
            cap = int(nh.value)
        key2 = np.where(hits["strand"] == 0, hits["start"].astype(np.int64),
                        -hits["end"].astype(np.int64))
        order = np.lexsort((key2, hits["strand"], hits["pattern"], hits["seq"]))
        return hits[order]

    # ---- pychopper-style reorientation (include/dmx.h dmx_chop_*) --------------
    def chop_set(self, primers, rules, cutoff: float, keep_primers: bool = True):
        """primers: IUPAC strings (label 2p = primer p, 2p+1 = its reverse complement);
        rules: [(left label, right label, strand 0 '+' / 1 '-')]; cutoff: maximum edit distance
        as a fraction of the primer length; keep_primers: pychopper -p."""
        seqs = [s.encode("ascii") for s in primers]
        arr = (ctypes.c_char_p * max(len(seqs), 1))(*seqs)
        lens = (ctypes.c_int * max(len(seqs), 1))(*[len(s) for s in seqs])
        nr = len(rules)
        rl = (ctypes.c_int * max(nr, 1))(*[int(r[0]) for r in rules])
        rr = (ctypes.c_int * max(nr, 1))(*[int(r[1]) for r in rules])
        rs = (ctypes.c_int * max(nr, 1))(*[int(r[2]) for r in rules])
        self._check(self._L.dmx_chop_set(self._h, arr, lens, len(seqs), rl, rr, rs, nr,
                                         float(cutoff), int(bool(keep_primers))), "dmx_chop_set")

    def chop_exec(self):
        """Hits and segments of the resident batch (after load); returns (n_hits, n_segs)."""
        nh, ns = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self._L.dmx_chop_exec(self._h, ctypes.byref(nh), ctypes.byref(ns)),
                    "dmx_chop_exec")
        self._chop_tot = (int(nh.value), int(ns.value))
        return self._chop_tot

    def chop_fetch(self, segs: bool = True, hits: bool = False):
        """(segments per read, hits per read, CHOP_SEG_DTYPE records, CHOP_HIT_DTYPE records),
        records in read order."""
        nh, ns = self._chop_tot
        n = getattr(self, "_n_loaded", 0)
        nseg = np.zeros(n, dtype=np.uint32)
        nhit = np.zeros(n, dtype=np.uint32)
        sg = np.zeros(ns if segs else 0, dtype=CHOP_SEG_DTYPE)
        ht = np.zeros(nh if hits else 0, dtype=CHOP_HIT_DTYPE)
        self._check(self._L.dmx_chop_fetch(self._h, nseg.ctypes.data if n else None,
                                           nhit.ctypes.data if n else None,
                                           sg.ctypes.data if len(sg) else None, len(sg),
                                           ht.ctypes.data if len(ht) else None, len(ht)),
                    "dmx_chop_fetch")
        return nseg, nhit, sg, ht

    def chop_stats(self):
        ms = (ctypes.c_float * 2)()
        nbig = self._check(self._L.dmx_chop_stats(self._h, ms, 2), "dmx_chop_stats")
        return {"chop": float(ms[0]), "order": float(ms[1]), "big_blocks": int(nbig)}

    def n_counts(self) -> int:
        a1 = 0 if self.mode == MODE_SINGLE else self.panel_sizes[1]
        return (self.panel_sizes[0] + 1) * (a1 + 1) + 2

    def counts(self) -> np.ndarray:
        out = np.zeros(self.n_counts(), dtype=np.uint64)
        self._check(self._L.dmx_counts(self._h, out.ctypes.data, len(out)), "dmx_counts")
        return out

    # ---- RCCL count exchange (include/dmx.h "Multi-GPU count exchange") -----------------------
    def comm_init_rank(self, comm_id: bytes, n_ranks: int, rank: int):
        """Join an n_ranks RCCL communicator (one process per GPU); comm_id from
        comm_unique_id() on rank 0.  Blocks until every rank has joined."""
        buf = ctypes.create_string_buffer(bytes(comm_id), COMM_ID_BYTES)
        with _stdout_to_stderr():
            rc = self._L.dmx_comm_init_rank(self._h, buf, int(n_ranks), int(rank))
        self._check(rc, "dmx_comm_init_rank")

    def comm_size(self) -> int:
        return self._check(self._L.dmx_comm_size(self._h), "dmx_comm_size")

    def allreduce_counts(self) -> np.ndarray:
        """Per-bin counts of the last exec summed over every rank (RCCL all-reduce in HBM on
        this context's stream; collective)."""
        out = np.zeros(self.n_counts(), dtype=np.uint64)
        self._check(self._L.dmx_allreduce_counts(self._h, out.ctypes.data, len(out)),
                    "dmx_allreduce_counts")
        return out

    def debug_fetch(self, what: int, rnd: int = 0) -> np.ndarray:
        """An intermediate list of the last exec (diagnostics: include/dmx.h dmx_debug_fetch)."""
        nb = self._check(self._L.dmx_debug_fetch(self._h, what, rnd, None, 0), "dmx_debug_fetch")
        buf = np.zeros(nb, dtype=np.uint8)
        self._check(self._L.dmx_debug_fetch(self._h, what, rnd, buf.ctypes.data if nb else None,
                                            nb), "dmx_debug_fetch")
        if what == DBG_FLAGS:
            return buf.view(np.uint32)
        return buf.view(CAND_DTYPE if what in (DBG_CANDS0, DBG_CANDS1) else WINDOW_DTYPE)

    def stats(self):
        ms = (ctypes.c_float * 17)()
        cl = np.zeros(14, dtype=np.uint64)
        fl = ctypes.c_int()
        self._check(self._L.dmx_stats(self._h, ms, 17, cl.ctypes.data, 14, ctypes.byref(fl)),
                    "dmx_stats")
        # filterN: the whole filter stage (with the piece screen, when on: piecesN is its part)
        names = ["scan0", "resolve0", "finalize0", "scan1", "resolve1", "finalize1", "total",
                 "filter0", "verify0", "filter1", "verify1", "screen0", "wscan0", "screen1",
                 "wscan1", "pieces0", "pieces1"]
        return {"ms": dict(zip(names, list(ms))), "clusters": cl[:2].tolist(),
                "windows": cl[2:4].tolist(), "resolved": cl[4:6].tolist(),
                "traces": cl[6:8].tolist(), "windows_raw": cl[8:10].tolist(),
                "tasks": cl[10:12].tolist(), "filter_tasks": cl[12:14].tolist(),
                "flags": fl.value}


def panel_reach(seqs, flags: int, max_errors: float = 0.1, min_overlap: int = 3,
                wheres=None):
    """Host only: (status, reach) of the panel dmx_set_panel would build — how far the kernels'
    gathers reach around a read view, in nt (include/dmx.h dmx_panel_reach)."""
    L = load()
    arr = (ctypes.c_char_p * len(seqs))(*[s.encode("ascii") for s in seqs])
    lens = (ctypes.c_int * len(seqs))(*[len(s) for s in seqs])
    wh = (ctypes.c_int * len(seqs))(*wheres) if wheres is not None else None
    out = np.zeros(6, dtype=np.int32)
    rc = L.dmx_panel_reach(arr, lens, wh, len(seqs), float(max_errors), int(min_overlap),
                           int(flags), out.ctypes.data, 6)
    return rc, dict(zip(["pre_raw", "pre", "post", "need_pre", "need_post", "guard"],
                        out.tolist()))


PIECE_FIELDS = ["step", "pieces", "keys", "entries", "front_reach", "part_max", "lo_off",
                "dlo_min"]


def panel_pieces(seqs, flags: int, max_errors: float = 0.1, min_overlap: int = 3):
    """Host only: (status, info, entries) of the piece screen dmx_set_panel would build
    (include/dmx.h dmx_panel_pieces).  entries: dicts of the packed (piece, offset) entries."""
    L = load()
    arr = (ctypes.c_char_p * len(seqs))(*[s.encode("ascii") for s in seqs])
    lens = (ctypes.c_int * len(seqs))(*[len(s) for s in seqs])
    out = np.zeros(8, dtype=np.int32)
    ent = np.zeros(4096, dtype=np.uint64)
    rc = L.dmx_panel_pieces(arr, lens, len(seqs), float(max_errors), int(min_overlap), int(flags),
                            out.ctypes.data, 8, ent.ctypes.data, len(ent))
    info = dict(zip(PIECE_FIELDS, out.tolist()))
    ents = []
    for v in ent[:info["entries"]].tolist():
        ents.append({"val": v & 0xFFFFFFFF, "len": (v >> 32) & 31, "o": (v >> 37) & 1,
                     "off": (v >> 38) & 3, "dlo": ((v >> 40) & 255) - 128,
                     "dhi": ((v >> 48) & 255) - 128})
    return rc, info, ents


def host_register(arrays) -> list:
    """Page-lock the given numpy arrays (upload sources); returns the registered ones."""
    L = load()
    done = []
    for a in arrays:
        if a.nbytes and L.dmx_host_register(a.ctypes.data, a.nbytes) == 0:
            done.append(a)
    return done


def host_unregister(arrays):
    L = load()
    for a in arrays:
        L.dmx_host_unregister(a.ctypes.data)


def device_count() -> int:
    """Visible HIP devices (0 without a GPU)."""
    return int(load().dmx_device_count())


@contextlib.contextmanager
def _stdout_to_stderr():
    """RCCL prints its version banner on stdout at initialisation; keep stdout for the callers'
    own output (bench.py's one JSON line, CLI reports)."""
    sys.stdout.flush()
    libc = ctypes.CDLL(None)
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        libc.fflush(None)
        os.dup2(saved, 1)
        os.close(saved)


def comm_unique_id() -> bytes:
    """A fresh RCCL communicator id (rank 0 draws it; every rank passes it to comm_init_rank)."""
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    with _stdout_to_stderr():
        rc = load().dmx_comm_unique_id(buf)
    if rc != 0:
        why = load().dmx_last_error(None)   # the context-free message (e.g. RCCL not loadable)
        raise DmxError(f"dmx_comm_unique_id failed ({rc}): "
                       f"{why.decode(errors='replace') if why else 'no message'}")
    return buf.raw


def comm_init_all(ctxs) -> bool:
    """One RCCL communicator over contexts on distinct devices (ncclCommInitAll); run_multi then
    sums its per-bin counts on the devices.  Returns False (no communicator) when contexts share
    a device, where RCCL cannot place two ranks."""
    if len({c.device for c in ctxs}) != len(ctxs):
        return False
    L = load()
    arr = (ctypes.c_void_p * len(ctxs))(*[c._h.value for c in ctxs])
    with _stdout_to_stderr():
        rc = L.dmx_comm_init_all(arr, len(ctxs))
    if rc < 0:
        msg = L.dmx_last_error(ctxs[0]._h)
        raise DmxError(f"dmx_comm_init_all failed ({rc}): {msg.decode() if msg else ''}")
    return True


def open_group(devices) -> list:
    """One context per device; contexts on distinct devices share one RCCL communicator
    (dmx_comm_init_all), so run_batch sums their per-bin counts on the GPUs over xGMI."""
    ctxs = [Context(d) for d in devices]
    if len(ctxs) > 1:
        try:
            comm_init_all(ctxs)
        except DmxError as e:   # dmx_run_multi then sums the shards' counts on the host
            print(f"dmx: RCCL communicator unavailable ({e}); per-bin counts are summed on the "
                  "host", file=sys.stderr)
    return ctxs


def run_batch(ctxs, p: Packed):
    """One packed batch on one or several contexts: (per-read results, per-bin counts).  With
    several contexts the batch is sharded by dmx_run_multi (counts all-reduced by RCCL when the
    contexts are one open_group communicator)."""
    if len(ctxs) == 1:
        res = ctxs[0].run(p)
        return res, ctxs[0].counts()
    return run_multi(ctxs, p)


def bin_totals(counts: np.ndarray, a0: int, a1: int) -> np.ndarray:
    """dmx_counts layout -> matrix [bin1 + 1, bin2 + 1] ((A0+1) x (A1+1); A1 = 0 in SINGLE mode;
    row/column 0 = no match)."""
    return np.asarray(counts[:(a0 + 1) * (a1 + 1)], dtype=np.int64).reshape(a0 + 1, a1 + 1)


def run_multi(ctxs, p: Packed):
    """Shard one packed batch over several contexts (one per GPU); returns (results, counts)."""
    L = load()
    if not ctxs:
        raise DmxError("run_multi needs at least one context")
    out = np.zeros(p.n_reads, dtype=RESULT_DTYPE)
    counts = np.zeros(ctxs[0].n_counts(), dtype=np.uint64)
    arr = (ctypes.c_void_p * len(ctxs))(*[c._h.value for c in ctxs])
    rc = L.dmx_run_multi(arr, len(ctxs), p.seq2b.ctypes.data, p.nmask.ctypes.data,
                         p.offsets.ctypes.data, p.lengths.ctypes.data, p.n_words, p.n_reads,
                         out.ctypes.data, counts.ctypes.data, len(counts))
    if rc < 0:
        msg = L.dmx_last_error(ctxs[0]._h)
        raise DmxError(f"dmx_run_multi failed ({rc}): {msg.decode() if msg else ''}")
    return out, counts
