"""ctypes binding of libdmx_io.so (include/dmx_io.h): native FASTQ/FASTA(.gz) ingest + packing
and per-bin writers with parallel gzip.

The CLI's record path: `Reader` yields `NativeBatch`es (record spans + the packed device layout,
straight into `lib.Context.run`), `Sink` writes each read to its bin (or nowhere) with its trim
coordinates and orientation.  Replaces dnaio/xopen around cutadapt's per-read loop
(SURVEY.md §8f rank 1).  Like libdmx there is no Python fallback: a missing library raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .lib import DmxError, Packed

HERE = os.path.dirname(os.path.abspath(__file__))
# DMX_LIBDIR: an alternative build directory (host sanitizer builds: make sanitize)
IO_PATH = os.path.join(os.environ.get("DMX_LIBDIR") or HERE, "libdmx_io.so")
IO_EXPORTS = ["dmx_io_abi_version", "dmx_reader_open", "dmx_reader_next", "dmx_reader_error",
              "dmx_reader_close", "dmx_batch_free", "dmx_sink_open", "dmx_sink_write",
              "dmx_sink_close", "dmx_sink_error", "dmx_sink_free", "dmx_sink_write_rows",
              "dmx_batch_mean_qual", "dmx_io_gzip", "dmx_sink_retain", "dmx_io_retained_bytes",
              "dmx_io_drop_retained", "dmx_sink_retain_output", "dmx_reader_in_memory",
              "dmx_io_inflate", "dmx_sink_write_rows2", "dmx_batch_pack_views",
              "dmx_io_set_memory_budget"]


class _CBatch(ctypes.Structure):
    _fields_ = [("n_reads", ctypes.c_size_t), ("fasta", ctypes.c_int32), ("_pad", ctypes.c_int32),
                ("text", ctypes.c_void_p), ("head", ctypes.c_void_p),
                ("seqtext", ctypes.c_void_p), ("seq", ctypes.c_void_p),
                ("qual", ctypes.c_void_p), ("lens", ctypes.c_void_p),
                ("seq2b", ctypes.c_void_p), ("nmask", ctypes.c_void_p),
                ("offsets", ctypes.c_void_p), ("n_words", ctypes.c_size_t),
                ("total_nt", ctypes.c_uint64)]


_io = None


def load() -> ctypes.CDLL:
    global _io
    if _io is not None:
        return _io
    if not os.path.exists(IO_PATH):
        raise DmxError(f"{IO_PATH} not built: run `make -C nanopore-barcoding-orc_amd`")
    L = ctypes.CDLL(IO_PATH)
    P, c_int, c_size = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    L.dmx_io_abi_version.restype = c_int
    L.dmx_reader_open.argtypes = [ctypes.c_char_p, c_size, c_int, ctypes.POINTER(P)]
    L.dmx_reader_next.argtypes = [P, ctypes.POINTER(ctypes.POINTER(_CBatch))]
    L.dmx_reader_error.argtypes = [P]
    L.dmx_reader_error.restype = ctypes.c_char_p
    L.dmx_reader_close.argtypes = [P]
    L.dmx_reader_close.restype = None
    L.dmx_batch_free.argtypes = [ctypes.POINTER(_CBatch)]
    L.dmx_batch_free.restype = None
    L.dmx_sink_open.argtypes = [ctypes.POINTER(ctypes.c_char_p), c_int, c_int, c_int, c_int,
                                ctypes.POINTER(P)]
    L.dmx_sink_write.argtypes = [P, ctypes.POINTER(_CBatch), P, P, P, P, P]
    L.dmx_sink_write_rows.argtypes = [P, ctypes.POINTER(_CBatch), c_size, P, P, P, P, P, P]
    L.dmx_batch_mean_qual.argtypes = [ctypes.POINTER(_CBatch), P]
    L.dmx_sink_close.argtypes = [P, P, P]
    L.dmx_sink_error.argtypes = [P]
    L.dmx_sink_error.restype = ctypes.c_char_p
    L.dmx_sink_free.argtypes = [P]
    L.dmx_sink_free.restype = None
    L.dmx_io_gzip.argtypes = [ctypes.c_char_p, c_size, c_int, P, c_size, P]
    L.dmx_sink_retain.argtypes = [P, ctypes.c_uint64]
    L.dmx_io_retained_bytes.restype = ctypes.c_uint64
    L.dmx_io_drop_retained.restype = None
    L.dmx_sink_retain_output.argtypes = [P, c_int, c_int]
    L.dmx_reader_in_memory.argtypes = [P]
    L.dmx_reader_in_memory.restype = c_int
    L.dmx_io_inflate.argtypes = [ctypes.c_char_p, c_size, c_int, P, c_size, P]
    L.dmx_io_inflate.restype = c_int
    L.dmx_sink_write_rows2.argtypes = [P, ctypes.POINTER(_CBatch), c_size] + [P] * 9
    L.dmx_batch_pack_views.argtypes = [ctypes.POINTER(_CBatch), c_size, P, P, P, P, c_int,
                                       P, P, P, P, c_size]
    L.dmx_io_set_memory_budget.argtypes = [ctypes.c_uint64]
    L.dmx_io_set_memory_budget.restype = ctypes.c_uint64
    if L.dmx_io_abi_version() != 1:
        raise DmxError("libdmx_io ABI mismatch")
    L.dmx_io_set_memory_budget(int(memory_budget_bytes() or 0))
    _io = L
    return L


def gzip_member(data: bytes, level: int = 1) -> bytes:
    """One gzip member of `data` in the writers' format (dmx_io_gzip)."""
    L = load()
    cap = 2 * len(data) + 4096
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    if L.dmx_io_gzip(data, len(data), int(level), ctypes.addressof(out), cap,
                     ctypes.addressof(n)) != 0:
        raise DmxError("dmx_io_gzip failed")
    return out.raw[:n.value]


def _view(ptr, n, dtype):
    if n == 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    ct = np.ctypeslib.as_ctypes_type(np.dtype(dtype))
    return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ct)), shape=(n,))


class NativeBatch:
    """One batch of records owned by libdmx_io (numpy views valid until `free`)."""

    def __init__(self, ptr):
        self._ptr = ptr
        c = ptr.contents
        n = int(c.n_reads)
        self.n = n
        self.fasta = bool(c.fasta)
        self.lens = _view(c.lens, n, np.uint32)
        self.head = _view(c.head, 2 * n, np.uint64).reshape(n, 2)
        self.seq = _view(c.seq, 2 * n, np.uint64).reshape(n, 2)
        self.qual = None if self.fasta else _view(c.qual, 2 * n, np.uint64).reshape(n, 2)
        nw = int(c.n_words)
        self.packed = Packed(_view(c.seq2b, nw, np.uint32), _view(c.nmask, nw, np.uint32),
                             _view(c.offsets, n, np.uint64), self.lens)
        self.total_nt = int(c.total_nt)
        self._text, self._seqtext = c.text, c.seqtext

    def __len__(self):
        return self.n

    # record access (tests / small consumers; the CLI never loops over records in Python)
    def _bytes(self, base, a, b):
        return ctypes.string_at(base + int(a), int(b - a)) if b > a else b""

    def header(self, i) -> bytes:
        return self._bytes(self._text, *self.head[i])

    def sequence(self, i) -> bytes:
        return self._bytes(self._seqtext, *self.seq[i])

    def quality(self, i):
        return None if self.qual is None else self._bytes(self._text, *self.qual[i])

    def mean_qual(self) -> np.ndarray:
        """Per-read mean quality (pychopper -Q): -10 log10 of the mean error probability."""
        out = np.zeros(self.n, dtype=np.float64)
        rc = load().dmx_batch_mean_qual(self._ptr, out.ctypes.data if self.n else None)
        if rc != 0:
            raise ValueError("mean quality needs FASTQ input")
        return out

    def pack_views(self, read, start, stop, rc, threads: int = 0) -> Packed:
        """Views read[i][start[i]:stop[i]] (reverse-complemented where rc[i]) packed into the
        device layout as reads of their own (dmx_batch_pack_views): segments handed to the
        demultiplexer without rendering them."""
        from .lib import load as load_dmx
        arrs = [np.ascontiguousarray(read, np.uint32), np.ascontiguousarray(start, np.int32),
                np.ascontiguousarray(stop, np.int32), np.ascontiguousarray(rc, np.uint8)]
        n = len(arrs[0])
        if any(len(a) != n for a in arrs):
            raise ValueError("view arrays must have equal lengths")
        total = int((arrs[2].astype(np.int64) - arrs[1]).sum()) if n else 0
        words = int(load_dmx().dmx_pack_words(total, n))
        seq = np.empty(words, np.uint32)
        nm = np.empty(words, np.uint32)
        offs = np.empty(n, np.uint64)
        lens = np.empty(n, np.uint32)
        r = load().dmx_batch_pack_views(self._ptr, n, *[a.ctypes.data for a in arrs],
                                        int(threads), seq.ctypes.data, nm.ctypes.data,
                                        offs.ctypes.data, lens.ctypes.data, words)
        if r != 0:
            raise ValueError(f"dmx_batch_pack_views failed ({r})")
        return Packed(seq, nm, offs, lens)

    def free(self):
        if self._ptr is not None:
            load().dmx_batch_free(self._ptr)
            self._ptr = None
            self.packed = None


class Reader:
    """Batches of a FASTQ/FASTA(.gz) file ("-" = stdin), parsed and packed natively."""

    def __init__(self, path: str, batch_bytes: int = 256 << 20, threads: int = 0):
        self._L = load()
        h = ctypes.c_void_p()
        rc = self._L.dmx_reader_open(path.encode(), int(batch_bytes), int(threads),
                                     ctypes.byref(h))
        if rc != 0:
            raise OSError(f"cannot open {path}")
        self._h = h
        self.path = path

    @property
    def in_memory(self) -> bool:
        """The text comes from a retained sink output of this process (dmx_reader_in_memory)."""
        return bool(self._h) and bool(self._L.dmx_reader_in_memory(self._h))

    def __iter__(self):
        while True:
            b = self.next()
            if b is None:
                return
            yield b

    def next(self):
        p = ctypes.POINTER(_CBatch)()
        rc = self._L.dmx_reader_next(self._h, ctypes.byref(p))
        if rc != 0:
            msg = self._L.dmx_reader_error(self._h)
            raise ValueError(f"{self.path}: {msg.decode() if msg else 'read error'}")
        return NativeBatch(p) if p else None

    def close(self):
        if getattr(self, "_h", None):
            self._L.dmx_reader_close(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def retained_bytes() -> int:
    """Output text held for later readers (dmx_sink_retain)."""
    return int(load().dmx_io_retained_bytes())


def drop_retained():
    load().dmx_io_drop_retained()


def _read_int(path: str):
    try:
        with open(path) as fh:
            v = fh.read().strip()
        return None if v in ("", "max") else int(v)
    except (OSError, ValueError):
        return None


# Where the cgroup hierarchy is mounted and where this process's membership is listed (module
# attributes: tests point them at a fake tree).
CGROUP_ROOT = "/sys/fs/cgroup"
PROC_CGROUP = "/proc/self/cgroup"
_NO_LIMIT = 1 << 60   # v1 reports "unlimited" as a huge number


def _cgroup_memory_dirs():
    """(directory, limit file, usage file) of every memory cgroup this process is in, from its
    own cgroup up to the hierarchy's root: the v2 unified line "0::<path>" and the v1 "memory"
    controller line of /proc/self/cgroup.  A SLURM job without a cgroup namespace sits in a
    nested cgroup (…/job_N/step_M/…) whose limit the root files do not show; the root itself
    is always listed last (a container's own namespace shows "0::/")."""
    out = []
    try:
        with open(PROC_CGROUP) as fh:
            lines = fh.read().splitlines()
    except OSError:
        lines = []
    for line in lines:
        parts = line.split(":", 2)
        if len(parts) != 3:
            continue
        hid, ctrls, path = parts
        if hid == "0" and ctrls == "":
            root, files = CGROUP_ROOT, ("memory.max", "memory.current")
        elif "memory" in ctrls.split(","):
            root, files = os.path.join(CGROUP_ROOT, "memory"), ("memory.limit_in_bytes",
                                                                 "memory.usage_in_bytes")
        else:
            continue
        rel = [x for x in path.strip().strip("/").split("/") if x and x != ".."]
        for i in range(len(rel), -1, -1):
            d = os.path.join(root, *rel[:i])
            out.append((d, os.path.join(d, files[0]), os.path.join(d, files[1])))
    # without /proc/self/cgroup: the mount roots, as before
    out.append((CGROUP_ROOT, os.path.join(CGROUP_ROOT, "memory.max"),
                os.path.join(CGROUP_ROOT, "memory.current")))
    out.append((os.path.join(CGROUP_ROOT, "memory"),
                os.path.join(CGROUP_ROOT, "memory", "memory.limit_in_bytes"),
                os.path.join(CGROUP_ROOT, "memory", "memory.usage_in_bytes")))
    return out


def _budget_env_mb():
    """DMX_MEM_BUDGET_MB in MB: a number of MB, or with a SLURM-style suffix K, M, G or T
    (2048, 2048M, 2G, 1.5G); 0 or empty = unset.  Anything else raises DmxError naming the
    variable (it would otherwise surface as a bare ValueError on the first I/O call)."""
    raw = os.environ.get("DMX_MEM_BUDGET_MB", "").strip()
    if not raw:
        return None
    v = raw.upper().rstrip("B")
    scale = {"K": 1 / 1024, "M": 1, "G": 1024, "T": 1024 * 1024}
    mult = 1
    if v and v[-1] in scale:
        mult = scale[v[-1]]
        v = v[:-1]
    try:
        mb = int(float(v) * mult)
    except ValueError:
        raise DmxError(f"DMX_MEM_BUDGET_MB={raw!r}: expected MB, or a size such as 2048M or "
                       "2G") from None
    if mb < 0:
        raise DmxError(f"DMX_MEM_BUDGET_MB={raw!r}: must not be negative")
    return mb or None


def memory_budget_bytes():
    """The job's memory limit, which the readers' and writers' buffers are sized to
    (dmx_io_set_memory_budget, batch_bytes_for_budget): DMX_MEM_BUDGET_MB when set, else the
    smallest finite limit of the process's memory cgroups, from its own up to the root (v2
    memory.max, v1 limit_in_bytes; a SLURM job's --mem: 02_cutadapt_loop.sh runs under --mem=4G,
    01_pychopper.sh under 2G), else None (no limit)."""
    mb = _budget_env_mb()
    if mb:
        return mb << 20
    lims = [v for _, lim, _ in _cgroup_memory_dirs()
            for v in [_read_int(lim)] if v is not None and v < _NO_LIMIT]
    return min(lims) if lims else None


# fixed part of a process's peak: the HIP runtime holds ~0.9 GB of anonymous memory after its
# first device operations and pageable copies (tools/microbench/rss_hip.hip), plus the
# interpreter, numpy and the inflate / pool buffers; and the batch-sized buffers alive at once
# in the fused --reorient pipeline (reader queue, the batch in flight, the writers' render and
# compressed copies, the reoriented views): profiles/r5_rss_probe*.json
_FIXED_BYTES = 1300 << 20
_BATCHES_ALIVE = 20


def batch_bytes_for_budget(default: int = 256 << 20) -> int:
    """Reader batch size under memory_budget_bytes(): (budget - 1300 MB) / 20, 32 MB .. default
    (2G: 37 MB, 4G: 140 MB)."""
    b = memory_budget_bytes()
    if not b:
        return default
    return int(min(default, max(32 << 20, (b - _FIXED_BYTES) // _BATCHES_ALIVE)))


def peak_rss_mb() -> float:
    """This process's peak resident set (VmHWM, MB): what a SLURM job's --mem limit meets.
    0.0 where /proc is not readable."""
    try:
        with open("/proc/self/status") as fh:
            for line in fh:
                if line.startswith("VmHWM:"):
                    return int(line.split()[1]) / 1024
    except (OSError, ValueError, IndexError):
        pass
    return 0.0


def available_memory_bytes():
    """Memory this process can still take: the smallest of MemAvailable (/proc/meminfo) and, for
    every memory cgroup of the process from its own up to the root, the limit minus the usage
    (v2 memory.max / memory.current, or v1 limit / usage; a SLURM job's --mem lands in a nested
    one).  None when nothing is readable."""
    cands = []
    try:
        with open("/proc/meminfo") as fh:
            for line in fh:
                if line.startswith("MemAvailable:"):
                    cands.append(int(line.split()[1]) * 1024)
                    break
    except (OSError, ValueError, IndexError):
        pass
    for _, lim, cur in _cgroup_memory_dirs():   # every cgroup up to the root: the tightest
        limit, used = _read_int(lim), _read_int(cur)
        if limit is not None and used is not None and limit < _NO_LIMIT:
            cands.append(max(0, limit - used))
    mb = _budget_env_mb()
    if mb:   # a stated budget: what this process does not hold yet
        cands.append(max(0, (mb << 20) - _rss_bytes()))
    return min(cands) if cands else None


def rss_parts_mb() -> dict:
    """Current resident set by kind (MB): anonymous memory (what a cgroup limit cannot
    reclaim), file-backed pages (shared libraries, reclaimable) and shmem."""
    out = {}
    try:
        with open("/proc/self/status") as fh:
            for line in fh:
                k = line.split(":")[0]
                if k in ("RssAnon", "RssFile", "RssShmem"):
                    out[k] = int(line.split()[1]) / 1024
    except (OSError, ValueError, IndexError):
        pass
    return out


def _rss_bytes() -> int:
    try:
        with open("/proc/self/status") as fh:
            for line in fh:
                if line.startswith("VmRSS:"):
                    return int(line.split()[1]) * 1024
    except (OSError, ValueError, IndexError):
        pass
    return 0


def default_retain_bytes(cap_mb=None) -> int:
    """The resident server's round-2 cache cap: DMX_RETAIN_MB when set (0 disables), else a
    quarter of the memory still available to the process (cgroup limit or MemAvailable) and
    at most 8 GiB.  02_cutadapt_loop.sh runs under `#SBATCH --mem=4G`: retaining more than the
    job can hold would get the server OOM-killed in the middle of the loop."""
    env = os.environ.get("DMX_RETAIN_MB", "").strip() if cap_mb is None else str(cap_mb)
    if env:
        return max(0, int(env)) << 20
    avail = available_memory_bytes()
    if avail is None:
        return 0
    return int(min(8 << 30, avail // 4))


class Sink:
    """Outputs (created now) receiving records in input order; '.gz' paths are gzip members."""

    def __init__(self, paths, fasta_out: bool, level: int = 1, threads: int = 0,
                 retain_bytes: int = 0):
        """retain_bytes > 0: keep the gzip outputs' text in memory (up to that many bytes held
        in the process) for a later Reader of the same, unchanged files (dmx_sink_retain)."""
        self._L = load()
        self.paths = list(paths)
        arr = (ctypes.c_char_p * len(self.paths))(*[p.encode() for p in self.paths])
        h = ctypes.c_void_p()
        rc = self._L.dmx_sink_open(arr, len(self.paths), int(bool(fasta_out)), int(level),
                                   int(threads), ctypes.byref(h))
        self._h = h
        if rc != 0:
            msg = self._L.dmx_sink_error(h).decode() if h else "cannot open outputs"
            self._L.dmx_sink_free(h)
            self._h = None
            raise OSError(msg)
        self.n_written = self.bp_written = None
        if retain_bytes > 0:
            self._L.dmx_sink_retain(self._h, int(retain_bytes))

    def retain_output(self, o: int, keep: bool):
        """Include or exclude output o from retention (dmx_sink_retain_output)."""
        if self._L.dmx_sink_retain_output(self._h, int(o), int(bool(keep))) != 0:
            raise ValueError(f"no output {o}")

    def write(self, batch: NativeBatch, out_idx, start, stop, rc, n_rc):
        n = len(batch)
        arrs = [np.ascontiguousarray(out_idx, np.int32), np.ascontiguousarray(start, np.int32),
                np.ascontiguousarray(stop, np.int32), np.ascontiguousarray(rc, np.uint8),
                np.ascontiguousarray(n_rc, np.uint8)]
        for a in arrs:
            if len(a) != n:
                raise ValueError("per-read arrays must have one entry per read")
        r = self._L.dmx_sink_write(self._h, batch._ptr, *[a.ctypes.data for a in arrs])
        if r != 0:
            raise OSError(self._L.dmx_sink_error(self._h).decode())

    def write_rows(self, batch: NativeBatch, read, out_idx, start, stop, rc, name_mode):
        """Several records per read (include/dmx_io.h dmx_sink_write_rows): row r writes
        read[r][start[r]:stop[r]] (positions on the read as given; reverse-complemented if
        rc[r]) to output out_idx[r]; name_mode 1 names it "start:stop|id strand=+|- ..."."""
        arrs = [np.ascontiguousarray(read, np.uint32), np.ascontiguousarray(out_idx, np.int32),
                np.ascontiguousarray(start, np.int32), np.ascontiguousarray(stop, np.int32),
                np.ascontiguousarray(rc, np.uint8), np.ascontiguousarray(name_mode, np.uint8)]
        n = len(arrs[0])
        if any(len(a) != n for a in arrs):
            raise ValueError("row arrays must have equal lengths")
        r = self._L.dmx_sink_write_rows(self._h, batch._ptr, n, *[a.ctypes.data for a in arrs])
        if r != 0:
            raise OSError(self._L.dmx_sink_error(self._h).decode())

    def write_rows2(self, batch: NativeBatch, read, out_idx, start, stop, rc, name_start,
                    name_stop, name_strand, n_rc):
        """Rows named as segments "{name_start}:{name_stop}|id strand=..." plus n_rc " rc"
        suffixes (dmx_sink_write_rows2); the sequence is read[start:stop], reverse-complemented
        if rc (positions on the read as given)."""
        arrs = [np.ascontiguousarray(read, np.uint32), np.ascontiguousarray(out_idx, np.int32),
                np.ascontiguousarray(start, np.int32), np.ascontiguousarray(stop, np.int32),
                np.ascontiguousarray(rc, np.uint8), np.ascontiguousarray(name_start, np.int32),
                np.ascontiguousarray(name_stop, np.int32),
                np.ascontiguousarray(name_strand, np.uint8), np.ascontiguousarray(n_rc, np.uint8)]
        n = len(arrs[0])
        if any(len(a) != n for a in arrs):
            raise ValueError("row arrays must have equal lengths")
        r = self._L.dmx_sink_write_rows2(self._h, batch._ptr, n, *[a.ctypes.data for a in arrs])
        if r != 0:
            raise OSError(self._L.dmx_sink_error(self._h).decode())

    def close(self):
        if self._h is None:
            return
        n = np.zeros(len(self.paths), np.uint64)
        bp = np.zeros(len(self.paths), np.uint64)
        r = self._L.dmx_sink_close(self._h, n.ctypes.data, bp.ctypes.data)
        msg = self._L.dmx_sink_error(self._h).decode()
        self._L.dmx_sink_free(self._h)
        self._h = None
        self.n_written, self.bp_written = n, bp
        if r != 0:
            raise OSError(msg)

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.dmx_sink_free(self._h)
            self._h = None
