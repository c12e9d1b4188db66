"""FASTQ / FASTA I/O for the drop-in CLI (host side; plain or gzip).

Records are kept as views into one raw byte buffer per batch: sequence bytes are handed to
the packer by offset (no copy), headers/qualities are sliced only when a record is written.
Matches dnaio's conventions that cutadapt relies on: a FASTQ "name" is the whole header line
after '@' (a " rc" suffix is appended to it), qualities are reversed with the sequence.
"""
from __future__ import annotations

import gzip
import io
import zlib
from dataclasses import dataclass

import numpy as np

_COMP = bytes.maketrans(b"ACGTUMRWSYKVHDBNacgtumrwsykvhdbn", b"TGCAAKYWSRMBDHVNtgcaakywsrmbdhvn")


def revcomp(seq: bytes) -> bytes:
    return seq.translate(_COMP)[::-1]


def open_read(path: str):
    if path == "-":
        import sys
        return sys.stdin.buffer
    with open(path, "rb") as fh:
        magic = fh.read(2)
    if magic == b"\x1f\x8b":
        return gzip.open(path, "rb")
    return open(path, "rb")


@dataclass
class Batch:
    """A batch of records in one buffer; line spans are [start, end) offsets into buf."""
    buf: bytes
    arr: np.ndarray          # uint8 view of buf
    head: np.ndarray         # (n, 2) header span (without '>' / '@')
    seq: np.ndarray          # (n, 2) sequence span (FASTQ; FASTA sequences are re-assembled)
    qual: np.ndarray | None  # (n, 2) quality span, None for FASTA
    fasta: bool
    seq_blob: np.ndarray | None = None   # FASTA: concatenated sequences
    seq_off: np.ndarray | None = None

    def __len__(self):
        return len(self.head)

    def seq_offsets(self):
        """(blob, offsets, lengths) of the sequences for dmx.lib.pack."""
        if self.fasta:
            return self.seq_blob, self.seq_off, (self.seq[:, 1] - self.seq[:, 0]).astype(np.uint32)
        return self.arr, self.seq[:, 0].astype(np.uint64), \
            (self.seq[:, 1] - self.seq[:, 0]).astype(np.uint32)

    def header(self, i) -> bytes:
        return self.buf[self.head[i, 0]:self.head[i, 1]]

    def sequence(self, i) -> bytes:
        if self.fasta:
            o = int(self.seq_off[i])
            return self.seq_blob[o:o + int(self.seq[i, 1] - self.seq[i, 0])].tobytes()
        return self.buf[self.seq[i, 0]:self.seq[i, 1]]

    def quality(self, i) -> bytes | None:
        if self.qual is None:
            return None
        return self.buf[self.qual[i, 0]:self.qual[i, 1]]


def _strip_cr(arr, ends):
    e = ends.copy()
    m = (e > 0) & (arr[np.maximum(e - 1, 0)] == 13)
    e[m] -= 1
    return e


def _fastq_batch(buf: bytes) -> Batch:
    arr = np.frombuffer(buf, dtype=np.uint8)
    nl = np.flatnonzero(arr == 10)
    n = len(nl) // 4
    nl = nl[:4 * n]
    starts = np.empty(4 * n, dtype=np.int64)
    starts[0] = 0
    starts[1:] = nl[:-1] + 1
    ends = _strip_cr(arr, nl.astype(np.int64))
    st = starts.reshape(n, 4)
    en = ends.reshape(n, 4)
    if n and (arr[st[:, 0]] != ord("@")).any():
        raise ValueError("FASTQ record does not start with '@'")
    if n and (arr[st[:, 2]] != ord("+")).any():
        raise ValueError("FASTQ record third line does not start with '+'")
    head = np.stack([st[:, 0] + 1, en[:, 0]], axis=1)
    seq = np.stack([st[:, 1], en[:, 1]], axis=1)
    qual = np.stack([st[:, 3], en[:, 3]], axis=1)
    if n and ((qual[:, 1] - qual[:, 0]) != (seq[:, 1] - seq[:, 0])).any():
        raise ValueError("FASTQ sequence and quality lengths differ")
    return Batch(buf, arr, head, seq, qual, fasta=False)


def _fasta_batch(text: bytes) -> Batch:
    heads, seqs = [], []
    cur_h, cur = None, []
    for line in text.split(b"\n"):
        line = line.rstrip(b"\r")
        if line.startswith(b">"):
            if cur_h is not None:
                heads.append(cur_h)
                seqs.append(b"".join(cur))
            cur_h, cur = line[1:], []
        elif line.strip():
            if cur_h is None:
                raise ValueError("FASTA sequence before the first '>'")
            cur.append(line.strip())
    if cur_h is not None:
        heads.append(cur_h)
        seqs.append(b"".join(cur))
    buf = b"\n".join(heads)
    arr = np.frombuffer(buf, dtype=np.uint8) if buf else np.zeros(0, np.uint8)
    hs = np.zeros((len(heads), 2), dtype=np.int64)
    pos = 0
    for i, h in enumerate(heads):
        hs[i] = (pos, pos + len(h))
        pos += len(h) + 1
    lens = np.array([len(s) for s in seqs], dtype=np.int64)
    off = np.zeros(len(seqs), dtype=np.uint64)
    if len(seqs) > 1:
        off[1:] = np.cumsum(lens[:-1])
    blob = np.frombuffer(b"".join(seqs), dtype=np.uint8) if seqs else np.zeros(0, np.uint8)
    seq = np.stack([np.zeros(len(seqs), np.int64), lens], axis=1) if seqs else \
        np.zeros((0, 2), np.int64)
    return Batch(buf, arr, hs, seq, None, fasta=True, seq_blob=blob, seq_off=off)


def read_batches(path: str, batch_bytes: int = 256 << 20):
    """Yield Batch objects (FASTQ streamed in chunks of complete records; FASTA whole)."""
    fh = open_read(path)
    first = fh.read(1)
    if not first:
        return
    if first == b">":
        yield _fasta_batch(first + fh.read())
        return
    if first != b"@":
        raise ValueError(f"{path}: neither FASTQ nor FASTA")
    pending = first
    while True:
        chunk = fh.read(batch_bytes)
        data = pending + chunk
        if not chunk:
            if data.strip():
                if not data.endswith(b"\n"):
                    data += b"\n"
                yield _fastq_batch(data)
            return
        # cut after the last complete 4-line record
        arr = np.frombuffer(data, dtype=np.uint8)
        nl = np.flatnonzero(arr == 10)
        k = (len(nl) // 4) * 4
        if k == 0:
            pending = data
            continue
        cut = int(nl[k - 1]) + 1
        yield _fastq_batch(data[:cut])
        pending = data[cut:]


class Writer:
    """One output file; gzip when the name ends in .gz (cutadapt's xopen convention)."""

    def __init__(self, path: str, fasta: bool, level: int = 1):
        self.path, self.fasta, self.level = path, fasta, level
        self._raw = open(path, "wb")
        self._z = zlib.compressobj(level, zlib.DEFLATED, 31) if path.endswith(".gz") else None
        self.n = 0
        self.bp = 0

    def write_chunks(self, chunks: list):
        data = b"".join(chunks)
        if self._z is not None:
            data = self._z.compress(data)
        if data:
            self._raw.write(data)

    def close(self):
        if self._z is not None:
            self._raw.write(self._z.flush())
        self._raw.close()


def render(batch: Batch, i: int, start: int, stop: int, rc: bool, suffix: bytes,
           fasta_out: bool) -> bytes:
    """One output record: sequence[start:stop] of the (optionally reverse-complemented) read."""
    seq = batch.sequence(i)
    qual = batch.quality(i)
    if rc:
        seq = revcomp(seq)
        if qual is not None:
            qual = qual[::-1]
    seq = seq[start:stop]
    name = batch.header(i) + suffix
    if fasta_out or qual is None:
        return b">" + name + b"\n" + seq + b"\n"
    return b"@" + name + b"\n" + seq + b"\n+\n" + qual[start:stop] + b"\n"


def is_fasta_path(path: str) -> bool:
    p = path[:-3] if path.endswith(".gz") else path
    return p.endswith((".fa", ".fasta", ".fna", ".fas"))


__all__ = ["Batch", "Writer", "read_batches", "render", "revcomp", "is_fasta_path", "io"]
