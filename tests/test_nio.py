"""Native record I/O (libdmx_io, include/dmx_io.h) against the Python record layer (CPU only).

The Python reader/renderer in dmx/fastx.py restates dnaio/xopen's conventions in a few lines and
serves as the checker here; the CLI itself uses the native path."""
import gzip
import os
import re
import subprocess
import zlib

import numpy as np
import pytest

from dmx import fastx, lib, nio

ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__file__))


def _records(n, seed=0, crlf=False):
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(n):
        L = int(rng.integers(0, 400))
        s = "".join(rng.choice(list("ACGTNacgtRY"), L))
        q = "".join(chr(33 + int(x)) for x in rng.integers(0, 41, L))
        recs.append((f"read{i} runid=x ch={i % 7}", s, q))
    eol = "\r\n" if crlf else "\n"
    text = "".join(f"@{h}{eol}{s}{eol}+{eol}{q}{eol}" for h, s, q in recs)
    return recs, text


def test_io_library_exports_every_declared_symbol():
    hdr = open(f"{ROOT}/include/dmx_io.h").read()
    declared = set(re.findall(r"^\s*(?:int|void|const char\*|uint64_t)\s+(dmx_\w+)\(", hdr,
                              re.M))
    assert declared == set(nio.IO_EXPORTS)
    out = subprocess.run(["nm", "-D", "--defined-only", nio.IO_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert declared <= set(re.findall(r" T (dmx_\w+)", out))
    assert nio.load().dmx_io_abi_version() == 1


@pytest.mark.parametrize("kind", ["plain", "gz", "gz_members", "crlf"])
@pytest.mark.parametrize("batch_bytes", [1 << 16, 64 << 20])
def test_reader_matches_python_and_packer(tmp_path, kind, batch_bytes):
    recs, text = _records(3000, seed=1, crlf=(kind == "crlf"))
    data = text.encode()
    p = tmp_path / ("in.fastq.gz" if kind.startswith("gz") else "in.fastq")
    if kind == "gz":
        p.write_bytes(gzip.compress(data, 1))
    elif kind == "gz_members":   # pigz/bgzip-like: several members back to back
        cut = [0, len(data) // 3, len(data) // 2, len(data)]
        p.write_bytes(b"".join(gzip.compress(data[a:b], 6) for a, b in zip(cut, cut[1:])))
    else:
        p.write_bytes(data)
    got = []
    with nio.Reader(str(p), batch_bytes=batch_bytes, threads=4) as r:
        for b in r:
            ref = lib.pack(np.frombuffer(b"".join(b.sequence(i) for i in range(len(b))) or b"\0",
                                         np.uint8),
                           np.concatenate([[0], np.cumsum(b.lens[:-1], dtype=np.uint64)])
                           .astype(np.uint64) if len(b) else np.zeros(0, np.uint64), b.lens)
            assert np.array_equal(b.packed.offsets, ref.offsets)
            assert np.array_equal(b.packed.seq2b, ref.seq2b)
            assert np.array_equal(b.packed.nmask, ref.nmask)
            for i in range(len(b)):
                got.append((b.header(i).decode(), b.sequence(i).decode(), b.quality(i).decode()))
            b.free()
    assert got == recs


def test_reader_fasta_multiline_and_edge_cases(tmp_path):
    p = tmp_path / "c.fasta"
    p.write_text("\n>a x\nACGT \nAC\n\n>b\nGG\n>empty\n>last\r\nTT")
    with nio.Reader(str(p), batch_bytes=1 << 16) as r:
        bs = list(r)
    assert sum(len(b) for b in bs) == 4
    b = bs[0]
    assert [b.header(i) for i in range(4)] == [b"a x", b"b", b"empty", b"last"]
    assert [b.sequence(i) for i in range(4)] == [b"ACGTAC", b"GG", b"", b"TT"]
    assert b.quality(0) is None and b.fasta
    # big FASTA through several batches
    rng = np.random.default_rng(3)
    seqs = ["".join(rng.choice(list("ACGT"), int(rng.integers(1, 3000)))) for _ in range(500)]
    txt = "".join(f">s{i}\n" + "\n".join(s[k:k + 60] for k in range(0, len(s), 60)) + "\n"
                  for i, s in enumerate(seqs))
    (tmp_path / "m.fa.gz").write_bytes(gzip.compress(txt.encode()))
    out = []
    with nio.Reader(str(tmp_path / "m.fa.gz"), batch_bytes=1 << 16, threads=3) as r:
        for b in r:
            out += [b.sequence(i).decode() for i in range(len(b))]
    assert out == seqs


def test_reader_empty_and_errors(tmp_path):
    (tmp_path / "e.fq").write_bytes(b"")
    with nio.Reader(str(tmp_path / "e.fq")) as r:
        assert list(r) == []
    (tmp_path / "e.fq.gz").write_bytes(gzip.compress(b""))
    with nio.Reader(str(tmp_path / "e.fq.gz")) as r:
        assert list(r) == []
    for bad, msg in [(b"@a\nAC\n-\nII\n", "third line"), (b"@a\nAC\n+\nI\n", "lengths"),
                     (b"@a\nAC\n+\n", "truncated"), (b"xyz\n", "neither")]:
        (tmp_path / "b.fq").write_bytes(bad)
        with pytest.raises(ValueError, match=msg):
            with nio.Reader(str(tmp_path / "b.fq")) as r:
                list(r)
    (tmp_path / "t.fq.gz").write_bytes(gzip.compress(b"@a\nAC\n+\nII\n" * 1000)[:-20])
    with pytest.raises(ValueError, match="truncated gzip"):
        with nio.Reader(str(tmp_path / "t.fq.gz")) as r:
            list(r)
    with pytest.raises(OSError):
        nio.Reader(str(tmp_path / "missing.fq"))


@pytest.mark.parametrize("fasta_out", [False, True])
def test_sink_matches_python_render(tmp_path, fasta_out):
    recs, text = _records(2500, seed=2)
    (tmp_path / "in.fq").write_text(text)
    rng = np.random.default_rng(5)
    n_out = 5
    ext = ".fasta" if fasta_out else ".fastq"
    paths = [str(tmp_path / f"o{k}{ext}.gz") if k % 2 == 0 else str(tmp_path / f"o{k}{ext}")
             for k in range(n_out)]
    expect = [[] for _ in range(n_out)]
    sink = nio.Sink(paths, fasta_out, level=1, threads=4)
    pyb = list(fastx.read_batches(str(tmp_path / "in.fq"), batch_bytes=1 << 28))
    assert len(pyb) == 1
    pb = pyb[0]
    base = 0
    with nio.Reader(str(tmp_path / "in.fq"), batch_bytes=1 << 16) as r:
        for b in r:
            n = len(b)
            lens = b.lens.astype(np.int64)
            idx = rng.integers(-1, n_out - 1, n).astype(np.int32)   # last output stays empty
            a = (rng.random(n) * (lens + 1)).astype(np.int64)
            z = a + (rng.random(n) * (lens - a + 1)).astype(np.int64)
            rc = rng.integers(0, 2, n).astype(np.uint8)
            nrc = (rc + rng.integers(0, 2, n) * 2).astype(np.uint8)
            for i in range(n):
                if idx[i] >= 0:
                    expect[idx[i]].append(fastx.render(pb, base + i, int(a[i]), int(z[i]),
                                                       bool(rc[i]), b" rc" * int(nrc[i]),
                                                       fasta_out))
            sink.write(b, idx, a, z, rc, nrc)
            b.free()   # the sink keeps its own reference until the batch is written
            base += n
    sink.close()
    for k in range(n_out):
        raw = open(paths[k], "rb").read()
        if paths[k].endswith(".gz"):
            raw = gzip.decompress(raw)
        assert raw == b"".join(expect[k]), k
        assert int(sink.n_written[k]) == len(expect[k])
    assert len(expect[-1]) == 0 and gzip.decompress(open(paths[-1], "rb").read()) == b""


def test_sink_rejects_bad_coordinates(tmp_path):
    (tmp_path / "in.fq").write_text("@a\nACGT\n+\nIIII\n")
    sink = nio.Sink([str(tmp_path / "o.fq")], False)
    with nio.Reader(str(tmp_path / "in.fq")) as r:
        b = r.next()
        sink.write(b, [0], [1], [9], [0], [0])
        b.free()
    with pytest.raises(OSError, match="out of range"):
        sink.close()


def _bgzf(data: bytes, block: int = 60000) -> bytes:
    """BGZF (bgzip/htslib) blocks: gzip members with a 'BC' extra subfield = block size - 1."""
    import struct
    out = []
    for k in range(0, max(len(data), 1), block):
        chunk = data[k:k + block]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        raw = c.compress(chunk) + c.flush()
        hdr = b"\x1f\x8b\x08\x04" + b"\0" * 4 + b"\0\xff" + struct.pack("<H", 6) + b"BC" + \
            struct.pack("<HH", 2, 18 + len(raw) + 8 - 1)
        out.append(hdr + raw + struct.pack("<II", zlib.crc32(chunk), len(chunk)))
    return b"".join(out) + bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def _read_all(path, batch_bytes=1 << 20, threads=4):
    got = []
    with nio.Reader(str(path), batch_bytes=batch_bytes, threads=threads) as r:
        for b in r:
            got += [(b.header(i).decode(), b.sequence(i).decode(), b.quality(i).decode())
                    for i in range(len(b))]
            b.free()
    return got


@pytest.mark.parametrize("batch_bytes", [1 << 16, 1 << 20, 64 << 20])
def test_sized_members_parallel_inflate(tmp_path, batch_bytes):
    """Our writer's DX members (several per output: <= 4 MiB each), BGZF blocks, and a DX file
    followed by an ordinary member all read back exactly; the files are plain gzip to others."""
    recs, text = _records(30000, seed=4)
    (tmp_path / "in.fq").write_text(text)
    sink = nio.Sink([str(tmp_path / "dx.fq.gz")], False, level=1, threads=4)
    with nio.Reader(str(tmp_path / "in.fq"), batch_bytes=2 << 20) as r:
        for b in r:
            n = len(b)
            z = np.zeros(n, np.uint8)
            sink.write(b, np.zeros(n, np.int32), np.zeros(n, np.int32), b.lens.astype(np.int32),
                       z, z)
            b.free()
    sink.close()
    dx = (tmp_path / "dx.fq.gz").read_bytes()
    assert dx[12:14] == b"DX" and dx.count(b"\x1f\x8b\x08\x04") > 4
    assert gzip.decompress(dx) == text.encode()
    assert _read_all(tmp_path / "dx.fq.gz", batch_bytes) == recs
    (tmp_path / "b.fq.gz").write_bytes(_bgzf(text.encode()))
    assert gzip.decompress((tmp_path / "b.fq.gz").read_bytes()) == text.encode()
    assert _read_all(tmp_path / "b.fq.gz", batch_bytes) == recs
    extra, etext = _records(500, seed=6)
    (tmp_path / "mix.fq.gz").write_bytes(dx + gzip.compress(etext.encode()))
    assert _read_all(tmp_path / "mix.fq.gz", batch_bytes) == recs + extra


def test_sized_member_crc_mismatch_is_an_error(tmp_path):
    recs, text = _records(200, seed=7)
    blob = bytearray(_bgzf(text.encode(), block=10000))
    blob[200] ^= 0x40   # flip a bit inside the first block's deflate data
    (tmp_path / "bad.fq.gz").write_bytes(bytes(blob))
    with pytest.raises(ValueError):
        _read_all(tmp_path / "bad.fq.gz")


def test_huffman_gzip_members_inflate_with_zlib():
    """The writers' level-1 members (csrc/dmx_deflate.h: dynamic-Huffman blocks, no LZ77) are
    standard gzip: Python's zlib inflates them byte-exact, over block boundaries (256 KB),
    constant input, every byte value, one very rare byte (code lengths past 15 bits are
    flattened), empty input, and real FASTQ text; the reader inflates them too."""
    import gzip
    import zlib
    rng = np.random.default_rng(5)
    skew = rng.choice(256, size=600_000, p=np.r_[[0.5], np.full(255, 0.5 / 255)]).astype(np.uint8)
    rare = np.full(1 << 20, 65, np.uint8)
    rare[::3] = 67
    rare[12345] = 7                      # probability 1e-6: depth > 15 before flattening
    fib = np.repeat(np.arange(24, dtype=np.uint8),
                    [int(1.6 ** i) + 1 for i in range(24)])   # Fibonacci-like frequencies
    cases = [b"", b"A", b"AAAA" * 1000, bytes(range(256)) * 3000, skew.tobytes(),
             rare.tobytes(), rng.permutation(fib).tobytes(),
             rng.integers(0, 256, size=(1 << 20) + 17, dtype=np.uint8).tobytes(),
             b"@r1 x\nACGTN\n+\nIIII#\n" * 50_000]
    for data in cases:
        for level in (1, 6):
            m = nio.gzip_member(data, level)
            assert gzip.decompress(m) == data
            assert zlib.decompress(m, 31) == data
    fq = b"".join(b"@r%d\n%s\n+\n%s\n" % (i, b"ACGT" * (i % 50 + 1), b"I" * (4 * (i % 50 + 1)))
                  for i in range(20000))
    assert len(nio.gzip_member(fq, 1)) < 0.45 * len(fq)


def test_retained_outputs_read_back_without_the_file(tmp_path):
    """dmx_sink_retain (the resident server's round-2 cache, 02_cutadapt_loop.sh:91-103): a
    reader of an unchanged retained .gz output gets the same records from memory; a changed
    file (or a second read) goes to disk; the cap is honoured."""
    recs, text = _records(3000, seed=5)
    src = tmp_path / "in.fastq"
    src.write_text(text)
    outs = [str(tmp_path / f"bin{i}.fastq.gz") for i in range(3)]
    nio.drop_retained()
    base = nio.retained_bytes()

    def write_bins(retain):
        with nio.Reader(str(src), 64 << 10, threads=4) as r:
            s = nio.Sink(outs, False, 1, threads=4, retain_bytes=retain)
            for b in r:
                k = len(b)
                idx = (np.arange(k) % 3).astype(np.int32)
                s.write(b, idx, np.zeros(k, np.int32), b.lens.astype(np.int32),
                        (np.arange(k) % 2).astype(np.uint8), np.zeros(k, np.uint8))
                b.free()
            s.close()

    def read_all(path):
        got = []
        with nio.Reader(path, 64 << 10, threads=4) as r:
            for b in r:
                got += [(b.header(i), b.sequence(i), b.quality(i)) for i in range(len(b))]
                b.free()
        return got

    write_bins(0)
    ref = [read_all(p) for p in outs]       # from disk
    assert nio.retained_bytes() == base
    write_bins(1 << 30)
    held = nio.retained_bytes()
    assert held > 0
    assert read_all(outs[0]) == ref[0]      # from memory
    assert nio.retained_bytes() < held
    assert read_all(outs[0]) == ref[0]      # again: from disk
    os.utime(outs[1], ns=(1, 1))            # a changed file is read from disk
    assert read_all(outs[1]) == ref[1]
    assert read_all(outs[2]) == ref[2]
    assert nio.retained_bytes() == base
    write_bins(1000)                        # over the cap: nothing retained
    assert nio.retained_bytes() == base
    assert [read_all(p) for p in outs] == ref
    write_bins(1 << 30)
    nio.drop_retained()
    assert nio.retained_bytes() == base
