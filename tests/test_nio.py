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


@pytest.mark.parametrize("level", [1, 5, 9])
@pytest.mark.parametrize("fasta_out", [False, True])
def test_sink_matches_python_render(tmp_path, fasta_out, level):
    """Rendered records, inflated by Python's gzip (zlib) at -Z (1: Huffman-only members) and at
    cutadapt's default level 5 and at 9 (record-aware members, csrc/dmx_deflate.h fq_deflate)."""
    recs, text = _records(2500, seed=2)
    (tmp_path / "in.fq").write_text(text)
    rng = np.random.default_rng(5)
    n_out = 5
    ext = ".fasta" if fasta_out else ".fastq"
    paths = [str(tmp_path / f"o{k}{ext}.gz") if k % 2 == 0 else str(tmp_path / f"o{k}{ext}")
             for k in range(n_out)]
    expect = [[] for _ in range(n_out)]
    sink = nio.Sink(paths, fasta_out, level=level, threads=4)
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
    # the member header says which compressor wrote it (XFL 4 = fastest, 2 = best)
    assert open(paths[0], "rb").read()[8] == {1: 4, 5: 0, 9: 2}[level]


def test_default_level_is_cutadapts_and_smaller_than_z(tmp_path):
    """cutadapt 4.9's --compression-level default (5) is the drop-in's default; -Z (level 1) is
    Huffman-only.  At 5 the members (record-aware encoder) are no more than a few percent
    larger than zlib's level 5 on the same 1 MiB pieces of these short-header, random-quality
    records (and 10 % smaller on nanopore-style FASTQ: the test below), and smaller than at -Z."""
    from dmx import cli
    args = cli.build_parser().parse_args(["-g", "ACGT", "-o", "x.fq.gz", "in.fq"])
    assert args.compression_level == 5 and not args.zlevel1
    text = _records(3000, seed=8)[1].encode()
    pieces = [text[i:i + (1 << 20)] for i in range(0, len(text), 1 << 20)]
    z5 = sum(len(zlib.compress(p, 5)) for p in pieces)
    d5 = sum(len(nio.gzip_member(p, 5)) for p in pieces)
    d1 = sum(len(nio.gzip_member(p, 1)) for p in pieces)
    assert d5 < 1.05 * z5
    assert d5 < d1


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


def test_record_aware_gzip_members_inflate_with_zlib():
    """Levels >= 2 (csrc/dmx_deflate.h fq_deflate: LZ77 matches in header lines, sequence lines
    in blocks of their own) are standard gzip on every shape of text the writers can be handed
    or a member can be cut from: records cut mid-line at both ends, quality lines starting with
    '@' or '>' (not headers: they follow a lone "+"), "+name" separator lines, empty sequence
    lines, FASTA, headers longer than a match (258) repeated further apart than 4 KiB and
    than the 32 KiB window, non-FASTQ bytes, and short inputs."""
    import gzip
    import zlib
    rng = np.random.default_rng(11)

    def dna(n):
        return bytes(rng.choice(list(b"ACGT"), n).astype(np.uint8))

    def qual(n, first=None):
        q = bytes((rng.integers(2, 41, n) + 33).astype(np.uint8))
        return (first + q[1:]) if first and n else q

    long_head = b"@" + b"x" * 300 + b" runid=" + b"ab12" * 20
    recs = []
    for i in range(3000):
        n = int(rng.integers(0, 400)) if i % 7 else 0
        head = long_head + b" %d" % i if i % 5 == 0 else b"@read%d ch=%d runid=%s" % (
            i, i % 512, b"0f" * 20)
        sep = b"+" if i % 11 else b"+" + head[1:]
        recs.append(head + b"\n" + dna(n) + b"\n" + sep + b"\n" +
                    qual(n, first=b"@>"[i % 2:i % 2 + 1] if i % 3 == 0 else None) + b"\n")
    fq = b"".join(recs)
    far = b"".join(b"@" + b"h" * 40 + b"%d\n" % i + dna(20000) + b"\n+\n" + qual(20000) + b"\n"
                   for i in range(4))          # the previous header 40 kB back: no window match
    fa = b"".join(b">seq%d descr=abc%d\n%s\n" % (i, i % 9, dna(int(rng.integers(1, 300))))
                  for i in range(2000))
    cases = [b"A", b"@\n", b"@r\nAC\n+\nII\n", fq, fq[12345:612345], fa, fa[777:], far,
             rng.integers(0, 256, size=300_000, dtype=np.uint8).tobytes(),
             b"@same header line\n" * 40_000, fq * 2]
    for data in cases:
        for level in (5, 9):
            m = nio.gzip_member(data, level)
            assert zlib.decompress(m, 31) == data
        assert gzip.decompress(nio.gzip_member(data, 2)) == data
    assert nio.gzip_member(b"", 5) and gzip.decompress(nio.gzip_member(b"", 5)) == b""


def test_record_aware_level5_is_smaller_than_zlib_level5():
    """cutadapt's default --compression-level 5 (dmx/cli.py): on nanopore-style FASTQ
    (tests/fastq_like.py) the writers' 1 MiB members come out smaller than zlib -5's and
    libdeflate -5's (profiles/r5_gzip_levels.json: 2.32 vs 2.10 and 2.15 on 48 MB)."""
    import zlib

    from fastq_like import nanopore_fastq
    data = nanopore_fastq(3 << 20, seed=3)
    M = 1 << 20
    ours = sum(len(nio.gzip_member(data[k:k + M], 5)) for k in range(0, len(data), M))
    z5 = sum(len(zlib.compress(data[k:k + M], 5)) for k in range(0, len(data), M))
    assert ours < 0.95 * z5


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


def test_retain_plan_keeps_only_bins_read_back(tmp_path, monkeypatch):
    """the resident server retains only outputs a later call reads back — round 1's
    bins, not its `unknown` bin (02_cutadapt_loop.sh:79 skips it) and nothing of a call whose
    input came from the cache (round 2) — under a cap that fits the job's memory."""
    from dmx import cli
    recs, text = _records(3000, seed=6)
    src = tmp_path / "in.fastq"
    src.write_text(text)
    r1 = [str(tmp_path / f"SP5_{i}.fastq.gz") for i in range(2)] + [str(tmp_path / "unknown.fastq.gz")]
    nio.drop_retained()
    base = nio.retained_bytes()
    monkeypatch.setenv("DMX_RETAIN_MB", "64")

    def call(inp, outs, untrimmed):
        with nio.Reader(inp, 64 << 10, threads=4) as r:
            cap, keep = cli.retain_plan(outs, untrimmed, r.in_memory, True)
            s = nio.Sink(outs, False, 1, threads=4, retain_bytes=cap)
            for o, k in enumerate(keep):
                if cap and not k:
                    s.retain_output(o, False)
            sizes = np.zeros(len(outs), np.int64)
            for b in r:
                k = len(b)
                idx = (np.arange(k) % len(outs)).astype(np.int32)
                for o in range(len(outs)):
                    sel = idx == o
                    sizes[o] += sum(len(b.header(i)) + 2 * int(b.lens[i]) + 6
                                    for i in np.nonzero(sel)[0])
                s.write(b, idx, np.zeros(k, np.int32), b.lens.astype(np.int32),
                        np.zeros(k, np.uint8), np.zeros(k, np.uint8))
                b.free()
            s.close()
            return cap, keep, sizes, r.in_memory

    cap, keep, sizes, mem = call(str(src), r1, 2)          # round 1
    assert cap == 64 << 20 and keep == [True, True, False] and not mem
    held = nio.retained_bytes() - base
    assert held == sizes[0] + sizes[1]                       # the unknown bin is not held
    r2 = [str(tmp_path / f"SP27_{i}.fastq.gz") for i in range(3)]
    cap, keep, _, mem = call(r1[0], r2, 2)                   # round 2 reads SP5_0 from memory
    assert mem and cap == 0 and keep == [False] * 3
    assert nio.retained_bytes() - base == sizes[1]           # SP5_0 dropped, nothing new held
    nio.drop_retained()
    assert nio.retained_bytes() == base
    # outside the resident server nothing is retained; DMX_RETAIN_MB=0 disables
    assert cli.retain_plan(r1, 2, False, False)[0] == 0
    monkeypatch.setenv("DMX_RETAIN_MB", "0")
    assert cli.retain_plan(r1, 2, False, True)[0] == 0


def test_default_retain_cap_follows_available_memory(monkeypatch):
    monkeypatch.delenv("DMX_RETAIN_MB", raising=False)
    monkeypatch.setattr(nio, "available_memory_bytes", lambda: 4 << 30)   # e.g. --mem=4G
    assert nio.default_retain_bytes() == 1 << 30
    monkeypatch.setattr(nio, "available_memory_bytes", lambda: 1 << 40)
    assert nio.default_retain_bytes() == 8 << 30
    monkeypatch.setattr(nio, "available_memory_bytes", lambda: None)
    assert nio.default_retain_bytes() == 0
    monkeypatch.setenv("DMX_RETAIN_MB", "100")
    assert nio.default_retain_bytes() == 100 << 20
    monkeypatch.undo()
    avail = nio.available_memory_bytes()      # this container: MemAvailable and/or the cgroup
    assert avail is None or avail > 0


# ---------------------------------------------------------------------------------------------
# Parallel inflate of ordinary (unsized) gzip streams (csrc/dmx_inflate.h, ParGzSource): the
# input of 02_cutadapt_loop.sh is a single-member `pychopped_<ds>.gz` (:15,28-34,71).  Output
# must be byte-identical to zlib's inflate for stored, fixed and dynamic blocks, several members
# (members straddling chunk edges, empty members, zero padding), every header field, and chunk
# sizes small enough to put dozens of chunk edges into a few MB; corrupt input must fail.

def _inflate(data, threads, cap=None):
    import ctypes
    L = nio.load()
    cap = cap if cap is not None else max(1024, len(data) * 30 + (8 << 20))
    out = np.empty(cap, np.uint8)
    n = ctypes.c_size_t()
    r = L.dmx_io_inflate(data, len(data), threads, out.ctypes.data, cap, ctypes.byref(n))
    return r, out[:n.value].tobytes()


def _zcompress(text, level=6, strategy=0, sync_every=0, wbits=31):
    c = zlib.compressobj(level, zlib.DEFLATED, wbits, 9, strategy)
    if not sync_every:
        return c.compress(text) + c.flush()
    parts = []
    for i in range(0, len(text), sync_every):
        parts.append(c.compress(text[i:i + sync_every]))
        parts.append(c.flush(zlib.Z_SYNC_FLUSH if (i // sync_every) % 2 else zlib.Z_FULL_FLUSH))
    parts.append(c.flush())
    return b"".join(parts)


def _gzip_with_header_fields(text):
    """A member with FTEXT, FHCRC, FEXTRA, FNAME and FCOMMENT set (RFC 1952)."""
    import struct
    raw = zlib.compressobj(6, zlib.DEFLATED, -15)
    body = raw.compress(text) + raw.flush()
    extra = b"AB" + struct.pack("<H", 3) + b"xyz"
    hdr = bytes([0x1f, 0x8b, 8, 1 | 2 | 4 | 8 | 16, 0, 0, 0, 0, 0, 3])
    hdr += struct.pack("<H", len(extra)) + extra + b"name.fq\0" + b"a comment\0"
    hdr += struct.pack("<H", zlib.crc32(hdr) & 0xFFFF)
    return hdr + body + struct.pack("<II", zlib.crc32(text), len(text) & 0xFFFFFFFF)


@pytest.fixture(scope="module")
def fq_text():
    return _records(6000, seed=11)[1].encode()


@pytest.mark.parametrize("chunk_kb", ["16", "64", "4096"])
@pytest.mark.parametrize("threads", [1, 3, 8])
def test_parallel_inflate_single_member_levels(fq_text, monkeypatch, chunk_kb, threads):
    monkeypatch.setenv("DMX_INFLATE_CHUNK_KB", chunk_kb)
    for level in (1, 6, 9):
        gz = gzip.compress(fq_text, compresslevel=level)
        r, out = _inflate(gz, threads)
        assert r == 0 and out == fq_text, (level, r, len(out))


@pytest.mark.parametrize("threads", [1, 4])
def test_parallel_inflate_match_periods(monkeypatch, threads):
    """LZ77 copies of every period 1..40 (csrc/dmx_inflate.h copy_match: fill for distance 1,
    elementwise below one 16-byte word, whole words above; both the byte decoder and the
    speculative 16-bit one), with lengths up to 258 and matches ending at chunk edges."""
    monkeypatch.setenv("DMX_INFLATE_CHUNK_KB", "16")
    rng = np.random.default_rng(5)
    parts = []
    for rep in range(6):
        for period in range(1, 41):
            unit = rng.integers(65, 91, period, dtype=np.uint8).tobytes()
            parts.append(unit * int(rng.integers(1, 400 // period + 3)))
            parts.append(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes())
    text = b"".join(parts) * 3
    for level in (1, 6, 9):
        gz = gzip.compress(text, compresslevel=level)
        r, out = _inflate(gz, threads)
        assert r == 0 and out == text, (level, r, len(out))


@pytest.mark.parametrize("kind", ["fixed", "stored", "huffman", "rle", "sync", "random_bytes",
                                  "header_fields", "text_mixed"])
def test_parallel_inflate_block_kinds(fq_text, monkeypatch, kind):
    monkeypatch.setenv("DMX_INFLATE_CHUNK_KB", "16")
    text = fq_text
    if kind == "fixed":
        gz = _zcompress(text, 6, zlib.Z_FIXED)
    elif kind == "stored":
        gz = _zcompress(text, 0)
    elif kind == "huffman":
        gz = _zcompress(text, 6, zlib.Z_HUFFMAN_ONLY)
    elif kind == "rle":
        gz = _zcompress(text, 6, zlib.Z_RLE)
    elif kind == "sync":             # empty stored blocks (sync / full flush) every 50 KB
        gz = _zcompress(text, 6, 0, sync_every=50000)
    elif kind == "random_bytes":     # incompressible: zlib falls back to stored blocks
        text = np.random.default_rng(3).integers(0, 256, 600000, dtype=np.uint8).tobytes()
        text = text + fq_text[:300000] + text[:100000]
        gz = _zcompress(text, 6)
    elif kind == "header_fields":
        gz = _gzip_with_header_fields(text)
    else:                            # long repeats (distances up to 32 KiB, lengths 258)
        rep = fq_text[:40000]
        text = rep * 8 + fq_text + b"A" * 100000 + rep
        gz = _zcompress(text, 9)
    assert gzip.decompress(gz) == text
    for threads in (1, 4, 8):
        r, out = _inflate(gz, threads)
        assert r == 0 and out == text, (kind, threads, r, len(out), len(text))


@pytest.mark.parametrize("threads", [1, 5])
def test_parallel_inflate_members_straddle_chunks(fq_text, monkeypatch, threads):
    """Unsized members of random sizes (empty ones too), some separated by zero padding, so
    member boundaries fall anywhere relative to the 16 KiB chunk edges."""
    monkeypatch.setenv("DMX_INFLATE_CHUNK_KB", "16")
    rng = np.random.default_rng(9)
    cuts = np.sort(rng.integers(0, len(fq_text), 40))
    pieces = np.split(np.frombuffer(fq_text, np.uint8), cuts)
    gz = b""
    for i, p in enumerate(pieces + [np.zeros(0, np.uint8)]):
        gz += gzip.compress(p.tobytes(), compresslevel=int(rng.integers(1, 10)))
        if i % 7 == 3:
            gz += b"\0" * int(rng.integers(1, 20))
    r, out = _inflate(gz, threads)
    assert r == 0 and out == fq_text


def test_parallel_inflate_rejects_corrupt_input(fq_text, monkeypatch):
    monkeypatch.setenv("DMX_INFLATE_CHUNK_KB", "16")
    gz = bytearray(gzip.compress(fq_text, 6))
    bad_crc = bytes(gz[:-8]) + bytes([gz[-8] ^ 1]) + bytes(gz[-7:])
    bad_len = bytes(gz[:-4]) + bytes([gz[-4] ^ 1]) + bytes(gz[-3:])
    for data in (bad_crc, bad_len, bytes(gz[:len(gz) // 2]), bytes(gz[:-3]),
                 bytes(gz) + b"garbage!"):
        for threads in (1, 6):
            r, _ = _inflate(data, threads)
            assert r == -2, (threads, len(data))
    flipped = bytearray(gz)                    # a flipped bit inside the data
    flipped[len(gz) // 3] ^= 0x10
    for threads in (1, 6):
        assert _inflate(bytes(flipped), threads)[0] == -2
    # too small an output buffer is reported as such
    assert _inflate(bytes(gz), 4, cap=len(fq_text) - 1)[0] == -3
    # empty input and an empty member
    assert _inflate(b"", 4) == (0, b"")
    assert _inflate(gzip.compress(b""), 4) == (0, b"")


def test_reader_single_member_gzip_records(tmp_path, monkeypatch):
    """The reader's records from a Python-gzip single-member file equal the plain file's, with
    chunk edges every 16 KiB (parallel inflate) and with DMX_SEQ_INFLATE=1 (zlib)."""
    recs, text = _records(5000, seed=12)
    plain = tmp_path / "r.fastq"
    plain.write_text(text)
    gz = tmp_path / "r.fastq.gz"
    gz.write_bytes(gzip.compress(text.encode(), 6))

    def read_all(path):
        got = []
        with nio.Reader(str(path), 256 << 10, threads=4) as r:
            for b in r:
                got += [(b.header(i), b.sequence(i), b.quality(i)) for i in range(len(b))]
                b.free()
        return got
    ref = read_all(plain)
    monkeypatch.setenv("DMX_INFLATE_CHUNK_KB", "16")
    assert read_all(gz) == ref
    # inflate running ahead on its own thread in 8 KiB blocks, and on the reader's thread
    monkeypatch.setenv("DMX_INFLATE_AHEAD_KB", "8")
    assert read_all(gz) == ref
    monkeypatch.setenv("DMX_INFLATE_AHEAD", "0")
    assert read_all(gz) == ref
    monkeypatch.delenv("DMX_INFLATE_AHEAD")
    with nio.Reader(str(gz), 64 << 10, threads=4) as r:   # closed with inflate still ahead
        b = next(iter(r))
        assert b.header(0) == ref[0][0]
        b.free()
    monkeypatch.setenv("DMX_SEQ_INFLATE", "1")
    assert read_all(gz) == ref


def _revcomp(s: bytes) -> bytes:
    return s.translate(bytes.maketrans(b"ACGTUMRWSYKVHDBNacgtumrwsykvhdbn",
                                       b"TGCAAKYWSRMBDHVNtgcaakywsrmbdhvn"))[::-1]


@pytest.mark.parametrize("n_views,n_rate", [(1500, 0.01), (6000, 0.2)])
def test_pack_views_equals_packing_the_oriented_text(tmp_path, n_views, n_rate):
    """dmx_batch_pack_views (segments handed to the demultiplexer, the fused 01 -> 02 loop):
    the packed words, mask, offsets and lengths equal dmx_pack of the oriented view texts.
    The views are word copies of the batch's own packing (shifted, or reversed and complemented):
    N-rich reads and several threads' ranges too."""
    recs, text = _records(800, seed=21)
    rng = np.random.default_rng(4)
    lines = text.split("\n")   # some N in the sequence lines (line 2 of each record)
    for k in range(1, len(lines), 4):
        lines[k] = "".join("N" if rng.random() < n_rate else c for c in lines[k])
    text = "\n".join(lines)
    (tmp_path / "in.fq").write_text(text)
    with nio.Reader(str(tmp_path / "in.fq"), 64 << 20, threads=4) as r:
        b = r.next()
        n = len(b)
        lens = b.lens.astype(np.int64)
        read = rng.integers(0, n, n_views)
        a = (rng.random(n_views) * (lens[read] + 1)).astype(np.int64)
        z = a + (rng.random(n_views) * (lens[read] - a + 1)).astype(np.int64)
        rc = rng.integers(0, 2, n_views).astype(np.uint8)
        got = b.pack_views(read, a, z, rc, threads=4)
        views = []
        for i in range(n_views):
            s = b.sequence(int(read[i]))[a[i]:z[i]]
            views.append(_revcomp(s) if rc[i] else s)
        b.free()
    blob = np.frombuffer(b"".join(views), np.uint8)
    offs = np.concatenate([[0], np.cumsum([len(v) for v in views])[:-1]]).astype(np.uint64)
    exp = lib.pack(blob, offs, np.array([len(v) for v in views], np.uint32))
    assert got.offsets.tolist() == exp.offsets.tolist()
    assert got.lengths.tolist() == exp.lengths.tolist()
    assert np.array_equal(got.seq2b, exp.seq2b) and np.array_equal(got.nmask, exp.nmask)


def test_rows2_segment_names_with_rc_suffixes(tmp_path):
    """dmx_sink_write_rows2: the segment name of (name_start, name_stop, name_strand), n_rc " rc"
    suffixes, and read[start:stop] oriented by rc — the fused 01 -> 02 records."""
    recs, text = _records(300, seed=22)
    (tmp_path / "in.fq").write_text(text)
    out = str(tmp_path / "o.fq")
    rng = np.random.default_rng(5)
    s = nio.Sink([out], False, 1, threads=2)
    exp = []
    with nio.Reader(str(tmp_path / "in.fq")) as r:
        b = r.next()
        n = len(b)
        lens = b.lens.astype(np.int64)
        ns = (rng.random(n) * (lens + 1)).astype(np.int64)
        ne = ns + (rng.random(n) * (lens - ns + 1)).astype(np.int64)
        a = ns + (rng.random(n) * (ne - ns + 1)).astype(np.int64)
        z = a + (rng.random(n) * (ne - a + 1)).astype(np.int64)
        rc = rng.integers(0, 2, n).astype(np.uint8)
        nst = rng.integers(0, 2, n).astype(np.uint8)
        nrc = rng.integers(0, 3, n).astype(np.uint8)
        s.write_rows2(b, np.arange(n), np.zeros(n), a, z, rc, ns, ne, nst, nrc)
        for i in range(n):
            h = b.header(i).decode()
            rid, _, com = h.partition(" ")
            name = (f"{ns[i]}:{ne[i]}|{rid} strand={'-' if nst[i] else '+'}" +
                    (" " + com if com else "") + " rc" * int(nrc[i]))
            seq, q = b.sequence(i)[a[i]:z[i]], b.quality(i)[a[i]:z[i]]
            if rc[i]:
                seq, q = _revcomp(seq), q[::-1]
            exp.append(f"@{name}\n{seq.decode()}\n+\n{q.decode()}\n")
        b.free()
    s.close()
    assert open(out).read() == "".join(exp)


def test_memory_budget_sizes_the_buffers(monkeypatch):
    """A job's memory limit (DMX_MEM_BUDGET_MB, else the cgroup's) sizes the reader batches:
    (budget - 1300 MB) / 20 within 32..256 MB (nio.batch_bytes_for_budget; 02_cutadapt_loop.sh
    runs under --mem=4G, 01_pychopper.sh under 2G)."""
    monkeypatch.setenv("DMX_MEM_BUDGET_MB", "2048")
    assert nio.memory_budget_bytes() == 2048 << 20
    assert nio.batch_bytes_for_budget() == ((2048 - 1300) << 20) // 20
    monkeypatch.setenv("DMX_MEM_BUDGET_MB", "4096")
    assert nio.batch_bytes_for_budget() == ((4096 - 1300) << 20) // 20
    assert nio.batch_bytes_for_budget(64 << 20) == 64 << 20
    monkeypatch.setenv("DMX_MEM_BUDGET_MB", "1000")
    assert nio.batch_bytes_for_budget() == 32 << 20
    monkeypatch.setenv("DMX_MEM_BUDGET_MB", "100000")
    assert nio.batch_bytes_for_budget() == 256 << 20
    avail = nio.available_memory_bytes()
    assert avail is not None and avail <= 100000 << 20


def test_single_member_gzip_under_a_memory_budget(tmp_path):
    """Under a small budget the speculative inflate cuts 256 KiB chunks and the read-ahead blocks
    and buffer pools shrink (dmx_io_set_memory_budget); the records are the same."""
    import zlib
    L = nio.load()
    recs, text = _records(6000, seed=21)
    c = zlib.compressobj(6, zlib.DEFLATED, 31)
    (tmp_path / "one.fq.gz").write_bytes(c.compress(text.encode()) + c.flush())
    prev = L.dmx_io_set_memory_budget(64 << 20)
    try:
        assert _read_all(tmp_path / "one.fq.gz", batch_bytes=256 << 10, threads=4) == recs
    finally:
        L.dmx_io_set_memory_budget(prev)


def test_record_aware_gzip_random_documents():
    """Seeded random documents for fq_deflate: FASTQ/FASTA-shaped lines mixed with arbitrary
    ones, CRLF, '@' / '>' / '+' in odd places, long and empty lines, repeated headers at random
    distances, and cuts at random offsets; every member inflates with zlib to its input."""
    import zlib
    rng = np.random.default_rng(2024)
    alph = [b"ACGT", b"ACGTN", bytes(range(33, 75)), b"@>+\n\r ", bytes(range(256))]
    heads = [b"@" + bytes(rng.integers(33, 127, int(rng.integers(1, 400)), dtype=np.uint8))
             for _ in range(6)]
    for case in range(150):
        parts = []
        for _ in range(int(rng.integers(1, 120))):
            kind = int(rng.integers(0, 6))
            if kind == 0:
                parts.append(heads[int(rng.integers(len(heads)))] + b"%d\n" % int(rng.integers(1e6)))
            elif kind == 1:
                a = alph[int(rng.integers(0, 2))]
                parts.append(rng.choice(list(a), int(rng.integers(0, 3000))).astype(np.uint8)
                             .tobytes() + b"\n")
            elif kind == 2:
                parts.append(b"+\n" if rng.random() < 0.8 else b"+x\r\n")
            elif kind == 3:
                parts.append(rng.choice(list(alph[2]), int(rng.integers(0, 3000)))
                             .astype(np.uint8).tobytes() + b"\n")
            elif kind == 4:
                parts.append(rng.choice(list(alph[3]), int(rng.integers(0, 20)))
                             .astype(np.uint8).tobytes())
            else:
                parts.append(bytes(rng.integers(0, 256, int(rng.integers(0, 500)), dtype=np.uint8)))
        doc = b"".join(parts)
        if len(doc) > 10 and rng.random() < 0.5:
            a = int(rng.integers(0, len(doc)))
            doc = doc[a:a + int(rng.integers(1, len(doc) - a + 1))]
        level = int(rng.integers(2, 10))
        assert zlib.decompress(nio.gzip_member(doc, level), 31) == doc, (case, level)


def test_large_reads_take_the_parallel_paths(tmp_path):
    """Reads of >= 8 MB from a regular file go out as parallel preads, read-ahead blocks of
    >= 8 MB are copied to the batch by several threads, and single-member inflate rounds are
    sized to the read-ahead block (csrc/dmx_io.cpp FdSource, AheadSource, ParGzSource): a
    ~40 MB FASTQ, plain and as one zlib member, read with 4 threads and 16 MB batches gives
    the records in order."""
    import zlib
    rng = np.random.default_rng(31)
    recs = []
    parts = []
    i = 0
    while sum(map(len, parts)) < (40 << 20):
        n = int(rng.integers(200, 4000))
        s = rng.choice(list(b"ACGT"), n).astype(np.uint8).tobytes().decode()
        q = bytes((rng.integers(0, 41, n) + 33).astype(np.uint8)).decode()
        h = f"r{i} ch={i % 512}"
        recs.append((h, s, q))
        parts.append(f"@{h}\n{s}\n+\n{q}\n".encode())
        i += 1
    text = b"".join(parts)
    (tmp_path / "big.fastq").write_bytes(text)
    c = zlib.compressobj(1, zlib.DEFLATED, 31)
    (tmp_path / "big.fastq.gz").write_bytes(c.compress(text) + c.flush())
    for name in ("big.fastq", "big.fastq.gz"):
        assert _read_all(tmp_path / name, batch_bytes=16 << 20, threads=4) == recs, name


def _fake_cgroup(tmp_path, monkeypatch, proc_line, files):
    root = tmp_path / "cg"
    for rel, val in files.items():
        p = root / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(val)
    proc = tmp_path / "proc_cgroup"
    proc.write_text(proc_line + "\n")
    monkeypatch.setattr(nio, "CGROUP_ROOT", str(root))
    monkeypatch.setattr(nio, "PROC_CGROUP", str(proc))
    monkeypatch.delenv("DMX_MEM_BUDGET_MB", raising=False)


def test_memory_budget_from_a_nested_v2_cgroup(tmp_path, monkeypatch):
    """a SLURM step without a cgroup namespace sits in a nested cgroup; its job's
    --mem is the memory.max of an ancestor, which the mount root does not show."""
    job = "system.slice/slurmstepd.scope/job_5"
    _fake_cgroup(tmp_path, monkeypatch, f"0::/{job}/step_0/user/task_0", {
        f"{job}/memory.max": str(4 << 30), f"{job}/memory.current": str(1 << 30),
        f"{job}/step_0/memory.max": "max", f"{job}/step_0/memory.current": str(1 << 30),
        f"{job}/step_0/user/task_0/memory.max": "max",
        f"{job}/step_0/user/task_0/memory.current": str(1 << 30),
        "memory.current": str(9 << 30)})
    assert nio.memory_budget_bytes() == 4 << 30
    assert nio.available_memory_bytes() <= 3 << 30
    assert nio.batch_bytes_for_budget() == (int((4 << 30) - (1300 << 20)) // 20)


def test_memory_budget_from_a_nested_v1_cgroup(tmp_path, monkeypatch):
    _fake_cgroup(tmp_path, monkeypatch, "7:memory:/slurm/uid_1/job_7/step_batch", {
        "memory/memory.limit_in_bytes": "9223372036854771712",   # v1 "unlimited"
        "memory/slurm/uid_1/job_7/memory.limit_in_bytes": str(2 << 30),
        "memory/slurm/uid_1/job_7/memory.usage_in_bytes": str(512 << 20),
        "memory/slurm/uid_1/job_7/step_batch/memory.limit_in_bytes": "9223372036854771712"})
    assert nio.memory_budget_bytes() == 2 << 30
    assert nio.available_memory_bytes() <= (2 << 30) - (512 << 20)


def test_memory_budget_without_limits(tmp_path, monkeypatch):
    _fake_cgroup(tmp_path, monkeypatch, "0::/", {"memory.current": "1000"})
    assert nio.memory_budget_bytes() is None


@pytest.mark.parametrize("val,mb", [("2048", 2048), ("2048M", 2048), ("2G", 2048),
                                    ("1.5G", 1536), ("4096MB", 4096), ("0", None), ("", None)])
def test_memory_budget_env_sizes(monkeypatch, val, mb):
    monkeypatch.setenv("DMX_MEM_BUDGET_MB", val)
    if mb is None:
        monkeypatch.setattr(nio, "PROC_CGROUP", "/nonexistent")
        monkeypatch.setattr(nio, "CGROUP_ROOT", "/nonexistent")
        assert nio.memory_budget_bytes() is None
    else:
        assert nio.memory_budget_bytes() == mb << 20


def test_memory_budget_env_garbage_names_the_variable(monkeypatch):
    monkeypatch.setenv("DMX_MEM_BUDGET_MB", "lots")
    with pytest.raises(lib.DmxError, match="DMX_MEM_BUDGET_MB"):
        nio.memory_budget_bytes()
