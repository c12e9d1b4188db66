"""FASTQ/FASTA layer of the CLI (CPU only)."""
import gzip

import numpy as np
import pytest

from dmx import cli, fastx, report, panel


def test_fastq_batches_and_render(tmp_path):
    p = tmp_path / "x.fastq.gz"
    recs = [(f"r{i} comment", "ACGTN" * (i % 7), "I" * (5 * (i % 7))) for i in range(1000)]
    with gzip.open(p, "wt") as fh:
        for h, s, q in recs:
            fh.write(f"@{h}\n{s}\n+\n{q}\n")
    got = []
    for b in fastx.read_batches(str(p), batch_bytes=997):   # tiny chunks: records straddle
        blob, offs, lens = b.seq_offsets()
        for i in range(len(b)):
            got.append((b.header(i).decode(), b.sequence(i).decode(), b.quality(i).decode()))
            assert bytes(blob[int(offs[i]):int(offs[i]) + int(lens[i])]) == b.sequence(i)
    assert got == recs
    b = next(fastx.read_batches(str(p)))
    r = fastx.render(b, 3, 1, 5, True, b" rc", False)
    seq = fastx.revcomp(recs[3][1].encode())[1:5]
    assert r == b"@r3 comment rc\n" + seq + b"\n+\n" + recs[3][2].encode()[::-1][1:5] + b"\n"


def test_fasta_multiline(tmp_path):
    p = tmp_path / "c.fasta"
    p.write_text(">a x\nACGT\nAC\n\n>b\nGG\n")
    b = next(fastx.read_batches(str(p)))
    assert [b.header(i) for i in range(2)] == [b"a x", b"b"]
    assert [b.sequence(i) for i in range(2)] == [b"ACGTAC", b"GG"]
    assert fastx.render(b, 0, 2, 6, False, b"", True) == b">a x\nGTAC\n"


def test_cli_rejects_unsupported(capsys):
    with pytest.raises(SystemExit):
        cli.run(["--action=mask", "-g", "ACGT", "-o", "x.fq", "in.fq"])
    with pytest.raises(SystemExit):
        cli.run(["-b", "ACGT", "-o", "x.fq", "in.fq"])


def test_report_schema():
    ads = [panel.Adapter("SP5_001", "ACGTACGTAC", "front")]
    st = report.Stats(ads)
    st.n_in, st.bp_in, st.n_out, st.bp_out, st.n_with_adapter = 10, 1000, 10, 900, 4
    st.matches[0] = 4
    st.add_match(0, False, "front", 12, 1)
    j = st.to_json(argv=["-g", "x"], cores=2, in_path="in.fq", error_rate=0.1)
    assert j["read_counts"]["read1_with_adapter"] == 4
    a = j["adapters_read1"][0]
    assert a["three_prime_end"] is None
    assert a["five_prime_end"]["trimmed_lengths"][0] == {"len": 12, "expect": 0.0,
                                                           "counts": [0, 1]}
