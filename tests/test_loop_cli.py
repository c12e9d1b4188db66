"""CPU checks of the drop-in surfaces' argument handling (no GPU calls): the fused loop's
round-2 name template (north_star's {name1}_{name2} layout) and the CLI's refusal of
{name1}/{name2} on single-end input, which points at the loop's option."""
import os
import subprocess

from dmx import loop
from helpers import CLI


def test_round2_default_template_is_the_scripts_naming():
    # 02_cutadapt_loop.sh:100: -o demuxed/SP27/{name}_${identifier}_${dataset}.fastq.gz
    assert loop.round2_path("/o", loop.DEFAULT_TEMPLATE, "SP5_003", "SP27_007", "ds") == \
        "/o/SP27/SP27_007_SP5_003_ds.fastq.gz"
    assert loop.round2_path("/o", "{name1}_{name2}.fastq.gz", "SP5_003", "SP27_007", "ds") == \
        "/o/SP27/SP5_003_SP27_007.fastq.gz"
    assert loop.round2_path("/o", "{name1}/{name2}.fq", "SP5_1", "unknown", "x") == \
        "/o/SP27/SP5_1/unknown.fq"


def test_round2_template_must_name_every_bin_apart():
    assert loop.check_template(loop.DEFAULT_TEMPLATE) is None
    assert loop.check_template("{name1}_{name2}.fastq.gz") is None
    assert "both" in loop.check_template("{name1}.fastq.gz")
    assert "both" in loop.check_template("{name2}_{ds}.fastq.gz")
    assert "only" in loop.check_template("{name1}_{name2}_{sample}.fastq")
    assert "under" in loop.check_template("../{name1}_{name2}.fastq")
    assert "under" in loop.check_template("/tmp/{name1}_{name2}.fastq")


def test_cli_refuses_two_name_template_and_names_the_loop(tmp_path):
    fq = tmp_path / "in.fastq"
    fq.write_text("@r\nACGT\n+\nIIII\n")
    r = subprocess.run([CLI, "-g", "ACGTACGT", "-o", str(tmp_path / "{name1}_{name2}.fastq"),
                        str(fq)], capture_output=True, text=True,
                       env=dict(os.environ, DMX_DAEMON="0"))
    assert r.returncode == 2
    assert "dmx-demux-loop" in r.stderr and "--template" in r.stderr


def test_loop_closes_reader_and_contexts_when_setup_fails(tmp_path, monkeypatch):
    """the reader (and its producer thread) is opened before the device contexts;
    a failure in any later setup step (here the round-2 sink) must close the reader, every
    sink already open and every context, not leave the reader inflating in the background."""
    from dmx import lib, nio
    fq = tmp_path / "reads.fastq"
    fq.write_text("@r1\nACGTACGTACGT\n+\nIIIIIIIIIIII\n")
    events = []

    class FakeReader:
        def __init__(self, *a, **k):
            events.append("reader open")

        def close(self):
            events.append("reader close")

    class FakeCtx:
        def set_panel(self, *a, **k):
            pass

        def set_mode(self, *a):
            pass

        def close(self):
            events.append("ctx close")

    class FakeSink:
        n = 0

        def __init__(self, *a, **k):
            FakeSink.n += 1
            if FakeSink.n == 2:
                raise lib.DmxError("sink failed")
            events.append("sink open")

        def close(self):
            events.append("sink close")

    monkeypatch.setattr(nio, "Reader", FakeReader)
    monkeypatch.setattr(nio, "Sink", FakeSink)
    monkeypatch.setattr(lib, "open_group", lambda devs: [FakeCtx(), FakeCtx()])
    monkeypatch.setattr(loop, "_devices", lambda args: [0, 1])
    import pytest
    with pytest.raises(lib.DmxError, match="sink failed"):
        loop.run([str(fq), "--outdir", str(tmp_path / "out")])
    assert events.count("reader close") == 1
    assert events.count("ctx close") == 2
    assert events.count("sink close") == events.count("sink open") == 1
