"""cutadapt-style report (dmx/report.py) from per-read results, on CPU: the oracle's results stand
in for the GPU's (the GPU CLI tests check the device path against the same oracle).

Checked against quantities derived independently from the oracle's per-read matches: the
removed-length x errors histograms, the bases preceding removed 3' adapters, per-adapter totals;
plus the allowed-errors text of cutadapt's report for the reference panels' lengths."""
import io
import json
from collections import Counter

import numpy as np

import oracle
from dmx import cli, fastx, lib, loop, panel, report, synth

rng = np.random.default_rng(3)


def _revcomp(s: str) -> str:
    return fastx.revcomp(s.encode()).decode()


def test_allowed_errors_text_and_error_lengths():
    sp5 = panel.load_panel(panel.SP5_FASTA)[1][0]          # 59 nt
    sp27 = panel.load_panel(panel.SP27RC_FASTA)[1][0]      # 57 nt
    assert report.allowed_errors_text(sp5, 0.1) == \
        "1-9 bp: 0; 10-19 bp: 1; 20-29 bp: 2; 30-39 bp: 3; 40-49 bp: 4; 50-59 bp: 5"
    assert report.allowed_errors_text(sp27, 0.1) == \
        "1-9 bp: 0; 10-19 bp: 1; 20-29 bp: 2; 30-39 bp: 3; 40-49 bp: 4; 50-57 bp: 5"
    assert report.error_lengths(sp5, 0.1) == [10, 20, 30, 40, 50]
    assert report.error_lengths("ACGTACGTAC", 0.0) == []
    # absolute counts are per adapter; N wildcards do not count towards the length
    assert report.error_lengths("A" * 20, 2) == [10, 20]
    assert report.effective_length("ACGNNT") == 4 and report.effective_length("ACGT") == 4


def test_view_codes_match_string_indexing():
    seqs = ["".join(rng.choice(list("ACGTN" if i % 7 == 0 else "ACGT"),
                               size=int(rng.integers(0, 90)))) for i in range(300)]
    blob, offs, lens = oracle.pack_ascii(seqs)
    pk = lib.pack(blob, offs, lens)
    reads, strands, pos, exp = [], [], [], []
    for r, s in enumerate(seqs):
        for st in (0, 1):
            v = s if st == 0 else _revcomp(s)
            for p in (-1, 0, len(s) // 2, len(s) - 1):
                if p >= len(s):
                    continue
                reads.append(r)
                strands.append(st)
                pos.append(p)
                c = v[p] if p >= 0 else ""
                exp.append("ACGT".index(c) if c in ("A", "C", "G", "T") and c else 4)
    got = report.view_codes(pk, np.array(reads), np.array(strands), np.array(pos))
    assert got.tolist() == exp


def test_single_round_report_from_oracle_results():
    """cli._plan + Stats on a 3' panel with --rc: histogram, adjacency and totals vs the
    oracle's per-read matches taken apart by hand."""
    d = synth.generate("c1", n=600, seed=7)
    ads = [panel.Adapter(f"SP27_{i}", s, "back") for i, s in enumerate(d["sp27"])]
    seqs = [bytes(d["blob"][o:o + n]).decode() for o, n in zip(d["offsets"], d["lengths"])]
    res = oracle.run_batch(oracle.Panel(d["sp27"], oracle.BACK), None, d["blob"], d["offsets"],
                           d["lengths"], mode=0, use_rc=True, threads=4)
    stats = report.Stats(ads)
    stats.rc_mode = True
    pk = lib.pack(d["blob"], d["offsets"], d["lengths"])
    cli._plan(res, ads, False, True, len(ads), d["lengths"], stats, pk)
    hist, adj, tot = Counter(), Counter(), Counter()
    for s, r in zip(seqs, res):
        b = int(r["bin1"])
        if b < 0:
            continue
        v = _revcomp(s) if r["rc1"] else s
        rs = int(r["m1_rstart"])
        hist[(b, len(v) - rs, int(r["m1_errors"]))] += 1
        adj[(b, v[rs - 1] if rs > 0 and v[rs - 1] in "ACGT" else "")] += 1
        tot[b] += 1
    assert sum(tot.values()) > 200
    js = stats.to_json(argv=["-a", "file:x"], cores=1, in_path="in.fq", error_rate=0.1)
    for a, ent in enumerate(js["adapters_read1"]):
        assert ent["total_matches"] == tot[a]
        end = ent["three_prime_end"]
        assert ent["five_prime_end"] is None
        assert end["error_lengths"] == [10, 20, 30, 40, 50]
        assert end["matches"] == tot[a]
        assert end["adjacent_bases"] == {k: adj[(a, k)] for k in ("A", "C", "G", "T", "")}
        got = {(e["len"], k): c for e in end["trimmed_lengths"]
               for k, c in enumerate(e["counts"]) if c}
        assert got == {(L, e): c for (b, L, e), c in hist.items() if b == a}
    json.dumps(js)                                     # serialisable
    buf = io.StringIO()
    stats.summary(out=buf, error_rate=0.1)
    text = buf.getvalue()
    assert "=== Adapter SP27_0 ===" in text and "Bases preceding removed adapters:" in text
    assert "Overview of removed sequences" in text and "No. of allowed errors:" in text


def test_fused_round2_adjacency_matches_per_call_view():
    """loop._round_stats maps a round-2 match back onto the read (round-1 trim and both
    orientations) — same bases as indexing the round-1 output record directly."""
    d = synth.generate("c2", n=800, seed=9)
    seqs = [bytes(d["blob"][o:o + n]).decode() for o, n in zip(d["offsets"], d["lengths"])]
    res = oracle.run_batch(oracle.Panel(d["sp5"], oracle.FRONT), oracle.Panel(d["sp27"],
                           oracle.BACK), d["blob"], d["offsets"], d["lengths"], mode=1,
                           threads=4)
    ads1 = [panel.Adapter(n, s, "front") for n, s in zip(d["names1"], d["sp5"])]
    ads2 = [panel.Adapter(n, s, "back") for n, s in zip(d["names2"], d["sp27"])]
    st1 = report.Stats(ads1)
    st2 = [report.Stats(ads2) for _ in ads1]
    pk = lib.pack(d["blob"], d["offsets"], d["lengths"])
    (s1, e1, o1), (s2, e2, o2, nrc2) = loop.plan_rounds(res, d["lengths"])
    b1 = res["bin1"].astype(np.int64)
    b2 = res["bin2"].astype(np.int64)
    m1, m2 = b1 >= 0, b2 >= 0
    u2rc = ~m2 & (res["rc2"] == 1)
    s2w = np.where(m2, s2, np.where(u2rc, 0, s1))
    e2w = np.where(m2, e2, np.where(u2rc, e1 - s1, e1))
    loop._round_stats(st1, st2, res, d["lengths"], m1, m2, b1, b2, s1, s2w, e2w,
                      np.zeros(len(ads1), np.int64), np.zeros(len(ads1), np.int64), pk)
    exp = Counter()
    for s, r in zip(seqs, res):
        if r["bin1"] < 0 or r["bin2"] < 0:
            continue
        t1 = (_revcomp(s) if r["rc1"] else s)[int(r["m1_rstop"]):]
        v2 = _revcomp(t1) if r["rc2"] else t1
        rs = int(r["m2_rstart"])
        exp[(int(r["bin1"]), int(r["bin2"]), v2[rs - 1] if rs > 0 and v2[rs - 1] in "ACGT"
             else "")] += 1
    assert sum(exp.values()) > 300
    got = Counter()
    for i, st in enumerate(st2):
        for a, v in st.adjacent.items():
            for k, key in enumerate(report.ADJ_KEYS):
                if v[k]:
                    got[(i, a, key)] += int(v[k])
    assert got == exp
