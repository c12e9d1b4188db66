"""pychopper-style read reorientation (scripts/01_pychopper.sh:45-57): libdmx's `dmx_chop_*`
(HIP) and the drop-in `bin/pychopper`, checked against the CPU restatement (oracle/chop_oracle.c
+ oracle/chopper.py).  Parity unpinned: pychopper v2.7.0 / edlib are not installed and the
reference ships no pychopper output."""
import os
import subprocess

import numpy as np
import pytest

import chopper as ochop
import oracle
from dmx import chop, lib, nio, panel, synth
from helpers import read_fastq, write_fastq

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "nanopore-barcoding-orc_amd", "bin", "pychopper")


def _ref_setup():
    primers = chop.load_primers(chop.PRIMERS_FASTA)
    with open(chop.CONFIG_FILE) as fh:
        text = fh.read()
    return primers, text


# ---- CPU ------------------------------------------------------------------------------------

def test_reference_primers_and_config():
    primers, text = _ref_setup()
    assert [p[0] for p in primers] == ["SP5", "SP27"]
    assert all(p[1].count("N") == 17 for p in primers)
    rules = chop.parse_config(text, ["SP5", "SP27"])
    assert rules == [(0, 3, 0), (2, 1, 1)]   # +:SP5,-SP27 | -:SP27,-SP5
    assert ochop.parse_config(text, ["SP5", "SP27"]) == rules


def test_oracle_c_dp_matches_python_dp():
    rng = np.random.default_rng(11)
    for _ in range(400):
        m = int(rng.integers(1, 12))
        pat = "".join(rng.choice(list("ACGTACGTRYSWKMN"), size=m))
        read = "".join(rng.choice(list("ACGTACGTACGTNacgt"), size=int(rng.integers(0, 50))))
        if rng.random() < 0.5 and len(read) > 2:   # plant an instance of the primer
            p = int(rng.integers(0, len(read)))
            inst = "".join(ochop._IUPAC[c][int(rng.integers(len(ochop._IUPAC[c])))] for c in pat)
            read = read[:p] + inst + read[p:]
        cutoff = float(rng.choice([0.0, 0.15, 0.3, 0.5, 0.9]))
        assert ochop.hits_c(pat, read, cutoff) == ochop.hits_py(pat, read, cutoff), (pat, read)


def _segments_brute(hits, rules, keep):
    """Every set of hit-disjoint candidates; the greatest summed length, ties -> the set that
    takes the earliest candidate where two sets first differ."""
    table = {}
    for r, (a, b, st) in enumerate(rules):
        table.setdefault((a, b), (r, st))
    cand = {}
    for i in range(len(hits) - 1):
        rs = table.get((hits[i][2], hits[i + 1][2]))
        if rs is not None:
            a = hits[i][0] if keep else hits[i][1]
            b = hits[i + 1][1] if keep else hits[i + 1][0]
            cand[i] = (a, max(a, b), rs[1], rs[0])
    best = None
    idx = sorted(cand)
    for mask in range(1 << len(idx)):
        pick = [idx[j] for j in range(len(idx)) if mask >> j & 1]
        if any(b - a < 2 for a, b in zip(pick, pick[1:])):
            continue
        key = (-sum(cand[i][1] - cand[i][0] for i in pick), [-(i in pick) for i in idx])
        if best is None or key < best[0]:
            best = (key, pick)
    return [cand[i] for i in best[1]] if best else []


def test_best_path_segments_match_brute_force():
    """Segment selection: hit-disjoint candidates of greatest summed length,
    ties to the earlier candidate, against an exhaustive search on random hit lists."""
    rng = np.random.default_rng(8)
    for _ in range(3000):
        nl = int(rng.integers(2, 7))
        rules = [(int(rng.integers(nl)), int(rng.integers(nl)), int(rng.integers(2)))
                 for _ in range(int(rng.integers(1, 6)))]
        hits = sorted({(int(a), int(a) + int(rng.integers(0, 30)), int(rng.integers(nl)), 0)
                       for a in rng.integers(0, 200, size=int(rng.integers(0, 11)))})
        keep = bool(rng.integers(2))
        got = ochop.segments(hits, rules, keep)
        exp = _segments_brute(hits, rules, keep)
        assert got == exp, (hits, rules, keep)


def test_best_path_prefers_the_longer_of_overlapping_pairs():
    # labels X=0, Y=1, Z=2; rules (X, Y) and (Y, Z): greedy pairing would take (X, Y)
    rules = [(0, 1, 0), (1, 2, 1)]
    hits = [(0, 10, 0, 0), (100, 110, 1, 0), (500, 510, 2, 0)]
    assert ochop.segments(hits, rules, True) == [(100, 510, 1, 1)]
    # equal lengths: the earlier candidate
    hits = [(0, 10, 0, 0), (100, 110, 1, 0), (200, 210, 2, 0)]
    assert ochop.segments(hits, rules, True) == [(0, 110, 0, 0)]
    # disjoint candidates are all taken (the reference layout's fused reads)
    primers, text = _ref_setup()
    r = chop.parse_config(text, ["SP5", "SP27"])
    hits = [(0, 58, 0, 3), (700, 758, 3, 2), (760, 818, 2, 1), (1500, 1558, 1, 4)]
    assert ochop.segments(hits, r, True) == [(0, 758, 0, 0), (760, 1558, 1, 1)]


def test_autotune_grid():
    g = chop.autotune_cutoffs()
    assert len(g) == 30 and g[0] == 0.1 and g[-1] == 0.6
    assert g == ochop.autotune_cutoffs()


def test_plan_rows_routes_in_input_order():
    nseg = np.array([0, 1, 2, 1, 0], np.uint32)
    segs = np.zeros(4, dtype=lib.CHOP_SEG_DTYPE)
    segs["read"] = [1, 2, 2, 3]
    segs["start"] = [0, 0, 40, 5]
    segs["stop"] = [100, 30, 200, 20]
    segs["strand"] = [0, 1, 0, 0]
    lens = np.array([150, 120, 250, 30, 10], np.uint32)
    qc = np.array([True, True, True, False, True])
    read, out, start, stop, rc, mode = chop.plan_rows(nseg, segs, lens, qc, 50, [0, 1, 2, 3, 4])
    assert read.tolist() == [0, 1, 2, 2, 3, 4]
    assert out.tolist() == [2, 0, 3, 1, 4, 2]
    assert start.tolist() == [0, 0, 0, 40, 0, 0]
    assert stop.tolist() == [150, 100, 30, 200, 30, 10]
    assert rc.tolist() == [0, 0, 1, 0, 0, 0]
    assert mode.tolist() == [0, 1, 1, 1, 0, 0]
    # outputs that are not written drop their rows
    read, out, *_ = chop.plan_rows(nseg, segs, lens, qc, 50, [0, -1, -1, 3, -1])
    assert read.tolist() == [1, 2] and out.tolist() == [0, 3]


def _fastq(tmp_path, rng, n=40):
    seqs = ["".join(rng.choice(list("ACGTN"), size=int(rng.integers(0, 90)))) for _ in range(n)]
    quals = ["".join(chr(33 + int(x)) for x in rng.integers(0, 42, size=len(s))) for s in seqs]
    names = [f"r{i}" + (f" runid=x ch={i}" if i % 2 else "") for i in range(n)]
    path = str(tmp_path / "in.fastq")
    write_fastq(path, names, seqs, quals)
    return path, names, seqs, quals


def test_native_mean_quality_matches_oracle(tmp_path):
    path, _, _, quals = _fastq(tmp_path, np.random.default_rng(2))
    with nio.Reader(path) as r:
        b = r.next()
        got = b.mean_qual()
        b.free()
    assert got.tolist() == [ochop.mean_qual(q) for q in quals]


def test_native_mean_quality_interleaved_chains(tmp_path):
    """dmx_batch_mean_qual sums four reads at a time in interleaved chains (each in read order):
    ragged and empty reads across several threads' ranges stay bit-exact with the oracle."""
    rng = np.random.default_rng(9)
    n = 9000
    lens = np.where(rng.random(n) < 0.05, 0, rng.integers(1, 400, n))
    seqs = ["A" * int(k) for k in lens]
    quals = ["".join(chr(33 + int(x)) for x in rng.integers(0, 60, size=int(k))) for k in lens]
    path = str(tmp_path / "q.fastq")
    write_fastq(path, [f"r{i}" for i in range(n)], seqs, quals)
    with nio.Reader(path) as r:
        b = r.next()
        got = b.mean_qual()
        b.free()
    assert got.tolist() == [ochop.mean_qual(q) for q in quals]


def test_sink_rows_render_segments(tmp_path):
    path, names, seqs, quals = _fastq(tmp_path, np.random.default_rng(3))
    out = str(tmp_path / "out.fastq")
    rows = []
    for i, s in enumerate(seqs):
        if len(s) >= 10:
            rows.append((i, 2, len(s) - 3, i % 2, 1))
            rows.append((i, 0, 5, 1 - i % 2, 1))
        else:
            rows.append((i, 0, len(s), 0, 0))
    with nio.Reader(path) as r:
        b = r.next()
        sink = nio.Sink([out], False)
        rd, a, z, rc, mode = (np.array(c) for c in zip(*rows))
        sink.write_rows(b, rd, np.zeros(len(rd), np.int32), a, z, rc, mode)
        sink.close()
        b.free()
    exp = []
    for i, a, z, rc, mode in rows:
        s, q = seqs[i][a:z], quals[i][a:z]
        if rc:
            s, q = ochop.revcomp(s), q[::-1]
        exp.append(("@" + (ochop.seg_name(names[i], a, z, rc) if mode else names[i]), s, q))
    assert read_fastq(out) == exp


# ---- GPU ------------------------------------------------------------------------------------

def _reads(rng, n):
    """Pre-pychopper ONT reads: SP5_i + insert + SP27rc_j on either strand (config 2's
    generator), plus fused reads (two amplicons), short and empty reads, N runs, and random
    padding that moves the primers across the kernel's 512-column segment boundaries."""
    d = synth.generate("c2", n=n, seed=int(rng.integers(1 << 30)))
    out = []
    for s in synth.to_strings(d):
        u = rng.random()
        if u < 0.10 and out:
            s = s + out[-1]
        elif u < 0.15:
            s = s[:int(rng.integers(0, 130))]
        elif u < 0.20:
            p = int(rng.integers(0, len(s)))
            s = s[:p] + "N" * int(rng.integers(1, 6)) + s[p:]
        elif u < 0.35:
            pad = int(rng.integers(380, 530))
            s = "".join(rng.choice(list("ACGT"), size=pad)) + s
        out.append(s)
    return out


def _gpu(ctx, seqs, primers, rules, cutoff, keep):
    blob, offs, lens = oracle.pack_ascii(seqs)
    ctx.load(lib.pack(blob, offs, lens))
    ctx.chop_set([p[1] for p in primers], rules, cutoff, keep)
    ctx.chop_exec()
    nseg, nhit, segs, hits = ctx.chop_fetch(hits=True)
    H = list(zip(*(hits[f].tolist() for f in ("read", "label", "dist", "start", "stop"))))
    S = list(zip(*(segs[f].tolist() for f in ("read", "start", "stop", "strand", "rule"))))
    return nseg, nhit, H, S


def _oracle(seqs, primers, rules, cutoff, keep):
    labs = ochop.labels(primers)
    H, S = [], []
    for r, s in enumerate(seqs):
        hs = ochop.read_hits(labs, s, cutoff)
        H += [(r, lab, d, a, b) for a, b, lab, d in hs]
        S += [(r, a, b, st, ri) for a, b, st, ri in ochop.segments(hs, rules, keep)]
    return H, S


@pytest.mark.gpu
@pytest.mark.parametrize("cutoff,keep", [(0.1, True), (0.2, True), (0.3, False)])
def test_chop_hits_and_segments_match_oracle(ctx, cutoff, keep):
    rng = np.random.default_rng(int(cutoff * 100))
    seqs = _reads(rng, 700)
    primers, text = _ref_setup()
    rules = chop.parse_config(text, [p[0] for p in primers])
    nseg, nhit, H, S = _gpu(ctx, seqs, primers, rules, cutoff, keep)
    eH, eS = _oracle(seqs, primers, rules, cutoff, keep)
    assert H == eH
    assert S == eS
    assert np.bincount([h[0] for h in eH], minlength=len(seqs)).tolist() == nhit.tolist()
    assert np.bincount([s[0] for s in eS], minlength=len(seqs)).tolist() == nseg.tolist()
    if cutoff <= 0.2:   # at 0.3 (k = 17 of 58) spurious hits break most reads' segments
        assert sum(1 for x in nseg if x == 1) > 0.5 * len(seqs)


@pytest.mark.gpu
def test_chop_random_primer_panels(ctx):
    """Random IUPAC primers (5..64 nt, up to 8 -> 16 labels), random rules and cutoffs, planted
    copies; short primers give many hits per read, overflowing the 64-read block's LDS hit list
    (redone by chop_big_kernel)."""
    rng = np.random.default_rng(23)
    for trial in range(8):
        npr = int(rng.integers(1, 9))
        lo = 5 if trial % 2 else 20
        primers = [(f"P{i}", "".join(rng.choice(list("ACGTACGTRYSWKMBDHVN"),
                                                size=int(rng.integers(lo, 65)))))
                   for i in range(npr)]
        nl = 2 * npr
        rules = [(int(rng.integers(nl)), int(rng.integers(nl)), int(rng.integers(2)))
                 for _ in range(int(rng.integers(0, 12)))]
        cutoff = float(rng.choice([0.0, 0.1] if trial % 2 else [0.0, 0.1, 0.2, 0.34, 0.45]))
        keep = bool(rng.integers(2))
        seqs = []
        for _ in range(160):
            s = "".join(rng.choice(list("ACGTACGTN" if rng.random() < 0.1 else "ACGT"),
                                   size=int(rng.integers(0, 1400))))
            for _ in range(int(rng.integers(0, 4))):
                lab = ochop.labels(primers)[int(rng.integers(nl))][1]
                inst = "".join(ochop._IUPAC[c][int(rng.integers(len(ochop._IUPAC[c])))]
                               for c in lab)
                p = int(rng.integers(0, len(s) + 1))
                s = s[:p] + inst + s[p:]
            seqs.append(s)
        _, _, H, S = _gpu(ctx, seqs, primers, rules, cutoff, keep)
        eH, eS = _oracle(seqs, primers, rules, cutoff, keep)
        assert H == eH, (trial, primers, cutoff)
        assert S == eS, (trial, rules)
    st = ctx.chop_stats()
    assert st["chop"] >= 0.0


@pytest.mark.gpu
def test_chop_reads_beyond_the_lds_hit_list(ctx):
    """Long tandem repeats of a primer (thousands of end locations at the least distance, 6-nt
    primers, one error allowed) overflow the 64-read block's 512-entry LDS hit list:
    chop_big_kernel redoes those blocks with global hit lists; the other blocks take the normal
    path."""
    rng = np.random.default_rng(41)
    primers = [(f"P{i}", "".join(rng.choice(list("ACGT"), size=6))) for i in range(8)]
    rules = [(0, 3, 0), (2, 1, 1), (4, 5, 0), (7, 6, 1)]

    def tandem(i):
        unit = primers[i % 8][1] + "".join(rng.choice(list("ACGT"), size=int(rng.integers(0, 3))))
        s = list(unit * (int(rng.integers(4000, 9000)) // len(unit)))
        for p in rng.integers(0, len(s), size=len(s) // 200):
            s[p] = "ACGT"[int(rng.integers(4))]
        return "".join(s)

    seqs = [tandem(i) if i % 3 == 0
            else "".join(rng.choice(list("ACGT"), size=int(rng.integers(0, 300))))
            for i in range(40)]
    for keep in (True, False):
        nseg, nhit, H, S = _gpu(ctx, seqs, primers, rules, 0.2, keep)
        eH, eS = _oracle(seqs, primers, rules, 0.2, keep)
        assert H == eH
        assert S == eS
        assert int(nhit.max()) > 512
        assert ctx.chop_stats()["big_blocks"] >= 1


@pytest.mark.gpu
def test_chop_fetch_after_new_load_is_refused(ctx):
    """A dmx_load replaces the resident batch, so the previous dmx_chop_exec's results are stale:
    dmx_chop_fetch must return DMX_E_STATE rather than copy the old batch's per-read counts into
    buffers sized for the new one."""
    rng = np.random.default_rng(5)
    primers, text = _ref_setup()
    rules = chop.parse_config(text, [p[0] for p in primers])
    _gpu(ctx, _reads(rng, 300), primers, rules, 0.1, True)
    blob, offs, lens = oracle.pack_ascii(_reads(rng, 20))
    ctx.load(lib.pack(blob, offs, lens))
    with pytest.raises(lib.DmxError, match=r"\(-5\)"):
        ctx.chop_fetch()
    ctx.chop_exec()
    nseg, _, _, _ = ctx.chop_fetch()
    assert len(nseg) == 20


def _records(rng, n):
    seqs = _reads(rng, n)
    quals = []
    for s in seqs:
        lo, hi = (2, 14) if rng.random() < 0.1 else (5, 41)
        quals.append("".join(chr(33 + int(x)) for x in rng.integers(lo, hi, size=len(s))))
    names = [f"r{i} runid=abc ch={i % 512}" for i in range(n)]
    return names, seqs, quals


@pytest.mark.gpu
@pytest.mark.parametrize("q", ["0.2", None])
def test_pychopper_dropin_matches_oracle(tmp_path, q):
    """scripts/01_pychopper.sh:45-57 verbatim (primers, config, -k LSK114 -Q 10 -p -m edlib,
    -w/-u/-l/-S, PASS on stdout), with -q given and autotuned."""
    names, seqs, quals = _records(np.random.default_rng(31), 1200)
    infile = str(tmp_path / "sample.fastq.gz")
    write_fastq(infile, names, seqs, quals)
    out = tmp_path / "pychopped"
    out.mkdir()
    paths = {k: str(out / f"sample_{k}.fastq") for k in ("rescued", "unclass", "short")}
    stats = str(out / "sample_stats.out")
    cmd = [BIN, "-b", chop.PRIMERS_FASTA, "-c", chop.CONFIG_FILE, "-k", "LSK114", "-Q", "10",
           "-w", paths["rescued"], "-u", paths["unclass"], "-l", paths["short"], "-S", stats,
           "-p", "-t", "4", "-m", "edlib", infile]
    if q:
        cmd[1:1] = ["-q", q]
    with open(out / "sample_pass.fastq", "wb") as fh:
        subprocess.run(cmd, stdout=fh, check=True)
    st = {}
    for line in open(stats).read().splitlines()[1:]:
        a, b, v = line.split("\t")
        st[(a, b)] = v
    cutoff = float(st[("Parameters", "cutoff")])
    primers, text = _ref_setup()
    records = list(zip(names, seqs, quals))
    if q:
        assert cutoff == float(q)
    else:
        assert cutoff == ochop.autotune(records, primers, text, keep=True, min_qual=10.0)
    exp = ochop.chop_records(records, primers, text, cutoff, keep=True, min_qual=10.0, min_len=50)
    fq = lambda recs: [("@" + h, s, qq) for h, s, qq in recs]  # noqa: E731
    assert read_fastq(str(out / "sample_pass.fastq")) == fq(exp["pass"])
    assert read_fastq(paths["rescued"]) == fq(exp["rescued"])
    assert read_fastq(paths["unclass"]) == fq(exp["unclass"])
    assert read_fastq(paths["short"]) == fq(exp["short"])
    assert int(st[("Reads", "Input")]) == len(seqs)
    assert int(st[("Classification", "QC_fail")]) == len(exp["qcfail"])
    assert int(st[("Classification", "Unusable")]) == len(exp["unclass"])
    assert len(exp["pass"]) > 0.6 * len(seqs)


@pytest.mark.gpu
def test_pychopper_fasta_and_empty_inputs(tmp_path):
    """FASTA input (no qualities: no QC, FASTA outputs) matches the oracle; an empty input still
    creates every output and reports cutoff NA."""
    names, seqs, _ = _records(np.random.default_rng(37), 300)
    fa = tmp_path / "in.fasta"
    fa.write_text("".join(f">{n}\n{s}\n" for n, s in zip(names, seqs)))
    out = {k: str(tmp_path / f"{k}.fasta") for k in ("rescued", "unclass", "short")}
    cmd = [BIN, "-b", chop.PRIMERS_FASTA, "-c", chop.CONFIG_FILE, "-q", "0.15", "-p",
           "-w", out["rescued"], "-u", out["unclass"], "-l", out["short"], "-m", "edlib", str(fa),
           str(tmp_path / "pass.fasta")]
    subprocess.run(cmd, check=True)
    primers, text = _ref_setup()
    exp = ochop.chop_records([(n, s, None) for n, s in zip(names, seqs)], primers, text, 0.15,
                             keep=True, min_len=50, fasta=True)

    def read_fa(path):
        lines = open(path).read().split("\n")
        return [(lines[i][1:], lines[i + 1]) for i in range(0, len(lines) - 1, 2)]

    assert read_fa(str(tmp_path / "pass.fasta")) == [(h, s) for h, s, _ in exp["pass"]]
    for k in ("rescued", "unclass", "short"):
        assert read_fa(out[k]) == [(h, s) for h, s, _ in exp[k]]
    empty = tmp_path / "empty.fastq"
    empty.write_text("")
    stats = tmp_path / "empty_stats.out"
    subprocess.run([BIN, "-b", chop.PRIMERS_FASTA, "-c", chop.CONFIG_FILE, "-u",
                    str(tmp_path / "e_unclass.fastq"), "-S", str(stats), str(empty),
                    str(tmp_path / "e_pass.fastq")], check=True)
    assert os.path.getsize(tmp_path / "e_pass.fastq") == 0
    assert os.path.exists(tmp_path / "e_unclass.fastq")
    assert "Parameters\tcutoff\tNA" in stats.read_text()


@pytest.mark.gpu
@pytest.mark.parametrize("q", ["0.2", None])
def test_fused_reorient_loop_equals_pychopper_then_loop(tmp_path, q):
    """01 -> 02 fused on the GPU (`dmx-demux-loop --reorient RAW`): pychopper's outputs and every
    02 output (records and reports) equal bin/pychopper (01_pychopper.sh:45-57) followed by
    dmx-demux-loop on its PASS file (02_cutadapt_loop.sh) — the PASS records are demultiplexed
    from the resident batch as oriented views, never written and read back.  Small batches put
    different batch edges in the two paths."""
    import glob
    import gzip
    import json
    import shutil
    from helpers import LOOP
    names, seqs, quals = _records(np.random.default_rng(32), 1500)
    two, fused = tmp_path / "two", tmp_path / "fused"
    for d in (two, fused):
        d.mkdir()
        write_fastq(str(d / "sample.fastq.gz"), names, seqs, quals)
    pych = two / "pychopped"
    pych.mkdir()
    cmd = [BIN, "-b", chop.PRIMERS_FASTA, "-c", chop.CONFIG_FILE, "-k", "LSK114", "-Q", "10",
           "-w", str(pych / "sample_rescued.fastq"), "-u", str(pych / "sample_unclass.fastq"),
           "-l", str(pych / "sample_short.fastq"), "-S", str(pych / "sample_stats.out"),
           "-p", "-t", "4", "-m", "edlib", "--batch-mb", "1", str(two / "sample.fastq.gz")]
    if q:
        cmd[1:1] = ["-q", q]
    with open(pych / "sample_pass.fastq", "wb") as fh:
        subprocess.run(cmd, stdout=fh, check=True)
    shutil.copy(pych / "sample_pass.fastq", pych / "pychopped_sample.fastq")   # 02's input
    subprocess.run([LOOP, str(pych / "pychopped_sample.fastq"), "-j", "4", "--batch-mb", "1"],
                   check=True, stdout=subprocess.DEVNULL)
    # with -q given the fused run takes other batch edges; the autotune (no -q) samples the
    # first batch's QC-passing reads (up to -Y), so there both runs read 1 MB batches
    fcmd = [LOOP, "--reorient", str(fused / "sample.fastq.gz"), "-j", "4", "--batch-mb",
            "2" if q else "1"]
    if q:
        fcmd += ["-q", q]
    subprocess.run(fcmd, check=True, stdout=subprocess.DEVNULL)
    for k in ("pass", "rescued", "unclass", "short"):
        a = (pych / f"sample_{k}.fastq").read_bytes()
        assert a == (fused / "pychopped" / f"sample_{k}.fastq").read_bytes(), k
    assert (pych / "sample_stats.out").read_text() == \
        (fused / "pychopped" / "sample_stats.out").read_text()
    outs = sorted(os.path.relpath(p, two / "demuxed")
                  for p in glob.glob(str(two / "demuxed" / "*" / "*")))
    assert outs == sorted(os.path.relpath(p, fused / "demuxed")
                          for p in glob.glob(str(fused / "demuxed" / "*" / "*")))
    assert sum(o.endswith(".fastq.gz") for o in outs) == 12 + 12 * 8
    n_rec = 0
    for o in outs:
        a, b = two / "demuxed" / o, fused / "demuxed" / o
        if o.endswith(".gz"):
            ta, tb = gzip.decompress(a.read_bytes()), gzip.decompress(b.read_bytes())
            assert ta == tb, o
            n_rec += ta.count(b"\n+\n")
        else:
            ja, jb = json.loads(a.read_text()), json.loads(b.read_text())
            for j in (ja, jb):
                j.pop("command_line_arguments")
                j.pop("input")
            assert ja == jb, o
    assert n_rec > 0.5 * len(seqs)


def _pychopper_cases():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "pychopper_cases", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(
            __file__))), "tools", "pychopper_cases.py"))
    pc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(pc)
    return pc


def test_unverified_pychopper_cases_tell_the_readings_apart():
    """Every [UNVERIFIED] pychopper switch (oracle/chopper.py RULES: autotune grid, autotune
    sample, autotune criterion, best-path score, record naming) has a case in
    tools/pychopper_cases.py whose outputs differ between the build's reading and the
    alternative one, so tools/parity_vs_pychopper.sh can settle each against a real
    pychopper v2.7.0; flipping one switch leaves the other cases' distinctions to their own."""
    pc = _pychopper_cases()
    assert set(v[0] for v in pc.CASES.values()) == set(ochop.DEFAULT_RULES)
    for name in pc.CASES:
        c = pc.build(name)
        a = pc.oracle_outputs(c)
        b = pc.oracle_outputs(c, {c["switch"]: ochop.ALT_RULES[c["switch"]]})
        assert a != b, name
        assert ochop.RULES == ochop.DEFAULT_RULES     # restored
        assert len(a["pass"]) + len(a["rescued"]) > 0, name


@pytest.mark.gpu
def test_unverified_pychopper_cases_match_the_default_readings(tmp_path):
    """The drop-in (bin/pychopper) on every [UNVERIFIED] case: outputs and tuned cutoff equal
    the oracle's default readings (what tools/parity_vs_pychopper.sh compares with a real
    pychopper v2.7.0)."""
    pc = _pychopper_cases()
    cases = tmp_path / "cases"
    pc.write(str(cases))
    for row in open(cases / "cases.tsv").read().splitlines():
        name, inp, opts = row.split("\t")
        o = tmp_path / name
        with open(f"{o}_pass.fastq", "wb") as fh:
            subprocess.run([BIN] + opts.split() + ["-w", f"{o}_rescued.fastq", "-u",
                                                   f"{o}_unclass.fastq", "-l", f"{o}_short.fastq",
                                                   "-S", f"{o}_stats.out", "-t", "4", inp],
                           stdout=fh, check=True, cwd=str(cases))
        exp = pc.oracle_outputs(pc.build(name))
        st = dict(((a, b), v) for a, b, v in (line.split("\t") for line in
                                              open(f"{o}_stats.out").read().splitlines()[1:]))
        assert float(st[("Parameters", "cutoff")]) == exp["cutoff"], name
        fq = lambda recs: [("@" + h, s, q) for h, s, q in recs]  # noqa: E731
        for k in ("pass", "rescued", "unclass", "short"):
            assert read_fastq(f"{o}_{k}.fastq") == fq(exp[k]), (name, k)
