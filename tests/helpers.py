"""Shared test helpers: expected cutadapt outputs rendered from the ORACLE's results."""
import gzip
import os

import numpy as np

import oracle
from dmx import fastx, panel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "nanopore-barcoding-orc_amd", "bin", "cutadapt")
LOOP = os.path.join(ROOT, "nanopore-barcoding-orc_amd", "bin", "dmx-demux-loop")


def write_fastq(path, names, seqs, quals):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "wt") as fh:
        for n, s, q in zip(names, seqs, quals):
            fh.write(f"@{n}\n{s}\n+\n{q}\n")


def read_fastq(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as fh:
        lines = fh.read().split("\n")
    return [tuple(lines[i:i + 4][:2] + [lines[i + 3]]) for i in range(0, len(lines) - 1, 4)]


def oracle_round(records, seqs_panel, where, rc):
    """One cutadapt invocation (oracle): returns {adapter index or -1: [(name, seq, qual)]}."""
    seqs = [r[1] for r in records]
    blob, offs, lens = oracle.pack_ascii(seqs)
    res = oracle.run_batch(oracle.Panel(seqs_panel, where), None, blob, offs, lens, mode=0,
                           use_rc=rc, threads=8)
    out = {}
    for (name, seq, qual), r in zip(records, res):
        b = int(r["bin1"])
        if r["rc1"]:   # also for an unmatched read taken reverse-complemented
            seq = fastx.revcomp(seq.encode()).decode()
            qual = qual[::-1]
            name = name + " rc"
        if b < 0:
            out.setdefault(-1, []).append((name[1:] if name.startswith("@") else name, seq,
                                           qual))
            continue
        if where == oracle.FRONT:
            s0, s1 = int(r["m1_rstop"]), len(seq)
        else:
            s0, s1 = 0, int(r["m1_rstart"])
        out.setdefault(b, []).append((name[1:] if name.startswith("@") else name,
                                      seq[s0:s1], qual[s0:s1]))
    return out


def random_quals(rng, lens):
    return ["".join(chr(33 + int(x)) for x in rng.integers(5, 41, size=L)) for L in lens]


def panel_seqs(path):
    return panel.load_panel(path)


_IUPAC = {"A": "A", "C": "C", "G": "G", "T": "T", "R": "AG", "Y": "CT", "S": "CG", "W": "AT",
          "K": "GT", "M": "AC", "B": "CGT", "D": "AGT", "H": "ACT", "V": "ACG", "N": "ACGT"}


def instantiate(rng, primer, err=0.06):
    """A sequenced copy of a degenerate primer: IUPAC codes resolved, then ONT-like edits."""
    out = []
    for c in primer:
        b = _IUPAC[c][int(rng.integers(len(_IUPAC[c])))]
        r = rng.random()
        if r < err * 0.6:
            out.append("ACGT"[int(rng.integers(4))])
        elif r < err * 0.8:
            pass
        elif r < err:
            out += [b, "ACGT"[int(rng.integers(4))]]
        else:
            out.append(b)
    return "".join(out)


def amplicon_reads(rng, pairs, n, body=(80, 700), flank=(0, 40)):
    """Consensus-like amplicons F + body + R (pairs = [(fwd, rev)], used as written, as the
    reference's `-g F...R`); ~10% miss the forward primer, ~10% the reverse, ~5% both, and a few
    carry a truncated primer at a read end."""
    seqs = []
    for _ in range(n):
        f, r = pairs[int(rng.integers(len(pairs)))]
        b = "".join(rng.choice(list("ACGT"), size=int(rng.integers(body[0], body[1] + 1))))
        u = rng.random()
        fs = "" if 0.10 <= u < 0.15 or u < 0.05 else instantiate(rng, f)
        rs = "" if 0.15 <= u < 0.25 or u < 0.05 else instantiate(rng, r)
        if rng.random() < 0.05 and fs:
            fs = fs[int(rng.integers(1, len(fs))):]
        if rng.random() < 0.05 and rs:
            rs = rs[:int(rng.integers(1, len(rs)))]
        lf = "".join(rng.choice(list("ACGT"), size=int(rng.integers(flank[0], flank[1] + 1))))
        rf = "".join(rng.choice(list("ACGT"), size=int(rng.integers(flank[0], flank[1] + 1))))
        seqs.append(lf + fs + b + rs + rf)
    return seqs


def oracle_linked(records, pairs):
    """One `cutadapt -g F...R [...] --untrimmed-output=U -o O` call (oracle): (trimmed, untrimmed)
    lists of (name, seq, qual-or-None); trimmed = read[front.rstop : front.rstop + back.rstart]."""
    seqs = [r[1] for r in records]
    blob, offs, lens = oracle.pack_ascii(seqs)
    res = oracle.run_batch(oracle.Panel([p[0] for p in pairs], oracle.FRONT),
                           oracle.Panel([p[1] for p in pairs], oracle.BACK),
                           blob, offs, lens, mode=2, use_rc=False, threads=8)
    trimmed, untrimmed = [], []
    for (name, seq, qual), r in zip(records, res):
        if int(r["bin1"]) < 0:
            untrimmed.append((name, seq, qual))
            continue
        s0 = int(r["m1_rstop"])
        s1 = s0 + int(r["m2_rstart"])
        trimmed.append((name, seq[s0:s1], qual[s0:s1] if qual is not None else None))
    return trimmed, untrimmed
