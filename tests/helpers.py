"""Shared test helpers: expected cutadapt outputs rendered from the ORACLE's results."""
import gzip
import os

import numpy as np

import oracle
from dmx import fastx, panel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "nanopore-barcoding-orc_amd", "bin", "cutadapt")


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
        if b < 0:
            out.setdefault(-1, []).append((name[1:] if name.startswith("@") else name, seq,
                                           qual))
            continue
        if r["rc1"]:
            seq = fastx.revcomp(seq.encode()).decode()
            qual = qual[::-1]
            name = name + " rc"
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
