"""One small case per pychopper choice the oracle marks [UNVERIFIED] (oracle/chopper.py RULES,
DESIGN.md §8d), built so that the build's reading and the alternative one give different
outputs.  tools/parity_vs_pychopper.sh runs every case through a real pychopper v2.7.0 (where one
is installed) and through the drop-in (bin/pychopper) and diffs the outputs: a DIFF names the
switch to flip.  tests/test_chop.py checks, with oracle/chopper.py switched to each alternative
reading, that every case really tells the readings apart, and (GPU) that the drop-in gives the
build's readings.

The reads come from seeded generators; the seeds were found by `--search` (the first seed whose
outputs differ between the readings).  The reference's own settings (01_pychopper.sh:45-57: -Q 10
-p -m edlib, autotuned -q) reach every switch.

Usage: python tools/pychopper_cases.py DIR   (writes DIR/<case>.fastq, DIR/<case>_primers.fa,
DIR/<case>_config.txt and DIR/cases.tsv: case, input, pychopper options; the outputs of case C
are @OUT@/C_{pass,rescued,unclass,short}.fastq and @OUT@/C_stats.out)
       python tools/pychopper_cases.py --search   (re-derive the seeds)
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "nanopore-barcoding-orc_amd"), os.path.join(ROOT, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

REF_PRIMERS = os.path.join(ROOT, "nanopore-barcoding-orc_amd", "dmx", "data",
                           "M13_seqs_for_pychopper.fa")
REF_CONFIG = os.path.join(ROOT, "nanopore-barcoding-orc_amd", "dmx", "data",
                          "M13_config_for_pychopper.txt")
ALPH = np.array(list("ACGT"))


def _dna(rng, n):
    return "".join(ALPH[rng.integers(0, 4, size=n)])


def _quals(rng, n, lo=12, hi=41):
    return "".join(chr(33 + int(x)) for x in rng.integers(lo, hi, size=n))


def _ref_primers():
    from dmx import chop
    return chop.load_primers(REF_PRIMERS), open(REF_CONFIG).read().strip()


def _synth_records(seed, n, noise):
    """c2-like reoriented-or-not reads (both primers, random orientation), adapter-region
    errors `noise`, a few fused and primer-less reads."""
    from dmx import synth
    d = synth.generate("c2", n=n, seed=seed)
    seqs = synth.to_strings(d)
    rng = np.random.default_rng(seed)
    out = []
    for i, s in enumerate(seqs):
        b = bytearray(s.encode())
        for j in np.nonzero(rng.random(len(b)) < noise)[0]:
            b[j] = ord("ACGT"[int(rng.integers(4))])
        s = b.decode()
        if rng.random() < 0.08 and i + 1 < len(seqs):
            s = s + seqs[i + 1]                       # fused
        out.append((f"r{i} runid=case ch={i}", s, _quals(rng, len(s))))
    return out


def case_tune_grid(seed):
    primers, config = _ref_primers()
    return dict(records=_synth_records(seed, 60, 0.04), primers=primers, config=config,
                opts=["-Q", "10", "-p", "-m", "edlib"])


def case_tune_sample(seed):
    primers, config = _ref_primers()
    recs = _synth_records(seed, 40, 0.02) + _synth_records(seed + 1, 80, 0.12)
    return dict(records=recs, primers=primers, config=config,
                opts=["-Q", "10", "-p", "-m", "edlib", "-Y", "30"])


def case_tune_score(seed):
    primers, config = _ref_primers()
    return dict(records=_synth_records(seed, 80, 0.10), primers=primers, config=config,
                opts=["-Q", "10", "-p", "-m", "edlib"])


def case_seg_score(seed):
    """Primers P, Q with the layout +:P,Q|+:Q,P: a read P.Q<long>P.Q has candidates (P,Q),
    (Q,P), (P,Q); the summed-length best path is the one long (Q,P) segment, the most-segments
    path the two short (P,Q) ones."""
    rng = np.random.default_rng(seed)
    p, q = _dna(rng, 22), _dna(rng, 22)
    recs = []
    for i in range(12):
        a, b = _dna(rng, int(rng.integers(60, 90))), _dna(rng, int(rng.integers(60, 90)))
        mid = _dna(rng, int(rng.integers(500, 900)))
        s = _dna(rng, 10) + p + a + q + mid + p + b + q + _dna(rng, 10)
        recs.append((f"f{i}", s, _quals(rng, len(s))))
        s = _dna(rng, 10) + p + _dna(rng, 300) + q + _dna(rng, 10)
        recs.append((f"s{i}", s, _quals(rng, len(s))))
    return dict(records=recs, primers=[("P", p), ("Q", q)], config="+:P,Q|+:Q,P",
                opts=["-Q", "10", "-p", "-m", "edlib", "-q", "0.1"])


def case_naming(seed):
    primers, config = _ref_primers()
    return dict(records=_synth_records(seed, 20, 0.02), primers=primers, config=config,
                opts=["-Q", "10", "-p", "-m", "edlib", "-q", "0.15"])


# name: (switch, generator, seed found by --search)
CASES = {
    "tune_grid": ("tune_grid", case_tune_grid, 101),
    "tune_sample": ("tune_sample", case_tune_sample, 202),
    "tune_score": ("tune_score", case_tune_score, 316),
    "seg_score": ("seg_score", case_seg_score, 404),
    "naming": ("naming", case_naming, 505),
}


def _opt(opts, flag, default=None):
    return opts[opts.index(flag) + 1] if flag in opts else default


def oracle_outputs(case: dict, rules: dict | None = None):
    """The case's outputs under the given readings (default: the build's): the cutoff and the
    pass / rescued / unclass / short record lists."""
    import chopper
    saved = dict(chopper.RULES)
    if rules:
        chopper.RULES.update(rules)
    try:
        opts = case["opts"]
        minq = float(_opt(opts, "-Q", 7.0))
        q = _opt(opts, "-q")
        if q is None:
            cut = chopper.autotune(case["records"], case["primers"], case["config"], keep=True,
                                   min_qual=minq, sample=int(float(_opt(opts, "-Y", 10000))),
                                   samples=int(_opt(opts, "-L", chopper.AUTOTUNE_SAMPLES)))
        else:
            cut = float(q)
        out = chopper.chop_records(case["records"], case["primers"], case["config"], cut,
                                   keep="-p" in opts, min_qual=minq, min_len=50)
    finally:
        chopper.RULES.clear()
        chopper.RULES.update(saved)
    return dict(cutoff=cut, **{k: out[k] for k in ("pass", "rescued", "unclass", "short")})


def build(name: str) -> dict:
    switch, gen, seed = CASES[name]
    c = gen(seed)
    c["switch"] = switch
    return c


def write(d: str):
    os.makedirs(d, exist_ok=True)
    rows = []
    for name in CASES:
        c = build(name)
        with open(os.path.join(d, f"{name}.fastq"), "w") as fh:
            for h, s, q in c["records"]:
                fh.write(f"@{h}\n{s}\n+\n{q}\n")
        with open(os.path.join(d, f"{name}_primers.fa"), "w") as fh:
            for n, s in c["primers"]:
                fh.write(f">{n}\n{s}\n")
        with open(os.path.join(d, f"{name}_config.txt"), "w") as fh:
            fh.write(c["config"] + "\n")
        opts = ["-b", f"{name}_primers.fa", "-c", f"{name}_config.txt"] + c["opts"]
        rows.append("\t".join([name, f"{name}.fastq", " ".join(opts)]))
    with open(os.path.join(d, "cases.tsv"), "w") as fh:
        fh.write("\n".join(rows) + "\n")


def search():
    """The first seed (from each case's start seed) whose outputs differ between the readings."""
    import chopper
    for name, (switch, gen, start) in CASES.items():
        for seed in range(start, start + 200):
            c = gen(seed)
            a = oracle_outputs(c)
            b = oracle_outputs(c, {switch: chopper.ALT_RULES[switch]})
            if a != b:
                print(name, seed, "cutoff", a["cutoff"], b["cutoff"])
                break
        else:
            print(name, "no seed found")


if __name__ == "__main__":
    if sys.argv[1:] == ["--search"]:
        search()
    else:
        write(sys.argv[1])
