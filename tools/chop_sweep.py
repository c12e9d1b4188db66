"""Randomised GPU-vs-oracle parity sweep of the pychopper-style reorientation (dmx_chop_*; run
on the GPU box; oracle/chop_oracle.c + oracle/chopper.py are the checker).

    python tools/chop_sweep.py [--seconds 150] [--seed 1] [--out gpurun_out/chop_sweep.json]

Draws random cases until the time budget is spent: 1..8 primers of 3..64 nt (IUPAC share
0..50 %) or the reference's M13 primers, 0..12 random rules (or the reference's layout), cutoff
0..0.45, -p on/off, 20..400 reads of 0..3000 nt (N share 0..5 %) carrying 0..4 planted primer
copies (either strand, 0..15 % edits, some truncated at a read end), plus config-2 reads with
fused pairs.  Every hit (read, label, distance, start, stop) and every segment (read, start,
stop, strand, rule) is compared; mismatching cases are written out with their parameters.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "nanopore-barcoding-orc_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import chopper as ochop  # noqa: E402  (checker only)
import oracle  # noqa: E402
from dmx import chop, lib, synth  # noqa: E402

IUPAC = list("RYSWKMBDHVN")


sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from provenance import provenance  # noqa: E402

def rand_primer(rng, n, iupac_share):
    return "".join(rng.choice(IUPAC) if rng.random() < iupac_share else "ACGT"[rng.integers(4)]
                   for _ in range(n))


def instance(rng, pat, err):
    out = []
    for c in pat:
        opts = ochop._IUPAC[c]
        b = opts[int(rng.integers(len(opts)))]
        r = rng.random()
        if r < err * 0.6:
            out.append("ACGT"[int(rng.integers(4))])
        elif r < err * 0.8:
            continue
        elif r < err:
            out += [b, "ACGT"[int(rng.integers(4))]]
        else:
            out.append(b)
    return "".join(out)


def make_case(rng):
    if rng.random() < 0.25:
        primers = chop.load_primers(chop.PRIMERS_FASTA)
        with open(chop.CONFIG_FILE) as fh:
            rules = chop.parse_config(fh.read(), [p[0] for p in primers])
    else:
        npr = int(rng.integers(1, 9))
        share = float(rng.choice([0.0, 0.1, 0.3, 0.5]))
        primers = [(f"P{i}", rand_primer(rng, int(rng.integers(3, 65)), share))
                   for i in range(npr)]
        nl = 2 * npr
        rules = [(int(rng.integers(nl)), int(rng.integers(nl)), int(rng.integers(2)))
                 for _ in range(int(rng.integers(0, 13)))]
    labs = [s for _, s in ochop.labels(primers)]
    short = min(len(p[1]) for p in primers) < 8
    cutoff = float(rng.choice([0.0, 0.05, 0.1, 0.15] if short else
                              [0.0, 0.05, 0.1, 0.15, 0.2, 0.3, 0.45]))
    keep = bool(rng.integers(2))
    seqs = []
    if rng.random() < 0.2:
        d = synth.generate("c2", n=int(rng.integers(20, 300)), seed=int(rng.integers(1 << 30)))
        for s in synth.to_strings(d):
            if seqs and rng.random() < 0.15:
                s = s + seqs[-1]
            seqs.append(s)
    else:
        nshare = float(rng.choice([0.0, 0.0, 0.01, 0.05]))
        for _ in range(int(rng.integers(20, 400))):
            n = int(rng.integers(0, 3000))
            s = "".join("N" if rng.random() < nshare else "ACGT"[int(rng.integers(4))]
                        for _ in range(n)) if nshare else \
                "".join(np.array(list("ACGT"))[rng.integers(0, 4, size=n)])
            for _ in range(int(rng.integers(0, 5))):
                inst = instance(rng, labs[int(rng.integers(len(labs)))],
                                float(rng.choice([0.0, 0.05, 0.15])))
                if rng.random() < 0.1:
                    inst = inst[int(rng.integers(0, len(inst) + 1)):]
                p = int(rng.integers(0, len(s) + 1))
                s = s[:p] + inst + s[p:]
            seqs.append(s)
    return dict(primers=primers, rules=rules, cutoff=cutoff, keep=keep, seqs=seqs)


def run_case(ctx, c):
    blob, offs, lens = oracle.pack_ascii(c["seqs"])
    ctx.load(lib.pack(blob, offs, lens))
    ctx.chop_set([p[1] for p in c["primers"]], c["rules"], c["cutoff"], c["keep"])
    ctx.chop_exec()
    _, _, segs, hits = ctx.chop_fetch(hits=True)
    H = list(zip(*(hits[f].tolist() for f in ("read", "label", "dist", "start", "stop"))))
    S = list(zip(*(segs[f].tolist() for f in ("read", "start", "stop", "strand", "rule"))))
    labs = ochop.labels(c["primers"])
    eH, eS = [], []
    for r, s in enumerate(c["seqs"]):
        hs = ochop.read_hits(labs, s, c["cutoff"])
        eH += [(r, lab, d, a, b) for a, b, lab, d in hs]
        eS += [(r, a, b, st, ri) for a, b, st, ri in ochop.segments(hs, c["rules"], c["keep"])]
    return H == eH and S == eS, len(H)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=150)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default="gpurun_out/chop_sweep.json")
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    ctx = lib.Context(0)
    t0 = time.time()
    cases = reads = hits = 0
    bad = []
    last = t0
    while time.time() - t0 < a.seconds:
        c = make_case(rng)
        ok, nh = run_case(ctx, c)
        cases += 1
        reads += len(c["seqs"])
        hits += nh
        if not ok:
            bad.append({k: c[k] for k in ("primers", "rules", "cutoff", "keep")} |
                       {"n_reads": len(c["seqs"])})
        if time.time() - last > 30:
            last = time.time()
            print(f"{cases} cases, {reads} reads, {hits} hits, {len(bad)} mismatching",
                  flush=True)
    res = {"seed": a.seed, "seconds": round(time.time() - t0, 1), "cases": cases, "reads": reads,
           "hits": hits, "mismatching_cases": len(bad), "mismatches": bad[:20],
           "provenance": provenance()}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "mismatches"}))
    ctx.close()
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
