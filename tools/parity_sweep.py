"""Randomised GPU-vs-oracle parity sweep (run on the GPU box; the oracle is the checker).

    python tools/parity_sweep.py [--seconds 150] [--out gpurun_out/sweep.json]

Draws random cases until the time budget is spent: panel shape (lengths 3..64, IUPAC share,
FRONT / BACK / mixed), -e (rate 0.0..0.3 or an absolute count 1..4), -O 1..12, --rc on/off,
reads 0..600 nt with N, planted adapters (full, partial at either end, internal, reverse
strand, 0..15 % edits), plus the seeded synthetic configs c1..c5 at random seeds and the
two-round / linked modes.  Every field of every read is compared; mismatching cases are written
out with their parameters so they can be replayed.
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

import oracle  # noqa: E402  (checker only)
from dmx import lib, synth  # noqa: E402

ALPH = np.array(list("ACGT"))


sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from provenance import provenance  # noqa: E402

def rand_seq(rng, n):
    return "".join(ALPH[rng.integers(0, 4, size=n)])


def rc(s):
    return s.translate(str.maketrans("ACGTN", "TGCAN"))[::-1]


def mutate(rng, a, err):
    out = []
    for c in a:
        if c not in "ACGT":
            c = "ACGT"[int(rng.integers(4))]
        r = rng.random()
        if r < err * 0.6:
            out.append("ACGT"[int(rng.integers(4))])
        elif r < err * 0.8:
            pass
        elif r < err:
            out += [c, "ACGT"[int(rng.integers(4))]]
        else:
            out.append(c)
    return "".join(out)


def random_panel(rng):
    n = int(rng.integers(1, 17))
    lo = int(rng.integers(3, 40))
    hi = int(rng.integers(lo, 65))
    wild = float(rng.choice([0.0, 0.0, 0.05, 0.2]))
    shared = rng.random() < 0.4          # common flanks (exercises the window filter path)
    pre, suf = rand_seq(rng, int(rng.integers(0, 25))), rand_seq(rng, int(rng.integers(10, 25)))
    out = []
    for _ in range(n):
        L = int(rng.integers(lo, hi + 1))
        s = rand_seq(rng, L)
        if shared:
            s = (pre + rand_seq(rng, int(rng.integers(3, 29))) + suf)[:64]
        s = "".join(c if rng.random() >= wild else str(rng.choice(list("NRYSWKMBDHV"))) for c in s)
        out.append(s)
    return out


def reads_for(rng, panel, n):
    seqs = []
    maxlen = int(rng.choice([40, 150, 600]))
    for _ in range(n):
        s = rand_seq(rng, int(rng.integers(0, maxlen + 1)))
        if rng.random() < 0.01:
            s = "".join(c if rng.random() > 0.05 else "N" for c in s)
        for _k in range(int(rng.integers(0, 3))):
            frag = mutate(rng, panel[int(rng.integers(len(panel)))], float(rng.uniform(0, 0.15)))
            u = rng.random()
            if u < 0.2 and len(frag) > 1:
                frag = frag[int(rng.integers(1, len(frag))):]
                s = frag + s
            elif u < 0.4 and len(frag) > 1:
                frag = frag[:int(rng.integers(1, len(frag)))]
                s = s + frag
            else:
                p = int(rng.integers(0, len(s) + 1))
                s = s[:p] + frag + s[p:]
        if rng.random() < 0.3:
            s = rc(s)
        seqs.append(s)
    return seqs


def compare(got, exp):
    g = got.view(np.uint8).reshape(len(got), -1)
    e = exp.view(np.uint8).reshape(len(exp), -1)
    return np.nonzero((g != e).any(axis=1))[0]


def case_random(rng, ctx):
    panel = random_panel(rng)
    e = float(rng.choice([0.0, 0.05, 0.1, 0.15, 0.2, 0.3])) if rng.random() < 0.8 else \
        float(rng.integers(1, 5))
    mo = int(rng.choice([1, 2, 3, 3, 3, 5, 8, 12]))
    use_rc = bool(rng.random() < 0.7)
    kind = str(rng.choice(["front", "back", "mixed"]))
    wh = [oracle.FRONT if (kind == "front" or (kind == "mixed" and rng.random() < 0.5))
          else oracle.BACK for _ in panel]
    seqs = reads_for(rng, panel, int(rng.integers(200, 3000)))
    blob, offs, lens = oracle.pack_ascii(seqs)
    exp = oracle.run_batch(oracle.Panel(panel, wh, max_errors=e, min_overlap=mo), None, blob, offs,
                           lens, mode=0, use_rc=use_rc, threads=16)
    ctx.set_panel_mixed(0, panel, [lib.DMX_FRONT if w == oracle.FRONT else lib.DMX_BACK
                                   for w in wh], use_rc, e, mo)
    ctx.set_mode(lib.MODE_SINGLE)
    got = ctx.run(lib.pack(blob, offs, lens))
    params = dict(kind="random", panel=panel, wheres=wh, e=e, min_overlap=mo, rc=use_rc)
    return len(seqs), compare(got, exp), params, seqs


def case_random_pair(rng, ctx):
    """Two random panels as two rounds (FRONT then BACK) or as linked -g F...R pairs."""
    linked = bool(rng.random() < 0.4)
    p1 = random_panel(rng)
    p2 = random_panel(rng)
    if linked:
        k = min(len(p1), len(p2))
        p1, p2 = p1[:k], p2[:k]
    e = float(rng.choice([0.05, 0.1, 0.15, 0.2])) if rng.random() < 0.85 else \
        float(rng.integers(1, 4))
    mo = int(rng.choice([1, 3, 3, 5]))
    use_rc = (not linked) and bool(rng.random() < 0.8)
    seqs = []
    for s in reads_for(rng, p1 + p2, int(rng.integers(200, 2500))):
        if linked and rng.random() < 0.6:
            a = int(rng.integers(len(p1)))
            s = (rand_seq(rng, int(rng.integers(0, 20))) + mutate(rng, p1[a], 0.05) +
                 rand_seq(rng, int(rng.integers(0, 200))) + mutate(rng, p2[a], 0.05) +
                 rand_seq(rng, int(rng.integers(0, 20))))
        seqs.append(s)
    blob, offs, lens = oracle.pack_ascii(seqs)
    exp = oracle.run_batch(oracle.Panel(p1, oracle.FRONT, max_errors=e, min_overlap=mo),
                           oracle.Panel(p2, oracle.BACK, max_errors=e, min_overlap=mo), blob,
                           offs, lens, mode=2 if linked else 1, use_rc=use_rc, threads=16)
    f = lib.DMX_RC if use_rc else 0
    ctx.set_panel(0, p1, lib.DMX_FRONT | f, e, mo)
    ctx.set_panel(1, p2, lib.DMX_BACK | f, e, mo)
    ctx.set_mode(lib.MODE_LINKED if linked else lib.MODE_TWO_ROUND)
    got = ctx.run(lib.pack(blob, offs, lens))
    params = dict(kind="pair", linked=linked, panel1=p1, panel2=p2, e=e, min_overlap=mo,
                  rc=use_rc)
    return len(seqs), compare(got, exp), params, seqs


def case_synth(rng, ctx):
    cfg = str(rng.choice(["c1", "c2", "c2x24", "c4", "c5"]))
    seed = int(rng.integers(1000, 10 ** 6))
    n = int(rng.integers(2000, 20000))
    e = 0.1 if rng.random() < 0.7 else float(rng.choice([0.05, 0.15, 0.2]))
    d = synth.generate(cfg, n=n, seed=seed)
    linked = cfg == "c5"
    p1 = oracle.Panel(d["sp5"], oracle.FRONT, max_errors=e)
    p2 = oracle.Panel(d["sp27"], oracle.BACK, max_errors=e)
    exp = oracle.run_batch(p1, p2, d["blob"], d["offsets"], d["lengths"], mode=2 if linked else 1,
                           use_rc=not linked, threads=16)
    f = 0 if linked else lib.DMX_RC
    ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | f, e)
    ctx.set_panel(1, d["sp27"], lib.DMX_BACK | f, e)
    ctx.set_mode(lib.MODE_LINKED if linked else lib.MODE_TWO_ROUND)
    got = ctx.run(lib.pack(d["blob"], d["offsets"], d["lengths"]))
    return n, compare(got, exp), dict(kind="synth", config=cfg, seed=seed, n=n, e=e), None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=150)
    ap.add_argument("--seed", type=int, default=int(time.time()))
    ap.add_argument("--out", default="gpurun_out/parity_sweep.json")
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    t0 = time.time()
    cases = reads = 0
    bad = []
    with lib.Context(0) as ctx:
        while time.time() - t0 < a.seconds:
            u = rng.random()
            fn = case_random if u < 0.5 else (case_random_pair if u < 0.8 else case_synth)
            n, idx, params, seqs = fn(rng, ctx)
            cases += 1
            reads += n
            if len(idx):
                params["n_bad"] = int(len(idx))
                if seqs is not None:
                    params["bad_reads"] = [seqs[int(i)] for i in idx[:5]]
                else:
                    params["bad_index"] = [int(i) for i in idx[:20]]
                bad.append(params)
                print("MISMATCH", json.dumps(params)[:400], flush=True)
            if cases % 20 == 0:
                print(f"{time.time() - t0:.0f}s: {cases} cases, {reads} reads, "
                      f"{len(bad)} mismatching cases", flush=True)
    res = dict(seed=a.seed, seconds=round(time.time() - t0, 1), cases=cases, reads=reads,
               mismatching_cases=len(bad), mismatches=bad, provenance=provenance())
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "mismatches"}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
