#!/usr/bin/env python3
"""Replay a tools/parity_sweep.py run's random draws on the CPU (no GPU, no oracle) up to the
case whose parameters match a recorded mismatch, and write that case (parameters + every read)
as JSON, so it can be run alone against the oracle with any libdmx build (--run, on the GPU box).

usage: python tools/replay_sweep.py SWEEP_JSON [--which 0] --out CASE_JSON
       python tools/replay_sweep.py --run CASE_JSON        (GPU: per-read diff vs the oracle)
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "nanopore-barcoding-orc_amd"), os.path.join(ROOT, "oracle"),
          os.path.dirname(os.path.abspath(__file__))):
    sys.path.insert(0, p)

import oracle  # noqa: E402  (checker only)


class _NoCtx:
    """Stands in for lib.Context while replaying the draws: records nothing, runs nothing."""

    def set_panel(self, *a, **k):
        pass

    set_panel_mixed = set_mode = set_panel

    def run(self, p):
        from dmx import lib
        return np.zeros(p.n_reads, dtype=lib.RESULT_DTYPE)


def find(sweep_json, which, out):
    import parity_sweep as ps
    rec = json.load(open(sweep_json))
    target = rec["mismatches"][which]
    rng = np.random.default_rng(rec["seed"])
    real = oracle.run_batch
    oracle.run_batch = lambda p1, p2, blob, offs, lens, **k: np.zeros(
        len(lens), dtype=oracle.RESULT_DTYPE)
    try:
        for case in range(rec["cases"]):
            u = rng.random()
            fn = ps.case_random if u < 0.5 else (ps.case_random_pair if u < 0.8
                                                 else ps.case_synth)
            _, _, params, seqs = fn(rng, _NoCtx())
            if all(params.get(k) == v for k, v in params.items() if k in target) and \
                    all(target.get(k) == params.get(k) for k in params):
                json.dump(dict(case=case, params=params, reads=seqs), open(out, "w"))
                print(f"case {case}: {params['kind']}, {len(seqs or [])} reads -> {out}")
                return 0
    finally:
        oracle.run_batch = real
    print("not found")
    return 1


def run(case_json):
    from dmx import lib
    c = json.load(open(case_json))
    p, seqs = c["params"], c["reads"]
    assert p["kind"] == "random", "only random single-round cases"
    blob, offs, lens = oracle.pack_ascii(seqs)
    exp = oracle.run_batch(oracle.Panel(p["panel"], p["wheres"], max_errors=p["e"],
                                        min_overlap=p["min_overlap"]), None, blob, offs, lens,
                           mode=0, use_rc=p["rc"], threads=8)
    with lib.Context(0) as ctx:
        ctx.set_panel_mixed(0, p["panel"], [lib.DMX_FRONT if w == oracle.FRONT else lib.DMX_BACK
                                            for w in p["wheres"]], p["rc"], p["e"],
                            p["min_overlap"])
        ctx.set_mode(lib.MODE_SINGLE)
        got = ctx.run(lib.pack(blob, offs, lens))
    g = got.view(np.uint8).reshape(len(got), -1)
    e = exp.view(np.uint8).reshape(len(exp), -1)
    bad = np.nonzero((g != e).any(axis=1))[0]
    print(f"{lib.LIB_PATH}: {len(bad)} of {len(seqs)} reads differ")
    for i in bad[:12]:
        print(i, repr(seqs[i][:80]), len(seqs[i]))
        print("  got", got[i])
        print("  exp", exp[i])
    return 1 if len(bad) else 0


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("sweep", nargs="?")
    ap.add_argument("--which", type=int, default=0)
    ap.add_argument("--out")
    ap.add_argument("--run")
    a = ap.parse_args()
    sys.exit(run(a.run) if a.run else find(a.sweep, a.which, a.out))
