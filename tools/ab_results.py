"""A/B check at benchmark scale (GPU box): the per-read results of one workload with the default
pipeline vs an alternative (environment toggles), and run-to-run determinism.

    python tools/ab_results.py [--workload c2x24] [--reads 2000000] [--env DMX_NO_SCREEN=1]

Every field of every read is compared; the oracle is not involved (the parity tests pin the
default path to it), so this covers sizes the oracle cannot finish."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nanopore-barcoding-orc_amd"))

from dmx import lib, synth  # noqa: E402


def run(d, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        with lib.Context(0) as ctx:   # env toggles are read at dmx_open
            ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC, 0.1)
            ctx.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC, 0.1)
            ctx.set_mode(lib.MODE_TWO_ROUND)
            ctx.load(lib.pack(d["blob"], d["offsets"], d["lengths"]))
            ctx.set_mode(lib.MODE_SINGLE)   # round 0 alone first: its intermediate lists
            ctx.exec()
            ctx.sync()
            lists = {nm: np.sort(ctx.debug_fetch(w, 0).view(np.uint8).reshape(-1, 40).view("V40")
                                 .ravel())
                     for nm, w in (("verified", lib.DBG_VERIFIED),
                                   ("tasks", lib.DBG_TASKS),
                                   ("cands0", lib.DBG_CANDS0), ("cands1", lib.DBG_CANDS1))}
            lists["flags"] = int(ctx.debug_fetch(lib.DBG_FLAGS)[0])
            ctx.set_mode(lib.MODE_TWO_ROUND)
            ctx.exec()
            ctx.sync()
            st = ctx.stats()
            st["lists"] = lists
            return ctx.fetch(), ctx.counts(), st
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2x24")
    ap.add_argument("--reads", type=int, default=2_000_000)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE for the B run")
    ap.add_argument("--env-all", action="append", default=[], help="KEY=VALUE for every run")
    a = ap.parse_args()
    d = synth.generate(a.workload, n=a.reads, seed=a.seed, threads=16)
    env_b = dict(kv.split("=", 1) for kv in a.env)
    os.environ.update(dict(kv.split("=", 1) for kv in a.env_all))
    r1, c1, s1 = run(d, {})
    r2, c2, s2 = run(d, {})
    rb, cb, sb = run(d, env_b)
    g = r1.view(np.uint8).reshape(len(r1), -1)
    det = np.nonzero((g != r2.view(np.uint8).reshape(len(r2), -1)).any(axis=1))[0]
    ab = np.nonzero((g != rb.view(np.uint8).reshape(len(rb), -1)).any(axis=1))[0]
    out = {"workload": a.workload, "reads": a.reads, "env_b": env_b,
           "rerun_mismatching_reads": int(len(det)), "ab_mismatching_reads": int(len(ab)),
           "first_ab_mismatches": [int(i) for i in ab[:10]],
           "counts_equal": bool(np.array_equal(c1, cb) and np.array_equal(c1, c2)),
           "ms_default": s1["ms"]["total"], "ms_b": sb["ms"]["total"],
           "flags": [s1["lists"]["flags"], s2["lists"]["flags"], sb["lists"]["flags"]],
           "round0_lists_equal_rerun": {k: bool(np.array_equal(v, s2["lists"][k]))
                                        for k, v in s1["lists"].items() if k != "flags"},
           "round0_list_sizes": {k: [len(v), len(s2["lists"][k])]
                                 for k, v in s1["lists"].items() if k != "flags"}}
    for k in ("tasks", "verified"):   # records in one run and not the other
        x, y = s1["lists"][k], s2["lists"][k]
        if len(x) and not np.array_equal(x, y):
            only1 = np.setdiff1d(x, y)
            only2 = np.setdiff1d(y, x)
            dec = lambda v: [{f: int(r[f]) for f in lib.WINDOW_DTYPE.names}
                             for r in v[:6].view(np.uint8).reshape(-1, 40).copy()
                             .view(lib.WINDOW_DTYPE).ravel()]
            out[f"{k}_only_run1"] = dec(only1)
            out[f"{k}_only_run2"] = dec(only2)
            out[f"{k}_n_only"] = [len(only1), len(only2)]
    bad = sorted(set(det.tolist()) | set(ab.tolist()))[:8]
    if bad:   # the differing reads: every run's result and the oracle's (checker only)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        offs = d["offsets"][bad]
        lens = d["lengths"][bad]
        exp = oracle.run_batch(oracle.Panel(d["sp5"], oracle.FRONT),
                               oracle.Panel(d["sp27"], oracle.BACK), d["blob"], offs, lens, mode=1)
        out["detail"] = []
        for k, i in enumerate(bad):
            row = {"read": int(i), "len": int(lens[k])}
            for nm, r in (("run1", r1), ("run2", r2), ("b", rb), ("oracle", exp)):
                x = r[i] if nm != "oracle" else r[k]
                row[nm] = {f: int(x[f]) for f in r.dtype.names if f != "pad"}
            out["detail"].append(row)
    print(json.dumps(out))
    sys.exit(1 if (len(det) or len(ab)) else 0)


if __name__ == "__main__":
    main()
