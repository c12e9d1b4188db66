"""Run-to-run determinism of the device pipeline (GPU box): the same resident batch executed
repeatedly must give identical per-read results and identical intermediate lists (as multisets:
list order is scheduling-dependent).

    python tools/determinism.py [--workload c2x24] [--reads 2000000] [--reps 8] [--mode two]

Reports, per repetition, which intermediate lists differ from the first repetition's and how
many reads' results differ, so a race can be located to the first stage that diverges."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nanopore-barcoding-orc_amd"))

from dmx import lib, synth  # noqa: E402

LISTS = (("verified", lib.DBG_VERIFIED), ("tasks", lib.DBG_TASKS),
         ("cands0", lib.DBG_CANDS0), ("cands1", lib.DBG_CANDS1))


def canon(rec: np.ndarray) -> np.ndarray:
    """Records as a sorted array of their named fields (implicit padding excluded)."""
    names = [n for n in rec.dtype.names if not n.startswith("pad")]
    if not len(rec):
        return np.zeros(0, dtype=[(n, rec.dtype[n]) for n in names])
    out = np.zeros(len(rec), dtype=[(n, rec.dtype[n]) for n in names])
    for n in names:
        out[n] = rec[n]
    return np.sort(out, order=names)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2x24")
    ap.add_argument("--reads", type=int, default=2_000_000)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--mode", default="single", choices=["single", "two"])
    a = ap.parse_args()
    d = synth.generate(a.workload, n=a.reads, threads=16)
    out = {"workload": a.workload, "reads": a.reads, "mode": a.mode, "reps": []}
    with lib.Context(0) as ctx:
        ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC, 0.1)
        ctx.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC, 0.1)
        ctx.set_mode(lib.MODE_SINGLE if a.mode == "single" else lib.MODE_TWO_ROUND)
        ctx.load(lib.pack(d["blob"], d["offsets"], d["lengths"]))
        ref = None
        rnd = 0 if a.mode == "single" else 1
        for rep in range(a.reps):
            ctx.exec()
            ctx.sync()
            res = ctx.fetch()
            # windows / tasks: the last round's (shared buffers); candidates: round 0's
            lists = {nm: canon(ctx.debug_fetch(w, 0 if nm.startswith("cands") else rnd))
                     for nm, w in LISTS}
            if a.mode == "two":   # the candidate lists of both rounds are kept
                lists["cands0_r1"] = canon(ctx.debug_fetch(lib.DBG_CANDS0, 1))
                lists["cands1_r1"] = canon(ctx.debug_fetch(lib.DBG_CANDS1, 1))
            flags = int(ctx.debug_fetch(lib.DBG_FLAGS)[0])
            if ref is None:
                ref = (res, lists)
                out["sizes"] = {k: len(v) for k, v in lists.items()}
                continue
            g = res.view(np.uint8).reshape(len(res), -1)
            bad = np.nonzero((g != ref[0].view(np.uint8).reshape(len(res), -1)).any(axis=1))[0]
            diff = {k: (len(np.setdiff1d(v, ref[1][k])), len(np.setdiff1d(ref[1][k], v)))
                    for k, v in lists.items() if not np.array_equal(v, ref[1][k])}
            out["reps"].append({"rep": rep, "reads_differing": int(len(bad)), "flags": flags,
                                "sizes": {k: len(v) for k, v in lists.items()
                                          if len(v) != len(ref[1][k])},
                                "lists_differing": diff,
                                "first_reads": [int(i) for i in bad[:5]]})
            print(json.dumps(out["reps"][-1]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
