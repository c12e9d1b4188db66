"""Round-1 (FRONT) near-start work on the GPU box: how much of the window scan and the band
stage goes to the "near pieces" that the index screen hands over with every adapter (windows
with j1 < jsplit), and what those pieces yield.

    python tools/near_stats.py [--workload c2x24] [--reads 2000000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nanopore-barcoding-orc_amd"))

from dmx import lib, synth  # noqa: E402


def common(seqs, suffix: bool) -> int:
    n = min(len(s) for s in seqs)
    k = 0
    while k < n and len({(s[-1 - k] if suffix else s[k]) for s in seqs}) == 1:
        k += 1
    return k


def pct(x, q=(50, 90, 99, 100)):
    return np.percentile(x, q).tolist() if len(x) else []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2x24")
    ap.add_argument("--reads", type=int, default=2_000_000)
    a = ap.parse_args()
    d = synth.generate(a.workload, n=a.reads, threads=16)
    ads = d["sp5"]
    ms = np.array([len(s) for s in ads])
    kk = (0.1 * ms).astype(np.int64)
    pl, sl = common(ads, False), common(ads, True)
    jsplit = int((ms - pl + kk).max())
    out = {"workload": a.workload, "reads": a.reads, "pre_len": pl, "suffix_len": sl,
           "jsplit": jsplit}
    with lib.Context(0) as ctx:
        ctx.set_panel(0, ads, lib.DMX_FRONT | lib.DMX_RC, 0.1)
        ctx.load(lib.pack(d["blob"], d["offsets"], d["lengths"]))
        ctx.set_mode(lib.MODE_SINGLE)
        ctx.exec()
        ctx.sync()
        res = ctx.fetch()
        w = ctx.debug_fetch(lib.DBG_VERIFIED, 0)
        t = ctx.debug_fetch(lib.DBG_TASKS, 0)
        c0 = ctx.debug_fetch(lib.DBG_CANDS0, 0)
        c1 = ctx.debug_fetch(lib.DBG_CANDS1, 0)
    j1 = w["j1"].astype(np.int64)
    nearw = j1 < jsplit
    out["windows"] = int(len(w))
    out["near_windows"] = int(nearw.sum())
    out["near_window_j1_pcts"] = pct(j1[nearw])
    out["near_window_j2_pcts"] = pct(w["j2"].astype(np.int64)[nearw])
    tj1, tj2 = t["j1"].astype(np.int64), t["j2"].astype(np.int64)
    m_of = ms[t["info"].astype(np.int64)]
    js = np.maximum(tj1 - m_of - 6, 0)
    cols = tj2 - js
    neart = tj2 < jsplit
    out["tasks"] = int(len(t))
    out["near_tasks"] = int(neart.sum())
    out["cols_total"] = int(cols.sum())
    out["near_cols_total"] = int(cols[neart].sum())
    for nm, c in (("cands0", c0), ("cands1", c1)):
        j = c["j"].astype(np.int64)
        near = (j < jsplit) & (c["iend"].astype(np.int64) == ms[c["a"].astype(np.int64)])
        out[nm] = {"n": int(len(c)), "near": int(near.sum()),
                   "near_cost_hist": np.bincount(c["cost"][near].astype(np.int64),
                                                 minlength=8).tolist(),
                   "cost_hist": np.bincount(c["cost"].astype(np.int64), minlength=8).tolist()}
    hit = res["bin1"] >= 0
    rstop = res["m1_rstop"].astype(np.int64)
    out["reads_with_match"] = int(hit.sum())
    out["winner_rstop_lt_jsplit"] = int((hit & (rstop < jsplit)).sum())
    out["winner_rstop_pcts"] = pct(rstop[hit], (1, 5, 10, 50))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
