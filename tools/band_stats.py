"""How many band-DP candidates could never win their read (GPU box): for round 1 of c2x24 in
single mode, every candidate cell of both lists (cost <= 3, cost >= 4) against its read's final
result.  A cell's score is at most min(iend, j + cost) - 2 cost; a cell whose bound is below the
read's final score cannot be the winner, so its DP only matters if no better cell is known when
it runs.

    python tools/band_stats.py [--workload c2x24] [--reads 2000000]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2x24")
    ap.add_argument("--reads", type=int, default=2_000_000)
    a = ap.parse_args()
    d = synth.generate(a.workload, n=a.reads, threads=16)
    out = {"workload": a.workload, "reads": a.reads}
    with lib.Context(0) as ctx:
        ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC, 0.1)
        ctx.load(lib.pack(d["blob"], d["offsets"], d["lengths"]))
        ctx.set_mode(lib.MODE_SINGLE)
        ctx.exec()
        ctx.sync()
        res = ctx.fetch()
        lists = [ctx.debug_fetch(lib.DBG_CANDS0, 0), ctx.debug_fetch(lib.DBG_CANDS1, 0)]
        st = ctx.stats()
        out["stats"] = {k: v for k, v in st.items() if k != "ms"}
    best = np.where(res["bin1"] >= 0, res["m1_score"].astype(np.int64), -10**6)
    errs = np.where(res["bin1"] >= 0, res["m1_errors"].astype(np.int64), -1)
    for li, c in enumerate(lists):
        cost = c["cost"].astype(np.int64)
        ub = np.minimum(c["iend"].astype(np.int64), c["j"].astype(np.int64) + cost) - 2 * cost
        fin = best[c["item"].astype(np.int64)]
        can = ub >= fin
        out[f"list{li}"] = {
            "cells": int(len(c)),
            "by_cost": np.bincount(cost, minlength=8).tolist(),
            "could_win_by_cost": np.bincount(cost[can], minlength=8).tolist(),
            "never_win_by_cost": np.bincount(cost[~can], minlength=8).tolist(),
            # cells that cannot win, of reads whose winner has cost >= 4 (list 1): the cells a
            # cost-ordered DP could skip that phase 1's screen (winner after list 0) keeps
            "never_win_read_cost4plus_by_cost": np.bincount(
                cost[~can & (errs[c["item"].astype(np.int64)] >= 4)], minlength=8).tolist(),
            "could_win_read_cost4plus_by_cost": np.bincount(
                cost[can & (errs[c["item"].astype(np.int64)] >= 4)], minlength=8).tolist(),
        }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
