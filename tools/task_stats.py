"""Shape of the window-scan work (GPU box): per round, the (window piece, adapter) tasks the
index screen passes, their column counts, and how much of a wave's time the longest lane sets
(tasks run one per lane, 64 consecutive list entries per wave, so a wave costs its longest task).

    python tools/task_stats.py [--workload c2x24] [--reads 2000000]
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


def shape(t, m_of, k):
    """Columns per task: js = j1 - m - k - 1 (clamped at 0) .. j2."""
    m = m_of[t["info"].astype(np.int64)]
    js = np.maximum(t["j1"].astype(np.int64) - m - k - 1, 0)
    cols = t["j2"].astype(np.int64) - js
    width = t["j2"].astype(np.int64) - t["j1"].astype(np.int64) + 1
    n = len(cols) // 64 * 64
    waves = cols[:n].reshape(-1, 64)
    srt = {}
    for blk in (256, 1024):   # sorted by column count inside groups of `blk` consecutive tasks
        nb = len(cols) // blk * blk
        sw = np.sort(cols[:nb].reshape(-1, blk), axis=1).reshape(-1, 64)
        srt[blk] = float(sw.max(axis=1).sum() / max(1, sw.mean(axis=1).sum()))
    return {"wave_max_over_mean_sorted_256": srt[256], "wave_max_over_mean_sorted_1024": srt[1024],"tasks": int(len(t)), "cols_mean": float(cols.mean()),
            "cols_pcts": np.percentile(cols, [50, 90, 99, 99.9, 100]).tolist(),
            "width_pcts": np.percentile(width, [50, 90, 99, 99.9, 100]).tolist(),
            "lastcol_frac": float((t["lastcol"] != 0).mean()),
            "wave_max_over_mean": float(waves.max(axis=1).sum() / max(1, waves.mean(axis=1).sum())),
            "cols_total": int(cols.sum()),
            "cols_wave_max_total": int(waves.max(axis=1).sum() * 64)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2x24")
    ap.add_argument("--reads", type=int, default=2_000_000)
    a = ap.parse_args()
    d = synth.generate(a.workload, n=a.reads, threads=16)
    out = {"workload": a.workload, "reads": a.reads}
    with lib.Context(0) as ctx:
        ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC, 0.1)
        ctx.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC, 0.1)
        ctx.load(lib.pack(d["blob"], d["offsets"], d["lengths"]))
        for rnd, mode in ((0, lib.MODE_SINGLE), (1, lib.MODE_TWO_ROUND)):
            ctx.set_mode(mode)
            ctx.exec()
            ctx.sync()
            ads = d["sp5"] if rnd == 0 else d["sp27"]
            m_of = np.array([len(s) for s in ads], dtype=np.int64)
            k = 5
            out[f"round{rnd}"] = {
                "tasks": shape(ctx.debug_fetch(lib.DBG_TASKS, rnd), m_of, k),
                "verified_windows": int(len(ctx.debug_fetch(lib.DBG_VERIFIED, rnd))),
                "stats": ctx.stats()["ms"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
