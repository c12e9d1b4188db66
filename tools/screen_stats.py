"""Shape of the index screen's work (GPU box): per round, the verified windows the packed screen
reads (iscreen4_kernel: one lane per (window, quad of adapters), 64 consecutive lanes per wave),
the 16-column chunks each lane scans, and how much of a wave's time its longest lane sets.

    python tools/screen_stats.py [--workload c2x24] [--reads 2000000]
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
    return min(k, 32)


def shape(w, ads, front: bool, rate: float):
    """Chunks per lane as iscreen4_kernel computes its column range (rows / last-column tests),
    ignoring the early exit once every adapter of the quad passes."""
    pl, sl = common(ads, False), common(ads, True)
    ms = np.array([len(s) for s in ads])
    kk = np.array([int(rate * m) for m in ms])
    kf = int(kk.max())
    ls = ms - pl - sl
    jsplit = int((ms - pl + kk).max()) if front else 0
    j1 = w["j1"].astype(np.int64)
    j2 = w["j2"].astype(np.int64)
    ln = w["len"].astype(np.int64)
    lastc = (~np.bool_(front)) & (w["lastcol"] != 0)
    jr = np.maximum(j1, jsplit)
    rows = (w["bmin"] != 255) & (jr <= j2)
    x1 = np.full(len(w), 1 << 30, np.int64)
    x1 = np.where(rows, jr - int(ls.max()) - sl - kf, x1)
    x1 = np.where(lastc, np.minimum(x1, ln - (int(ms.max()) - 1 - pl) - kf), x1)
    xe = np.where(rows, np.minimum(j2 - sl + kf, ln), -1)
    xe = np.where(lastc, ln, xe)
    need = rows | lastc
    nch = np.where(need, np.maximum(0, (xe - x1 + 15) // 16), 0)
    q = (len(ads) + 3) // 4
    lanes = np.repeat(nch, q)
    n = len(lanes) // 64 * 64
    waves = lanes[:n].reshape(-1, 64)
    # the same lanes sorted by chunk count inside each block iteration (256 lanes)
    nb = len(lanes) // 256 * 256
    srt = np.sort(lanes[:nb].reshape(-1, 256), axis=1).reshape(-1, 64)
    return {"windows": int(len(w)), "lanes": int(len(lanes)),
            "width_pcts": np.percentile(j2 - j1 + 1, [50, 90, 99, 99.9, 100]).tolist(),
            "chunks_lane_mean": float(lanes.mean()),
            "chunks_pcts": np.percentile(nch, [50, 90, 99, 99.9, 100]).tolist(),
            "no_scan_frac": float((nch == 0).mean()),
            "wave_max_mean": float(waves.max(axis=1).mean()),
            "wave_max_over_mean": float(waves.max(axis=1).sum() / max(1, waves.mean(axis=1).sum())),
            "wave_max_over_mean_block_sorted": float(srt.max(axis=1).sum() /
                                                     max(1, srt.mean(axis=1).sum())),
            "lastcol_frac": float(lastc.mean()),
            "params": {"pre_len": pl, "filter_len": sl, "kf": kf, "jsplit": jsplit,
                       "index_len": [int(ls.min()), int(ls.max())]}}


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
        # the rounds share the list buffers: round 1's lists after a single-round exec
        for rnd, mode, ads, front in ((0, lib.MODE_SINGLE, d["sp5"], True),
                                      (1, lib.MODE_TWO_ROUND, d["sp27"], False)):
            ctx.set_mode(mode)
            ctx.exec()
            ctx.sync()
            w = ctx.debug_fetch(lib.DBG_VERIFIED, rnd)
            out[f"round{rnd}"] = shape(w, ads, front, 0.1)
            out[f"round{rnd}"]["ms"] = ctx.stats()["ms"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
