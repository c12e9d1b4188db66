#!/usr/bin/env python3
"""Debug one read of a replay case (GPU box): windows, verified windows and wscan tasks of that
read, with the piece screen on and off, over the whole case and over the read alone.

usage: python tools/debug_case.py CASE_JSON READ_INDEX
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nanopore-barcoding-orc_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402  (its Where constants only)
from dmx import lib  # noqa: E402


def run(p, seqs, item, tag):
    blob = "".join(seqs).encode()
    lens = np.array([len(s) for s in seqs], dtype=np.uint32)
    offs = np.zeros(len(seqs), dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1])
    with lib.Context(0) as ctx:
        ctx.set_panel_mixed(0, p["panel"], [lib.DMX_FRONT if w == oracle.FRONT else lib.DMX_BACK
                                            for w in p["wheres"]], p["rc"], p["e"],
                            p["min_overlap"])
        ctx.set_mode(lib.MODE_SINGLE)
        got = ctx.run(lib.pack(np.frombuffer(blob, dtype=np.uint8), offs, lens))
        print(f"== {tag}: result {got[item]}")
        for what, name in ((lib.DBG_WINDOWS, "windows"), (lib.DBG_VERIFIED, "verified"),
                           (lib.DBG_TASKS, "tasks")):
            d = ctx.debug_fetch(what, 0)
            sel = d[d["item"] == item]
            print(f"  {name}: {len(d)} total, {len(sel)} for item")
            for r in sel[:40]:
                print("   ", {k: int(r[k]) for k in d.dtype.names})


def main():
    c = json.load(open(sys.argv[1]))
    i = int(sys.argv[2])
    p, seqs = c["params"], c["reads"]
    run(p, seqs, i, "all reads, pieces on")
    run(p, [seqs[i]], 0, "read alone, pieces on")
    os.environ["DMX_NO_PIECES"] = "1"
    run(p, seqs, i, "all reads, pieces off")


if __name__ == "__main__":
    main()
