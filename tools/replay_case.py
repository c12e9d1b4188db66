#!/usr/bin/env python3
"""Replay one synthetic parity-sweep case (tools/parity_sweep.py case_synth) against the oracle.
usage: python tools/replay_case.py CONFIG SEED N E   (run with DMX_DEBUG_SYNC=1 to name the
kernel of a device fault)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "nanopore-barcoding-orc_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

import oracle  # noqa: E402  (checker only)
from dmx import lib, synth  # noqa: E402


def main():
    cfg, seed, n, e = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4])
    d = synth.generate(cfg, n=n, seed=seed)
    linked = cfg == "c5"
    lens = d["lengths"]
    print(f"{cfg} seed {seed} n {n} e {e}: reads {len(lens)}, len {int(lens.min())}.."
          f"{int(lens.max())}, panels {len(d['sp5'])} x {len(d['sp27'])}", flush=True)
    p1 = oracle.Panel(d["sp5"], oracle.FRONT, max_errors=e)
    p2 = oracle.Panel(d["sp27"], oracle.BACK, max_errors=e)
    exp = oracle.run_batch(p1, p2, d["blob"], d["offsets"], d["lengths"], mode=2 if linked else 1,
                           use_rc=not linked, threads=16)
    f = 0 if linked else lib.DMX_RC
    with lib.Context(0) as ctx:
        ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | f, e)
        ctx.set_panel(1, d["sp27"], lib.DMX_BACK | f, e)
        ctx.set_mode(lib.MODE_LINKED if linked else lib.MODE_TWO_ROUND)
        got = ctx.run(lib.pack(d["blob"], d["offsets"], d["lengths"]))
    g = got.view(np.uint8).reshape(len(got), -1)
    x = exp.view(np.uint8).reshape(len(exp), -1)
    bad = np.nonzero((g != x).any(axis=1))[0]
    print(f"ok: {len(bad)} mismatching reads", flush=True)
    sys.exit(1 if len(bad) else 0)


if __name__ == "__main__":
    main()
