"""Host-side cost of one bench step beyond the device pipeline (c2x24, 10M reads by default):
times K steps of exec+sync, of exec+sync+stats, of exec+sync+RCCL count all-reduce, and of the
full bench step (all three), so the gap between the bench's ms_per_step and the device 'total'
stage can be attributed.  Usage: python tools/step_overhead.py [--reads N] [--steps K]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nanopore-barcoding-orc_amd"))

from dmx import lib, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reads", type=int, default=10_000_000)
ap.add_argument("--steps", type=int, default=5)
a = ap.parse_args()
d = synth.generate("c2x24", n=a.reads, threads=16)
packed = lib.pack(d["blob"], d["offsets"], d["lengths"])
ctx = lib.Context(0)
ctx.comm_init_rank(lib.comm_unique_id(), 1, 0)
ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC, 0.1)
ctx.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC, 0.1)
ctx.set_mode(lib.MODE_TWO_ROUND)
ctx.load(packed)
for _ in range(2):
    ctx.exec()
    ctx.sync()
    ctx.allreduce_counts()


def run(stats, allreduce):
    ctx.sync()
    t = time.perf_counter()
    dev = 0.0
    for _ in range(a.steps):
        ctx.exec()
        ctx.sync()
        if stats:
            dev += ctx.stats()["ms"]["total"]
        if allreduce:
            ctx.allreduce_counts()
    ctx.sync()
    return (time.perf_counter() - t) / a.steps * 1e3, dev / a.steps


for name, s, r in (("exec+sync", False, False), ("+stats", True, False),
                   ("+allreduce", False, True), ("bench step", True, True)) * 2:
    ms, dev = run(s, r)
    print(f"{name:12s} {ms:8.3f} ms/step" + (f"  device total {dev:.3f} ms" if s else ""),
          flush=True)
ctx.close()
