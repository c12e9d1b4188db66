#!/usr/bin/env python3
"""A/B: one GPU, the c2x24 batch split over S contexts (each its own HIP stream and buffers),
every context's two rounds enqueued from its own host thread per step, so the kernels of one
half can run beside the other half's latency-bound stages.  Prints ms per step and Mreads/s for
each S.  usage: python tools/ab_streams.py [reads] [steps] [S ...]"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nanopore-barcoding-orc_amd"))

import numpy as np  # noqa: E402

from dmx import lib, synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    variants = [int(x) for x in sys.argv[3:]] or [1, 2]
    t0 = time.perf_counter()
    d = synth.generate("c2x24", n=n, threads=16)
    print(f"generated {n} reads in {time.perf_counter() - t0:.1f} s", flush=True)
    ref = None
    for S in variants:
        cut = np.linspace(0, n, S + 1).astype(np.int64)
        ctxs = []
        for k in range(S):
            lo, hi = int(cut[k]), int(cut[k + 1])
            c = lib.Context(0)
            c.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC, 0.1)
            c.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC, 0.1)
            c.set_mode(lib.MODE_TWO_ROUND)
            c.load(lib.pack(d["blob"], d["offsets"][lo:hi], d["lengths"][lo:hi]))
            ctxs.append(c)

        def step():
            if S == 1:
                ctxs[0].exec()
                ctxs[0].sync()
                return
            th = [threading.Thread(target=lambda c=c: (c.exec(), c.sync())) for c in ctxs]
            for t in th:
                t.start()
            for t in th:
                t.join()

        for _ in range(2):
            step()
        t = time.perf_counter()
        for _ in range(steps):
            step()
        dt = (time.perf_counter() - t) / steps
        if S > 1:   # free-running: context k's loop starts k / S of a step late, no per-step join
            def loop(c, delay):
                time.sleep(delay)
                for _ in range(steps):
                    c.exec()
                    c.sync()
            th = [threading.Thread(target=loop, args=(c, k * dt / S)) for k, c in enumerate(ctxs)]
            t = time.perf_counter()
            for x in th:
                x.start()
            for x in th:
                x.join()
            dts = (time.perf_counter() - t) / steps
            print(f"S={S} staggered free-running: {dts * 1e3:.2f} ms/step  {n / dts / 1e6:.1f} "
                  "Mreads/s", flush=True)
        res = np.concatenate([c.fetch() for c in ctxs])
        same = None
        if ref is None:
            ref = res
        else:
            same = bool(np.array_equal(res.view(np.uint8), ref.view(np.uint8)))
        print(f"S={S}: {dt * 1e3:.2f} ms/step  {n / dt / 1e6:.1f} Mreads/s  results equal to S={variants[0]}: {same}",
              flush=True)
        for c in ctxs:
            c.close()


if __name__ == "__main__":
    main()
