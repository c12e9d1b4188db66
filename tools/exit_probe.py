"""Where a dmx process's exit time goes: wall time of a child process minus the time it had run
when its last statement finished (/proc, 10 ms resolution), for children that
  touch   : touch --mb MB of anonymous memory (numpy) and exit
  context : open and close one device context (dmx/lib.py Context) and exit
  both    : both
  pinned  : a context that ran one 200k-read c2 batch (the loop's device and pinned buffers)
Prints one JSON line.  Usage: python tools/exit_probe.py [--mb 3000] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys, time
sys.path.insert(0, os.path.join(%(root)r, "nanopore-barcoding-orc_amd"))
import numpy as np
def since_exec():
    with open("/proc/self/stat") as fh:
        start = int(fh.read().rsplit(")", 1)[1].split()[19])
    with open("/proc/uptime") as fh:
        up = float(fh.read().split()[0])
    return up - start / os.sysconf("SC_CLK_TCK")
mode, mb = %(mode)r, %(mb)d
keep = []
if mode in ("touch", "both"):
    a = np.ones(mb << 17, np.float64)
    keep.append(a)
if mode in ("context", "both", "pinned"):
    from dmx import lib, synth
    ctx = lib.Context(0)
    if mode == "pinned":
        d = synth.generate("c2", n=200000, seed=1)
        p = lib.pack(d["blob"], d["offsets"], d["lengths"])
        ctx.set_panel(0, list(d["sp5"]), lib.DMX_FRONT | lib.DMX_RC, 0.1, 3)
        ctx.set_mode(lib.MODE_SINGLE)
        ctx.run(p)
    ctx.close()
print("END", since_exec(), flush=True)
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=3000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    out = {"mb": a.mb}
    for mode in ("touch", "context", "both", "pinned"):
        rows = []
        for _ in range(a.reps):
            t = time.perf_counter()
            p = subprocess.run([sys.executable, "-c", CHILD % dict(root=ROOT, mode=mode, mb=a.mb)],
                               capture_output=True, text=True)
            wall = time.perf_counter() - t
            end = [float(ln.split()[1]) for ln in p.stdout.splitlines() if ln.startswith("END")]
            if p.returncode or not end:
                rows.append({"error": p.stderr[-400:]})
                continue
            rows.append({"wall": round(wall, 3), "end": round(end[0], 3),
                         "exit": round(wall - end[0], 3)})
        out[mode] = rows
        print(mode, rows, file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
