"""Cost of first-touching and of releasing large anonymous buffers with and without transparent
huge pages (madvise(MADV_HUGEPAGE)): a child maps --mb MB, fills it with numpy, and exits; the
parent reports the fill time and the exit time (wall minus the child's own run time, /proc).
Prints the host's THP settings and one JSON line.  Usage: python tools/thp_probe.py [--mb 3000]
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys
import time

CHILD = r"""
import mmap, os, time
import numpy as np
def since_exec():
    with open("/proc/self/stat") as fh:
        start = int(fh.read().rsplit(")", 1)[1].split()[19])
    with open("/proc/uptime") as fh:
        up = float(fh.read().split()[0])
    return up - start / os.sysconf("SC_CLK_TCK")
mb, huge = %(mb)d, %(huge)d
m = mmap.mmap(-1, mb << 20, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
if huge:
    m.madvise(mmap.MADV_HUGEPAGE)
a = np.frombuffer(m, np.uint8)
t = time.perf_counter()
a.fill(1)
fill = time.perf_counter() - t
ah = 0
with open("/proc/self/smaps_rollup") as fh:
    for ln in fh:
        if ln.startswith("AnonHugePages:"):
            ah = int(ln.split()[1]) >> 10
print("END", since_exec(), fill, ah, flush=True)
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=3000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    out = {"mb": a.mb}
    for k in ("enabled", "defrag"):
        try:
            with open(f"/sys/kernel/mm/transparent_hugepage/{k}") as fh:
                out["thp_" + k] = fh.read().strip()
        except OSError:
            out["thp_" + k] = None
    for huge in (0, 1):
        rows = []
        for _ in range(a.reps):
            t = time.perf_counter()
            p = subprocess.run([sys.executable, "-c", CHILD % dict(mb=a.mb, huge=huge)],
                               capture_output=True, text=True)
            wall = time.perf_counter() - t
            end = [ln.split()[1:] for ln in p.stdout.splitlines() if ln.startswith("END")]
            if p.returncode or not end:
                rows.append({"error": p.stderr[-300:]})
                continue
            ran, fill, ah = float(end[0][0]), float(end[0][1]), int(end[0][2])
            rows.append({"fill_s": round(fill, 3), "exit_s": round(wall - ran, 3),
                         "anon_huge_mb": ah})
        out["madv_hugepage" if huge else "default"] = rows
    print(json.dumps(out))


if __name__ == "__main__":
    main()
