"""Host-side cost of the fused loop's per-batch planning and writing (dmx/loop.py run), on CPU.

The GPU step is replaced by a fake context group that returns random but consistent two-round
results (lib.RESULT_DTYPE; per-bin counts from the same results), so dmx/loop.py's own code runs
unchanged around it: plan_rounds, the per-output index/coordinate arrays, Sink.write and
_round_stats.  Prints the loop's DMX_PROFILE_IO line and the top of a cProfile listing.  Not a
GPU measurement: it isolates what the fused loop spends on the host per batch.
  python tools/plan_profile.py [--reads 1000000] [--threads 16] [-Z] [--workdir DIR]
"""
from __future__ import annotations

import argparse
import cProfile
import os
import pstats
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nanopore-barcoding-orc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from dmx import lib, loop, synth  # noqa: E402
from e2e_bench import write_fastq  # noqa: E402


class FakeContext:
    def set_panel(self, *a, **k):
        pass

    def set_mode(self, *a, **k):
        pass

    def close(self):
        pass


def fake_run_batch(seed=[0]):
    def run_batch(ctxs, packed):
        seed[0] += 1
        rng = np.random.default_rng(seed[0])
        lens = packed.lengths.astype(np.int64)
        n = len(lens)
        res = np.zeros(n, lib.RESULT_DTYPE)
        b1 = rng.integers(-1, 12, n)
        b2 = np.where(b1 >= 0, rng.integers(-1, 12, n), -1)
        res["bin1"], res["bin2"] = b1, b2
        res["rc1"] = rng.integers(0, 2, n)
        res["rc2"] = np.where(b2 >= 0, rng.integers(0, 2, n), 0)
        s1 = np.where(b1 >= 0, np.minimum(lens, rng.integers(20, 80, n)), 0)
        r2 = np.where(b2 >= 0, np.maximum(0, lens - s1 - rng.integers(20, 80, n)), 0)
        res["m1_rstop"], res["m2_rstart"] = s1, r2
        res["m1_errors"] = np.where(b1 >= 0, rng.integers(0, 3, n), 0)
        res["m2_errors"] = np.where(b2 >= 0, rng.integers(0, 3, n), 0)
        cnt = np.zeros(13 * 13, np.uint64)
        np.add.at(cnt, (b1 + 1) * 13 + (b2 + 1), 1)
        return res, cnt
    return run_batch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("-Z", action="store_true")
    ap.add_argument("--workdir", default=None)
    a = ap.parse_args()
    wd = a.workdir or tempfile.mkdtemp(prefix="dmx_plan_")
    path = os.path.join(wd, "pychopped", "pychopped_p.fastq")
    os.makedirs(os.path.dirname(path))
    write_fastq(path, synth.generate("c2", n=a.reads, seed=77), seed=5)
    lib.open_group = lambda devices: [FakeContext()]
    lib.run_batch = fake_run_batch()
    loop._devices = lambda args: [0]
    os.environ["DMX_PROFILE_IO"] = "1"
    pr = cProfile.Profile()
    pr.enable()
    rc = loop.run([path, "-j", str(a.threads), "--outdir", os.path.join(wd, "out")] +
                  (["-Z"] if a.Z else []))
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    print("rc", rc)


if __name__ == "__main__":
    main()
