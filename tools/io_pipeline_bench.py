"""CPU-only timing and peak RSS of the host I/O of a 02_cutadapt_loop.sh round-1 call, without
the GPU: an ordinary single-member FASTQ.gz (what pychopped_<ds>.gz is) read by dmx_reader and
every read written to one of 13 gzip outputs (12 bins + unknown, as the SP5 call writes) by
dmx_sink at cutadapt's default level 5.  The demux itself (about 0.07 s of GPU time per 1 M
reads, profiles/r4_e2e_c2_1M_final.json) is replaced by a fixed assignment, read i -> output
i mod 13, so what is timed is what the round-1 call's read_wait and plan_write measure.

Modes (each in a child process of its own, so its peak RSS is its own):
  inflate  : read the .gz, drop the batches           (inflate + parse + pack)
  compress : read the plain FASTQ, write level 5      (parse + pack + render + compress)
  pipeline : read the .gz, write level 5              (the round-1 call's host work)
The sum of the first two, in core-seconds, over the thread count is the floor for the third.

Usage: python tools/io_pipeline_bench.py [--reads 250000] [--threads 8] [--workdir DIR]
                                         [--modes inflate,compress,pipeline] [--keep]
One JSON line: wall seconds, CPU seconds (user + sys) and peak RSS (MB) per mode.
"""
from __future__ import annotations

import argparse
import json
import os
import resource
import subprocess
import sys
import tempfile
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nanopore-barcoding-orc_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "tools"))

N_OUT = 13


def child(mode: str, src: str, outdir: str, threads: int, level: int, batch_mb: int = 0):
    from dmx import nio
    batch = (batch_mb << 20) if batch_mb > 0 else nio.batch_bytes_for_budget()
    t = time.perf_counter()
    waits = 0.0
    sink = None
    if mode != "inflate":
        os.makedirs(outdir, exist_ok=True)
        sink = nio.Sink([os.path.join(outdir, f"o{k}.fastq.gz") for k in range(N_OUT)], False,
                        level, threads=threads)
    n = base = 0
    with nio.Reader(src, batch, threads=threads) as r:
        while True:
            tw = time.perf_counter()
            b = r.next()
            waits += time.perf_counter() - tw
            if b is None:
                break
            k = len(b)
            if sink is not None:
                idx = ((np.arange(k, dtype=np.int64) + base) % N_OUT).astype(np.int32)
                z = np.zeros(k, np.uint8)
                sink.write(b, idx, np.zeros(k, np.int32), b.lens.astype(np.int32), z, z)
            b.free()
            n += k
            base += k
    if sink is not None:
        sink.close()
    wall = time.perf_counter() - t
    ru = resource.getrusage(resource.RUSAGE_SELF)
    # VmHWM, not ru_maxrss: after execve ru_maxrss keeps the forking parent's peak
    hwm = 0
    with open("/proc/self/status") as fh:
        for line in fh:
            if line.startswith("VmHWM:"):
                hwm = int(line.split()[1])
    print(json.dumps({"reads": n, "wall_s": round(wall, 3), "read_wait_s": round(waits, 3),
                      "cpu_s": round(ru.ru_utime + ru.ru_stime, 2),
                      "peak_rss_mb": round(hwm / 1024, 1)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=250_000)
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--level", type=int, default=5)
    ap.add_argument("--batch-mb", type=int, default=0,
                    help="default: 256, less under DMX_MEM_BUDGET_MB (nio.batch_bytes_for_budget)")
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--modes", default="inflate,compress,pipeline")
    ap.add_argument("--keep", action="store_true", help="keep the generated inputs")
    ap.add_argument("--child", nargs=3, metavar=("MODE", "SRC", "OUTDIR"))
    a = ap.parse_args()
    if a.child:
        child(a.child[0], a.child[1], a.child[2], a.threads, a.level, a.batch_mb)
        return
    from dmx import synth
    from e2e_bench import write_fastq
    wd = a.workdir or tempfile.mkdtemp(prefix="dmx_iob_")
    os.makedirs(wd, exist_ok=True)
    plain = os.path.join(wd, "in.fastq")
    gz1 = plain + ".gz"
    tag = f"{a.workload}_{a.reads}"
    stamp = os.path.join(wd, "inputs.txt")
    if not (os.path.exists(stamp) and open(stamp).read() == tag):
        d = synth.generate(a.workload, n=a.reads, seed=77)
        write_fastq(plain, d, seed=5)
        with open(plain, "rb") as fi, open(gz1, "wb") as fo:   # `gzip -1`-like single member
            c = zlib.compressobj(1, zlib.DEFLATED, 31, 8, zlib.Z_DEFAULT_STRATEGY)
            while True:
                chunk = fi.read(64 << 20)
                if not chunk:
                    break
                fo.write(c.compress(chunk))
            fo.write(c.flush())
        with open(stamp, "w") as fh:
            fh.write(tag)
    res = {"reads": a.reads, "threads": a.threads, "level": a.level, "batch_mb": a.batch_mb,
           "mem_budget_mb": os.environ.get("DMX_MEM_BUDGET_MB", ""),
           "fastq_bytes": os.path.getsize(plain), "gz_single_bytes": os.path.getsize(gz1)}
    env = dict(os.environ)
    for mode in a.modes.split(","):
        src = plain if mode == "compress" else gz1
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--threads",
                            str(a.threads), "--level", str(a.level), "--batch-mb", str(a.batch_mb),
                            "--child", mode, src,
                            os.path.join(wd, "out_" + mode)], check=True, env=env,
                           stdout=subprocess.PIPE, text=True)
        res[mode] = json.loads(p.stdout.strip().splitlines()[-1])
    if "inflate" in res and "compress" in res:
        floor = (res["inflate"]["cpu_s"] + res["compress"]["cpu_s"]) / a.threads
        res["pipeline_floor_s"] = round(floor, 3)
    if not a.keep and not a.workdir:
        subprocess.run(["rm", "-rf", wd], check=False)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
