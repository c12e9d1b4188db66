"""Peak RSS (VmHWM) of the fused loop under memory budgets, and of its fixed part (interpreter,
numpy, HIP runtime, libdmx's code objects, one context), for ADVICE r4's 2G / 4G job limits.

Generates `--reads` c2 reads as an ordinary single-member FASTQ.gz (what 01_pychopper.sh /
02_cutadapt_loop.sh read), then runs bin/dmx-demux-loop on it (with --reorient: the 01 -> 02
fused path) once per (budget, batch) setting and reports the peak RSS and wall time of each
from its DMX_PROFILE_IO line.  Needs the GPU.

Usage: python tools/rss_probe.py [--reads 300000] [--threads 24]
           [--settings 2048:0,2048:64,4096:0,0:0]   (budget MB : batch MB, 0 = default)
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nanopore-barcoding-orc_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "tools"))

BASE = r"""
import os, sys, json
sys.path.insert(0, %r)
from dmx import lib, nio, synth
out = {"after_import_mb": nio.peak_rss_mb()}
d = synth.generate("c2", n=20000, seed=3)
pk = lib.pack(d["blob"], d["offsets"], d["lengths"])
out["after_synth_pack_mb"] = nio.peak_rss_mb()
ctx = lib.Context(0)
out["after_context_mb"] = nio.peak_rss_mb()
ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC)
ctx.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC)
ctx.set_mode(lib.MODE_TWO_ROUND)
out["after_panels_mb"] = nio.peak_rss_mb()
ctx.run(pk)
out["after_first_run_mb"] = nio.peak_rss_mb()
out.update({"now_" + k + "_mb": v for k, v in nio.rss_parts_mb().items()})
d = synth.generate("c2", n=200000, seed=4)
pk = lib.pack(d["blob"], d["offsets"], d["lengths"])
out["after_synth_pack_200k_mb"] = nio.peak_rss_mb()
ctx.run(pk)
out["after_run_200k_mb"] = nio.peak_rss_mb()
print(json.dumps({k: round(v) for k, v in out.items()}))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=300_000)
    ap.add_argument("--threads", type=int, default=24)
    ap.add_argument("--settings", default="2048:0,2048:64,2048:32,4096:0,0:0")
    ap.add_argument("--no-reorient", action="store_true")
    a = ap.parse_args()
    from e2e_bench import write_fastq

    from dmx import synth
    wd = tempfile.mkdtemp(prefix="dmx_rss_")
    plain = os.path.join(wd, "raw.fastq")
    write_fastq(plain, synth.generate("c2", n=a.reads, seed=77), seed=5)
    gz = plain + ".gz"
    with open(plain, "rb") as fi, open(gz, "wb") as fo:
        c = zlib.compressobj(1, zlib.DEFLATED, 31)
        while True:
            chunk = fi.read(64 << 20)
            if not chunk:
                break
            fo.write(c.compress(chunk))
        fo.write(c.flush())
    os.remove(plain)
    base = subprocess.run([sys.executable, "-c", BASE % PKG], check=True, stdout=subprocess.PIPE,
                          text=True).stdout.strip().splitlines()[-1]
    res = {"reads": a.reads, "threads": a.threads, "gz_bytes": os.path.getsize(gz),
           "reorient": not a.no_reorient, "fixed": json.loads(base), "runs": []}
    print(json.dumps(res["fixed"]), flush=True)
    for k, st in enumerate(a.settings.split(",")):
        budget, batch = (int(x) for x in st.split(":"))
        env = dict(os.environ, DMX_PROFILE_IO="1")
        env.pop("DMX_MEM_BUDGET_MB", None)
        env.pop("DMX_BATCH_MB", None)
        if budget:
            env["DMX_MEM_BUDGET_MB"] = str(budget)
        if batch:
            env["DMX_BATCH_MB"] = str(batch)
        out = os.path.join(wd, f"o{k}")
        cmd = [os.path.join(PKG, "bin", "dmx-demux-loop"), gz, "-j", str(a.threads),
               "--outdir", out]
        if not a.no_reorient:
            cmd += ["--reorient", "--pychopper-dir", os.path.join(wd, f"p{k}")]
        t = time.perf_counter()
        p = subprocess.run(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                           text=True)
        dt = time.perf_counter() - t
        prof = [ln for ln in p.stderr.splitlines() if ln.startswith("io profile")]
        m = re.search(r"peak_rss_mb (\d+)", prof[-1]) if prof else None
        row = {"budget_mb": budget or None, "batch_mb": batch or None, "rc": p.returncode,
               "wall_s": round(dt, 3), "peak_rss_mb": int(m.group(1)) if m else None,
               "profile": prof[-1] if prof else p.stderr[-400:]}
        res["runs"].append(row)
        print(json.dumps(row), flush=True)
        subprocess.run(["rm", "-rf", out, os.path.join(wd, f"p{k}")], check=False)
    subprocess.run(["rm", "-rf", wd], check=False)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
