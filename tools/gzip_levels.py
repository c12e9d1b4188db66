"""Size and speed of the gzip writers' members against zlib and libdeflate, per level, on
nanopore-style FASTQ (tests/fastq_like.py) and on the c2 synthetic FASTQ of the e2e bench
(tools/e2e_bench.py write_fastq: short "@r<i> ch=<k>" headers, uniform qualities, reads that
carry the SP5/SP27 barcodes).  Members of 1 MiB, as the writers cut them (dmx_io.cpp
kMemberMax); one thread; decode speed with zlib (what a downstream `gzip -d` / Python reader
pays).  libdeflate rows come from a child process with DMX_GZIP_LIBDEFLATE=1 (the writers'
previous level-2..9 path).

Usage: python tools/gzip_levels.py [--mb 48] [--out profiles/r5_gzip_levels.json]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nanopore-barcoding-orc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

M = 1 << 20


def _members(data, fn):
    t = time.perf_counter()
    mem = [fn(data[k:k + M]) for k in range(0, len(data), M)]
    dt = time.perf_counter() - t
    t = time.perf_counter()
    for m in mem:
        zlib.decompress(m, 47)
    dd = time.perf_counter() - t
    size = sum(map(len, mem))
    return {"ratio": round(len(data) / size, 4), "bytes": size,
            "compress_MB_s": round(len(data) / dt / 1e6, 1),
            "zlib_inflate_MB_s": round(len(data) / dd / 1e6, 1)}


def dmx_rows(path, levels):
    from dmx import nio
    data = open(path, "rb").read()
    return {str(lv): _members(data, lambda x, lv=lv: nio.gzip_member(x, lv)) for lv in levels}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=48)
    ap.add_argument("--out", default=None)
    ap.add_argument("--dmx-child", nargs=2, metavar=("PATH", "LEVELS"))
    a = ap.parse_args()
    if a.dmx_child:
        print(json.dumps(dmx_rows(a.dmx_child[0], [int(x) for x in a.dmx_child[1].split(",")])))
        return
    from e2e_bench import write_fastq
    from fastq_like import nanopore_fastq

    from dmx import synth
    wd = tempfile.mkdtemp(prefix="dmx_gzl_")
    sets = {}
    p = os.path.join(wd, "nanopore_like.fastq")
    with open(p, "wb") as fh:
        fh.write(nanopore_fastq(a.mb << 20, seed=1))
    sets["nanopore_like"] = p
    p = os.path.join(wd, "c2_synthetic.fastq")
    d = synth.generate("c2", n=max(1000, (a.mb << 20) // 2400), seed=77)
    write_fastq(p, d, seed=5)
    sets["c2_synthetic"] = p
    res = {"member_bytes": M, "threads": 1, "host": os.uname().nodename,
           "note": "one thread of the build container's CPU; ratios are what matter, speeds "
                   "compare the encoders on the same core"}
    for name, path in sets.items():
        data = open(path, "rb").read()
        row = {"bytes": len(data)}
        for lv in (1, 5, 6, 9):
            row[f"zlib_{lv}"] = _members(data, lambda x, lv=lv: zlib.compress(x, lv))
        ours = json.loads(subprocess.run([sys.executable, __file__, "--dmx-child", path, "1,5,9"],
                                         check=True, stdout=subprocess.PIPE, text=True).stdout)
        row["dmx_1_huffman_only"] = ours["1"]
        row["dmx_5_record_aware"] = ours["5"]
        row["dmx_9_record_aware"] = ours["9"]
        env = dict(os.environ, DMX_GZIP_LIBDEFLATE="1")
        ld = json.loads(subprocess.run([sys.executable, __file__, "--dmx-child", path, "5,9"],
                                       check=True, stdout=subprocess.PIPE, text=True,
                                       env=env).stdout)
        row["libdeflate_5"] = ld["5"]
        row["libdeflate_9"] = ld["9"]
        res[name] = row
        os.remove(path)
    os.rmdir(wd)
    line = json.dumps(res)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)
    print(line)


if __name__ == "__main__":
    main()
