#!/usr/bin/env python3
"""Summary of tools/microbench/run_gather_calib.sh: per kernel, the lines it touched (each once),
FETCH_SIZE and TCC_EA0_RDREQ of its second (timed) dispatch, bytes counted per line, and the
factor that turns FETCH_SIZE into bytes delivered for that access width (128 B per line: the
whole line must cross the fabric whatever the request size, so FETCH_SIZE x factor = 128 B per
line; the request size itself is RDREQ per line).  usage: gather_calib_summary.py OUTDIR"""
import collections
import csv
import glob
import json
import re
import sys

out = sys.argv[1]
plain = open(f"{out}/plain.log").read()
ms = {m.group(1): float(m.group(2)) for m in re.finditer(r"^(\w+) lines \d+ ms ([\d.]+)", plain,
                                                          re.M)}
LINES = 1 << 24
cnt = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/**/run_counter_collection.csv", recursive=True) + \
        glob.glob(f"{out}/p*/run_counter_collection.csv"):
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"])
        per[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        names[k] = r["Kernel_Name"].split("(")[0]
    for (k, c), v in per.items():
        cnt[names[k]][c].append((k, v))
res = {"what": "FETCH_SIZE calibration for gathers on gfx950 (tools/microbench/gather_calib.hip): "
               "every 128-B line of a 2 GiB buffer touched once, scattered",
       "kernels": {}}
for kern, cs in sorted(cnt.items()):
    e = {"ms_timed_launch": ms.get(kern)}
    for c, vs in cs.items():
        v = sorted(vs)[-1][1]            # the second (timed) dispatch
        e[c] = v
    if "FETCH_SIZE" in e:
        fb = e["FETCH_SIZE"] * 1024.0    # rocprofv3 reports KiB
        if kern == "stream16":
            e["fetch_factor_vs_bytes_read"] = round((LINES * 128) / fb, 4)
        else:
            e["fetch_bytes_per_line"] = round(fb / LINES, 2)
            e["fetch_factor_vs_128B_lines"] = round(LINES * 128 / fb, 4)
    for c in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ"):
        if c in e:
            e["rdreq_per_line"] = round(e[c] / LINES, 3)
    res["kernels"][kern] = e
print(json.dumps(res, indent=1))
