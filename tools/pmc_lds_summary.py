#!/usr/bin/env python3
"""Per-kernel LDS table from tools/pmc_lds.sh: for each launch of one step, LDS instructions,
bank-conflict cycles per LDS instruction, and the share of wave cycles spent waiting on LDS.
usage: pmc_lds_summary.py OUTDIR"""
import collections
import csv
import glob
import os
import sys

for d in sorted(glob.glob(os.path.join(sys.argv[1], "*", "run_counter_collection.csv"))):
    acc = collections.OrderedDict()
    for r in csv.DictReader(open(d)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dmx::", "")
        e = acc.setdefault(int(r["Dispatch_Id"]), {"k": name, "ms": (
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    print(f"== {os.path.basename(os.path.dirname(d))}")
    for e in acc.values():
        if e["ms"] < 0.15:
            continue
        lds = max(1.0, e["SQ_INSTS_LDS"])
        print(f"{e['k'][:34]:34s} {e['ms']:7.3f} ms  LDS insts {e['SQ_INSTS_LDS'] / 1e6:8.1f} M  "
              f"conflict cycles / LDS inst {e['SQ_LDS_BANK_CONFLICT'] / lds:5.2f}  "
              f"LDS wait / wave cycles {e['SQ_WAIT_INST_LDS'] / max(1.0, e['SQ_WAVE_CYCLES']):5.3f}  "
              f"VALU {e['SQ_INSTS_VALU'] / 1e9:6.2f} G")
