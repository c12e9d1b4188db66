#!/usr/bin/env python3
"""Per-kernel L2 table from tools/pmc_l2.sh: for each launch of one step, L2 hit rate, fabric read
requests (one per 128-B line, profiles/r4_gather_calibration.json) and L1->L2 read requests.
usage: pmc_l2_summary.py OUTDIR"""
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
        hit = e["TCC_HIT_sum"] / max(1.0, e["TCC_HIT_sum"] + e["TCC_MISS_sum"])
        print(f"{e['k'][:34]:34s} {e['ms']:7.3f} ms  L2 hit {hit:.3f}  fabric lines "
              f"{e['TCC_EA0_RDREQ_sum'] / 1e6:8.1f} M ({e['TCC_EA0_RDREQ_sum'] * 128 / 1e9:6.2f} GB)  "
              f"L1->L2 reads {e['TCP_TCC_READ_REQ_sum'] / 1e6:8.1f} M  vmem insts "
              f"{e['SQ_INSTS_VMEM_RD'] / 1e6:7.1f} M")
