#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs per kernel dispatch (sums over XCDs/SEs).
usage: pmc_summary.py DIR [DIR...]"""
import collections
import csv
import sys

agg = collections.OrderedDict()
dur = {}
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        name = r["Kernel_Name"]
        if "rocclr" in name:
            continue
        key = (d.split("/")[-1], int(r["Dispatch_Id"]), name.split("(")[0])
        agg.setdefault(key, collections.defaultdict(float))[r["Counter_Name"]] += float(
            r["Counter_Value"])
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for k, v in agg.items():
    print(f"{k[0]} #{k[1]:3d} {k[2]:32s} {dur[k]:8.3f} ms  " +
          "  ".join(f"{a}={b:.3g}" for a, b in sorted(v.items())))
