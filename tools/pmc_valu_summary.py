#!/usr/bin/env python3
"""Summary of tools/pmc_valu.sh: per kernel (dispatches summed), the VALU issue counters and
their ratios.  lanes/inst = SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU x (ACTIVE cycles per
instruction of a full wave in the microbenchmark) — i.e. active lanes per VALU instruction;
active/insts = SQ_ACTIVE_INST_VALU per VALU instruction (issue cycles); valu share =
SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES.  The microbenchmark's kernels (every lane active, no
memory) give the normalisation.  usage: pmc_valu_summary.py OUTDIR"""
import collections
import csv
import glob
import json
import sys

out = sys.argv[1]
res = {}
for part in ("bench", "ilp"):
    files = glob.glob(f"{out}/{part}/**/run_counter_collection.csv", recursive=True) + \
        glob.glob(f"{out}/{part}/run_counter_collection.csv")
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    ndisp = collections.defaultdict(set)
    dur = collections.defaultdict(float)
    for f in files:
        seen = set()
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0]
            if "rocclr" in name:
                continue
            d = int(r["Dispatch_Id"])
            agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
            ndisp[name].add(d)
            if (name, d) not in seen:
                seen.add((name, d))
                dur[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    for k, v in agg.items():
        e = {c: v[c] for c in sorted(v)}
        e["dispatches"] = len(ndisp[k])
        e["ms"] = round(dur[k], 3)
        ai, iv = v.get("SQ_ACTIVE_INST_VALU", 0), v.get("SQ_INSTS_VALU", 0)
        if iv:
            e["active_cycles_per_valu_inst"] = round(ai / iv, 4)
        if ai:
            e["thread_cycles_per_active_cycle"] = round(v.get("SQ_THREAD_CYCLES_VALU", 0) / ai, 3)
        if v.get("SQ_WAVE_CYCLES"):
            e["valu_active_share_of_wave_cycles"] = round(ai / v["SQ_WAVE_CYCLES"], 4)
            e["wait_inst_any_share"] = round(v.get("SQ_WAIT_INST_ANY", 0) / v["SQ_WAVE_CYCLES"], 4)
        if v.get("GRBM_GUI_ACTIVE") and dur[k]:
            e["clock_ghz"] = round(v["GRBM_GUI_ACTIVE"] / 8 / (dur[k] * 1e-3) / 1e9, 3)
        res[f"{part}:{k}"] = e
print(json.dumps(res, indent=1))
