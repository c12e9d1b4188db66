#!/usr/bin/env python3
"""Per-kernel PMC table of one two-round step (rocprofv3 passes of tools/pmc_passes.sh over
`bench.py --steps 1 --warmup 0`): per launch of every pipeline kernel, its duration, VALU
instructions, HBM bytes, LDS instructions / bank-conflict cycles and the fraction of wave cycles
spent waiting.  bench.py reads the result to price each kernel's live time against the measured
VALU ceiling (profiles/r2_valu_ceiling.json).

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md: FETCH_SIZE / WRITE_SIZE are KiB;
FETCH_SIZE is doubled on gfx950 (the wide-read correction, calibrated in
profiles/r1_fetch_write_calibration.json; for kernels whose loads are narrower than 16 B per lane
the doubled figure is an upper bound).

usage: kernel_table_from_pmc.py P1 P2 P3 WORKLOAD READS OUT_JSON
  P1 = pass with FETCH_SIZE, SQ_INSTS_VALU; P2 = WRITE_SIZE, SQ_WAVE_CYCLES, SQ_WAIT_ANY;
  P3 = SQ_INSTS_LDS, SQ_LDS_BANK_CONFLICT.
"""
import collections
import csv
import json
import os
import sys

KERNELS = ("filter_kernel", "pscan_kernel<1>", "pscan_kernel<2>", "pscan_kernel<4>",
           "pcompact_kernel", "pscreen_kernel<1>", "pscreen_kernel<2>", "pscreen_kernel<4>",
           "ftask_kernel", "read_item_kernel", "read_view_kernel",
           "verify_kernel", "iscreen_kernel", "iscreen4_kernel",
           "wscan_kernel<true>", "band_cand_kernel<0, 3>", "band_cand_kernel<4, 5>",
           "band_cand_kernel<4, 7>", "select_cand_kernel", "finalize0_kernel", "finalize1_kernel",
           "chop_kernel", "scan_kernel<true>", "finalize0_linked_kernel",
           "finalize1_linked_kernel", "finalize2_linked_kernel")
# VALU lane-ops per shader cycle of the whole chip: 256 CUs x 4 SIMD x 32 lanes
VALU_LANES_PER_CLK = 256 * 4 * 32


def dispatches(d):
    acc = collections.OrderedDict()
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        name = r["Kernel_Name"]
        k = next((k for k in KERNELS if "::" + k + "(" in name or " " + k + "(" in name
                  or name.startswith(k + "(")), None)
        if k is None:
            continue
        ent = acc.setdefault(int(r["Dispatch_Id"]), {"kernel": k, "ms": (
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
        ent[r["Counter_Name"]] = ent.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(acc.values())


def main():
    p1, p2, p3, workload, reads, out = sys.argv[1:7]
    runs = [dispatches(p) for p in (p1, p2, p3)]
    table = collections.OrderedDict()
    for a, b, c in zip(*runs):
        assert a["kernel"] == b["kernel"] == c["kernel"], (a["kernel"], b["kernel"], c["kernel"])
        ent = table.setdefault(a["kernel"], [])
        valu = a["SQ_INSTS_VALU"]
        ent.append({
            "round": len(ent), "ms": round(a["ms"], 4),
            "valu_insts": valu,
            "valu_lane_ops_per_s": valu * 64 / (a["ms"] / 1e3),
            "hbm_bytes": 2.0 * a["FETCH_SIZE"] * 1024 + b["WRITE_SIZE"] * 1024,
            "fetch_kib_raw": a["FETCH_SIZE"], "write_kib": b["WRITE_SIZE"],
            "wait_frac": b["SQ_WAIT_ANY"] / max(1.0, b["SQ_WAVE_CYCLES"]),
            "lds_insts": c["SQ_INSTS_LDS"],
            "lds_conflict_cycles_per_inst": c["SQ_LDS_BANK_CONFLICT"] / max(1.0, c["SQ_INSTS_LDS"]),
        })
        if "GRBM_GUI_ACTIVE" in c:   # effective clock of this launch (pass 3's own duration)
            clk = c["GRBM_GUI_ACTIVE"] / 8.0 / (c["ms"] / 1e3)
            rate = valu * 64 / (c["ms"] / 1e3)
            ent[-1].update({"clock_ghz": clk / 1e9,
                            "valu_peak_at_clock": VALU_LANES_PER_CLK * clk,
                            "valu_frac_of_peak_at_clock": rate / (VALU_LANES_PER_CLK * clk)})
    data = {}
    if os.path.exists(out):
        data = json.load(open(out))
    data[f"{workload}:{reads}"] = {
        "kernels": table,
        "source": f"rocprofv3 --pmc passes {p1} {p2} {p3} (tools/pmc_passes.sh), one step; "
                  "FETCH_SIZE x2 gfx950 wide-read correction",
    }
    with open(out, "w") as fh:
        json.dump(data, fh, indent=1)
        fh.write("\n")
    for k, v in table.items():
        print(k, [(e["ms"], f"{e['valu_lane_ops_per_s'] / 1e12:.1f}T",
                   f"{e['hbm_bytes'] / 1e9:.2f}GB", f"wait {e['wait_frac']:.2f}",
                   f"lds {e['lds_conflict_cycles_per_inst']:.2f}",
                   f"clk {e.get('clock_ghz', 0):.2f}GHz",
                   f"valu@clk {e.get('valu_frac_of_peak_at_clock', 0):.2f}") for e in v])


if __name__ == "__main__":
    main()
