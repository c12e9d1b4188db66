#!/usr/bin/env python3
"""HBM traffic per launch of the filter kernel from rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE collected in separate runs of `bench.py --steps 1 --warmup 0`).

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced read, so it
is doubled (the filter's loads are 16-B and 8-B per lane); WRITE_SIZE is taken as reported.
usage: traffic_from_pmc.py FETCH_DIR WRITE_DIR WORKLOAD READS OUT_JSON [KERNEL[@LAUNCH]]

KERNEL defaults to filter_kernel (every launch of one step is averaged).  For chop_kernel the run
also holds the small autotune launches, so only the largest launch (the timed 10M-read pass) is
kept; the same launch index is read from the WRITE_SIZE pass.  KERNEL@N keeps launch N of the
step (scan_kernel<true>@0: config 5's round-1 front scan, the bench line's dominant kernel).
"""
import collections
import csv
import json
import os
import sys


def per_dispatch(d, counter, kernel="filter_kernel"):
    acc = collections.OrderedDict()
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] != counter or kernel not in r["Kernel_Name"]:
            continue
        acc[int(r["Dispatch_Id"])] = acc.get(int(r["Dispatch_Id"]), 0.0) + float(
            r["Counter_Value"])
    return list(acc.values())


def main():
    fdir, wdir, workload, reads, out = sys.argv[1:6]
    kernel = sys.argv[6] if len(sys.argv) > 6 else "filter_kernel"
    launch = None
    if "@" in kernel:
        kernel, launch = kernel.split("@")
        launch = int(launch)
    fetch = per_dispatch(fdir, "FETCH_SIZE", kernel)
    write = per_dispatch(wdir, "WRITE_SIZE", kernel)
    if launch is not None:
        fetch, write = [fetch[launch]], [write[launch]]
    elif kernel != "filter_kernel":
        i = max(range(len(fetch)), key=fetch.__getitem__)
        fetch, write = [fetch[i]], [write[i]]
    n = min(len(fetch), len(write))
    per_launch = [2.0 * fetch[i] * 1024 + write[i] * 1024 for i in range(n)]
    data = {}
    if os.path.exists(out):
        data = json.load(open(out))
    data[f"{workload}:{reads}"] = {
        "bytes_per_launch": sum(per_launch) / n,
        "launches": [{"fetch_kib_raw": fetch[i], "write_kib": write[i],
                      "bytes": per_launch[i]} for i in range(n)],
        "source": ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), filter_kernel, "
                   "FETCH_SIZE x2 (gfx950 wide-read correction), averaged over the round-1 and "
                   "round-2 launches of one step") if kernel == "filter_kernel" else
                  (f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), {kernel}, "
                   + (f"launch {launch} of one step" if launch is not None else "the timed launch")
                   + "; FETCH_SIZE x2 (gfx950 wide-read correction, uncalibrated for "
                   "this kernel's 4-B loads, so an upper bound on reads)"),
    }
    with open(out, "w") as fh:
        json.dump(data, fh, indent=1)
        fh.write("\n")
    print(json.dumps(data[f"{workload}:{reads}"]))


if __name__ == "__main__":
    main()
