"""Host-side cost of one bench step around the kernels (exec + sync, the stats read-back, the
per-bin count exchange), on one GPU: where the wall-clock step time exceeds the stage events'
"total".  Usage: python tools/microbench/step_overhead.py [c4|c5|c2x24] [reads] [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..",
                                "nanopore-barcoding-orc_amd"))
from dmx import lib, synth  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c5"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2_000_000
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    d = synth.generate(wl, n=n, first=0, threads=16)
    packed = lib.pack(d["blob"], d["offsets"], d["lengths"])
    ctx = lib.Context(0)
    ctx.comm_init_rank(lib.comm_unique_id(), 1, 0)
    if wl == "c5":
        ctx.set_panel(0, d["sp5"], lib.DMX_FRONT, 0.1)
        ctx.set_panel(1, d["sp27"], lib.DMX_BACK, 0.1)
        ctx.set_mode(lib.MODE_LINKED)
    else:
        ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC, 0.1)
        ctx.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC, 0.1)
        ctx.set_mode(lib.MODE_TWO_ROUND)
    ctx.load(packed)
    for _ in range(3):
        ctx.exec()
        ctx.sync()
        ctx.allreduce_counts()

    def run(extra):
        ctx.sync()
        tot = 0.0
        t = time.perf_counter()
        for _ in range(steps):
            ctx.exec()
            ctx.sync()
            if "stats" in extra:
                tot += ctx.stats()["ms"]["total"]
            if "allreduce" in extra:
                ctx.allreduce_counts()
            if "counts" in extra:
                ctx.counts()
        ctx.sync()
        return (time.perf_counter() - t) * 1e3 / steps, tot / steps

    out = {"workload": wl, "reads": n, "steps": steps}
    for name, extra in (("exec_sync", ()), ("stats", ("stats",)),
                        ("stats_allreduce", ("stats", "allreduce")),
                        ("stats_counts", ("stats", "counts")),
                        ("allreduce_only", ("allreduce",))):
        ms, tot = run(extra)
        out[name] = {"ms_per_step": round(ms, 3)}
        if tot:
            out[name]["stage_total_ms"] = round(tot, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
