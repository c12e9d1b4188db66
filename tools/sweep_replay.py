"""Replay the mismatching cases of a parity_sweep.json (their stored reads) on the GPU and the
oracle, printing both results per read.  python tools/sweep_replay.py gpurun_out/sweep.json [i]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "nanopore-barcoding-orc_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import oracle  # noqa: E402  (checker only)
import pyref  # noqa: E402
from dmx import lib  # noqa: E402

d = json.load(open(sys.argv[1]))
sel = [int(x) for x in sys.argv[2:]] or range(len(d["mismatches"]))
with lib.Context(0) as ctx:
    for ci in sel:
        m = d["mismatches"][ci]
        if m["kind"] != "random":
            continue
        seqs = m["bad_reads"]
        blob, offs, lens = oracle.pack_ascii(seqs)
        exp = oracle.run_batch(oracle.Panel(m["panel"], m["wheres"], max_errors=m["e"],
                                            min_overlap=m["min_overlap"]), None, blob, offs, lens,
                               mode=0, use_rc=m["rc"])
        ctx.set_panel_mixed(0, m["panel"], [lib.DMX_FRONT if w == oracle.FRONT else lib.DMX_BACK
                                            for w in m["wheres"]], m["rc"], m["e"],
                            m["min_overlap"])
        ctx.set_mode(lib.MODE_SINGLE)
        got = ctx.run(lib.pack(blob, offs, lens))
        print(f"case {ci}: e={m['e']} O={m['min_overlap']} rc={m['rc']} panel={m['panel']} "
              f"wheres={m['wheres']}")
        for i, s in enumerate(seqs):
            py = pyref.demux_round(m["panel"], m["wheres"], s, use_rc=m["rc"], e=m["e"])
            print(f"  read {s}\n    oracle {exp[i]}\n    gpu    {got[i]}\n    pyref  {py[:3]}")
