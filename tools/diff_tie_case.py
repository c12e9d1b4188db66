"""Debug: rebuild test_tie_stress_short_adapters' data for (where, e, mo) and print the reads
where libdmx and the oracle differ.  python tools/diff_tie_case.py front 3 1"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "nanopore-barcoding-orc_amd"),
          os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import oracle  # noqa: E402  (checker only)
import pyref  # noqa: E402
import test_gpu_parity as T  # noqa: E402
from dmx import lib  # noqa: E402

where, e, mo = sys.argv[1], float(sys.argv[2]), int(sys.argv[3])
e = int(e) if e >= 1 else e
rng = np.random.default_rng({"front": 41, "back": 42, "mixed": 43}[where] + int(e * 100))
panel = T._random_panel(rng, 12, 3, 14, 0.1)
seqs = T._reads_with(rng, panel, 4000, L=(0, 60), err=0.1)
blob, offs, lens = oracle.pack_ascii(seqs)
if where == "mixed":
    wh = [oracle.FRONT if rng.random() < 0.5 else oracle.BACK for _ in panel]
else:
    wh = [oracle.FRONT if where == "front" else oracle.BACK] * len(panel)
exp = oracle.run_batch(oracle.Panel(panel, wh, max_errors=e, min_overlap=mo), None, blob, offs,
                       lens, mode=0, use_rc=True, threads=8)
with lib.Context(0) as ctx:
    ctx.set_panel_mixed(0, panel, [lib.DMX_FRONT if w == oracle.FRONT else lib.DMX_BACK
                                   for w in wh], True, e, mo)
    ctx.set_mode(lib.MODE_SINGLE)
    got = ctx.run(lib.pack(blob, offs, lens))
print("panel", panel, "wheres", wh)
g = got.view(np.uint8).reshape(len(got), -1)
x = exp.view(np.uint8).reshape(len(exp), -1)
bad = np.nonzero((g != x).any(axis=1))[0]
print(len(bad), "differ")
for i in bad[:8]:
    print("read", repr(seqs[i]))
    print("  oracle", exp[i])
    print("  gpu   ", got[i])
    py = pyref.demux_round(panel, wh, seqs[i], use_rc=True, e=e, min_overlap=mo) \
        if "min_overlap" in pyref.demux_round.__code__.co_varnames else None
    print("  pyref ", py[:3] if py else None)
