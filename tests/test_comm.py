"""RCCL per-bin count exchange inside libdmx (include/dmx.h "Multi-GPU count exchange";
SURVEY.md §8b/§8e, §4.4: on a box with fewer GPUs, RCCL runs with a single-rank communicator).

The counts of a config-2 (24 x 24 panel) run, reduced in HBM by ncclAllReduce, must equal the
counts derived on the host from the per-read results, and the oracle's."""
import numpy as np
import pytest

import oracle
from dmx import lib, synth

pytestmark = pytest.mark.gpu


def host_counts(res, a0, a1):
    """dmx_counts layout from per-read results: bins, then the RC counts of both rounds."""
    c = np.zeros((a0 + 1) * (a1 + 1) + 2, dtype=np.int64)
    idx = (res["bin1"].astype(np.int64) + 1) * (a1 + 1) + (res["bin2"].astype(np.int64) + 1)
    np.add.at(c, idx, 1)
    c[-2] = int(res["rc1"].sum())
    c[-1] = int(res["rc2"][res["bin1"] >= 0].sum())
    return c


def _setup(ctx, d):
    ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC)
    ctx.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC)
    ctx.set_mode(lib.MODE_TWO_ROUND)


@pytest.fixture(scope="module")
def c2x24():
    d = synth.generate("c2x24", n=30000, seed=12)
    return d, lib.pack(d["blob"], d["offsets"], d["lengths"])


def test_single_rank_comm_allreduce_counts(c2x24):
    d, p = c2x24
    with lib.Context(0) as ctx:
        _setup(ctx, d)
        ctx.comm_init_rank(lib.comm_unique_id(), 1, 0)
        assert ctx.comm_size() == 1
        ctx.load(p)
        for _ in range(2):   # a second exec starts from fresh counts
            ctx.exec()
            local = ctx.counts()
            reduced = ctx.allreduce_counts()
            assert reduced.tolist() == local.tolist()
        res = ctx.fetch()
        a0, a1 = ctx.panel_sizes
        assert reduced.tolist() == host_counts(res, a0, a1).tolist()
        assert reduced[(a0 + 1) * (a1 + 1):].sum() > 0      # RC counts exercised
        assert ctx.counts().tolist() == reduced.tolist()     # dmx_counts returns the sum


def test_comm_group_run_multi_counts_match_oracle(c2x24):
    """dmx_comm_init_all over the box's devices (one here): dmx_run_multi reduces its counts
    with a grouped ncclAllReduce; results and counts vs the oracle."""
    d, p = c2x24
    ctxs = [lib.Context(0)]
    try:
        assert lib.comm_init_all(ctxs)
        _setup(ctxs[0], d)
        res, counts = lib.run_multi(ctxs, p)
        res2, counts2 = lib.run_batch(ctxs, p)      # the CLI / fused-loop path
    finally:
        for c in ctxs:
            c.close()
    p1, p2 = oracle.Panel(d["sp5"], oracle.FRONT), oracle.Panel(d["sp27"], oracle.BACK)
    sub = 6000   # oracle on a prefix (seconds); counts of the whole batch vs the host sum
    exp = oracle.run_batch(p1, p2, d["blob"], d["offsets"][:sub], d["lengths"][:sub], mode=1,
                           threads=8)
    assert res[:sub].view(np.uint8).tobytes() == exp.view(np.uint8).tobytes()
    a0, a1 = len(d["sp5"]), len(d["sp27"])
    assert counts.tolist() == host_counts(res, a0, a1).tolist()
    assert counts2.tolist() == counts.tolist()
    assert res2.tobytes() == res.tobytes()


def test_comm_init_all_rejects_shared_device():
    ctxs = [lib.Context(0), lib.Context(0)]
    try:
        assert not lib.comm_init_all(ctxs)    # RCCL cannot place two ranks on one device
        assert ctxs[0].comm_size() == 0
    finally:
        for c in ctxs:
            c.close()


def test_allreduce_without_communicator_is_refused(c2x24):
    d, p = c2x24
    with lib.Context(0) as ctx:
        _setup(ctx, d)
        ctx.load(p)
        ctx.exec()
        with pytest.raises(lib.DmxError, match=r"\(-5\)"):
            ctx.allreduce_counts()


def test_comm_in_a_torch_process_uses_its_rccl():
    """bench.py's multi-GPU path imports torch (which maps its own librccl.so, soname
    librccl.so.1) before libdmx opens RCCL at its first communicator (csrc/dmx_comm.cpp): the
    dlopen must resolve to that already-mapped copy, and a single-rank communicator must sum
    the counts.  Run in a child process so this process's RCCL state does not matter."""
    import os
    import subprocess
    import sys
    code = r"""
import os, sys, json
sys.path.insert(0, os.path.join(%r, "nanopore-barcoding-orc_amd"))
import torch
from dmx import lib, synth
d = synth.generate("c2", n=5000, seed=4)
with lib.Context(0) as ctx:
    ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC)
    ctx.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC)
    ctx.set_mode(lib.MODE_TWO_ROUND)
    ctx.comm_init_rank(lib.comm_unique_id(), 1, 0)
    ctx.load(lib.pack(d["blob"], d["offsets"], d["lengths"]))
    ctx.exec()
    local = ctx.counts().tolist()
    reduced = ctx.allreduce_counts().tolist()
maps = [l.split()[-1] for l in open("/proc/self/maps") if "librccl" in l]
print(json.dumps({"same": local == reduced, "n": sum(local), "rccl": sorted(set(maps))}))
""" % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    r = __import__("json").loads(out.stdout.strip().splitlines()[-1])
    assert r["same"] and r["n"] > 0
    assert len(r["rccl"]) == 1, r["rccl"]   # one RCCL mapped: torch's
