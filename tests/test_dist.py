"""World-size-2 sharding + count all-reduce with gloo, standing in for the N-GPU run: the merged
per-bin counts of two shards must equal the single-process counts.  On CPU each rank runs the
oracle on its shard; on the GPU box each rank runs libdmx on its shard (both ranks share the one
GPU, where RCCL cannot place two ranks, so gloo carries the counts; the RCCL leg itself is
tested single-rank in tests/test_comm.py)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from dmx import dist as ddist
from dmx import synth


def _counts(res, a0, a1):
    c = np.zeros((a0 + 1) * (a1 + 1) + 2, dtype=np.int64)
    idx = (res["bin1"].astype(np.int64) + 1) * (a1 + 1) + (res["bin2"].astype(np.int64) + 1)
    np.add.at(c, idx, 1)
    c[-2] = int(res["rc1"].sum())
    c[-1] = int(res["rc2"][res["bin1"] >= 0].sum())
    return c


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = synth.generate("c1", n=400)
    lo, hi = ddist.balanced_ranges(d["lengths"], world)[rank]
    p1, p2 = oracle.Panel(d["sp5"], oracle.FRONT), oracle.Panel(d["sp27"], oracle.BACK)
    res = oracle.run_batch(p1, p2, d["blob"], d["offsets"][lo:hi], d["lengths"][lo:hi], mode=1)
    merged = ddist.allreduce_counts(_counts(res, 4, 4))
    if rank == 0:
        q.put(merged.tolist())
    dist.barrier()
    dist.destroy_process_group()


def _gpu_worker(rank, world, port, q):
    """bench.py's multi-rank step on one shard: libdmx two-round demux + count all-reduce."""
    from dmx import lib
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = synth.generate("c2x24", n=6000, seed=31)
    lo, hi = ddist.balanced_ranges(d["lengths"], world)[rank]
    with lib.Context(0) as ctx:
        ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC)
        ctx.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC)
        ctx.set_mode(lib.MODE_TWO_ROUND)
        ctx.load(lib.pack(d["blob"], d["offsets"][lo:hi], d["lengths"][lo:hi]))
        ctx.exec()
        ctx.sync()
        res = ctx.fetch()
        local = ctx.counts()
    assert local.tolist() == _counts(res, 24, 24).tolist()
    merged = ddist.allreduce_counts(local.astype(np.int64))
    out = [None] * world
    dist.all_gather_object(out, (lo, hi, res.tobytes()))
    if rank == 0:
        q.put((merged.tolist(), out))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_balanced_ranges_cover_and_balance():
    lens = np.random.default_rng(0).integers(300, 6000, size=10001)
    for world in (1, 2, 3, 8):
        rs = ddist.balanced_ranges(lens, world)
        assert rs[0][0] == 0 and rs[-1][1] == len(lens)
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
        tot = [int(lens[a:b].sum()) for a, b in rs]
        assert max(tot) - min(tot) <= 2 * lens.max()


def test_two_rank_count_allreduce():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    merged = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    d = synth.generate("c1", n=400)
    p1, p2 = oracle.Panel(d["sp5"], oracle.FRONT), oracle.Panel(d["sp27"], oracle.BACK)
    full = oracle.run_batch(p1, p2, d["blob"], d["offsets"], d["lengths"], mode=1)
    assert merged == _counts(full, 4, 4).tolist()


@pytest.mark.gpu
def test_two_rank_libdmx_shards():
    """Two ranks, each running libdmx on its Σ-length-balanced shard: the shard results
    concatenated in rank order and the all-reduced counts equal one whole-batch run."""
    from dmx import lib
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    merged, shards = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    d = synth.generate("c2x24", n=6000, seed=31)
    assert [s[0] for s in shards] == [0, shards[0][1]] and shards[1][1] == 6000
    with lib.Context(0) as c:
        c.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC)
        c.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC)
        c.set_mode(lib.MODE_TWO_ROUND)
        full = c.run(lib.pack(d["blob"], d["offsets"], d["lengths"]))
        whole = c.counts()
    assert b"".join(s[2] for s in shards) == full.tobytes()
    assert merged == whole.astype(np.int64).tolist() == _counts(full, 24, 24).tolist()
