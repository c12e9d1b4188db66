"""dmx_run of a batch larger than one chunk (include/dmx.h dmx_run): chunks alternate between two
device input/result sets while the next chunk uploads and the previous one downloads on a copy
stream.  Results and per-bin counts must equal the one-shot run's byte for byte (and the
oracle's on a prefix), whatever the chunk size; dmx_counts / the RCCL all-reduce see the whole
batch; dmx_fetch after a chunked run is refused."""
import numpy as np
import pytest

import oracle
from dmx import lib, synth
from test_comm import host_counts

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c2x24():
    d = synth.generate("c2x24", n=20000, seed=21)
    return d, lib.pack(d["blob"], d["offsets"], d["lengths"])


def _setup(ctx, d):
    ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC)
    ctx.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC)
    ctx.set_mode(lib.MODE_TWO_ROUND)


def _run(d, p, chunk, monkeypatch):
    monkeypatch.setenv("DMX_RUN_CHUNK", str(chunk))
    with lib.Context(0) as ctx:
        _setup(ctx, d)
        res = ctx.run(p)
        counts = ctx.counts()
        refused = False
        if chunk and p.n_reads > chunk + chunk // 2:
            with pytest.raises(lib.DmxError):
                ctx.fetch()
            refused = True
        # the context stays usable: a plain load/exec/fetch afterwards
        ctx.load(p)
        ctx.exec()
        again = ctx.fetch()
    return res, counts, refused, again


@pytest.mark.parametrize("chunk", [997, 4096, 7000])
def test_chunked_run_matches_one_shot(c2x24, chunk, monkeypatch):
    d, p = c2x24
    res0, counts0, _, _ = _run(d, p, 0, monkeypatch)
    res, counts, refused, again = _run(d, p, chunk, monkeypatch)
    assert refused
    assert res.tobytes() == res0.tobytes()
    assert counts.tolist() == counts0.tolist()
    assert again.tobytes() == res0.tobytes()
    a0, a1 = len(d["sp5"]), len(d["sp27"])
    assert counts.tolist() == host_counts(res, a0, a1).tolist()
    sub = 3000
    exp = oracle.run_batch(oracle.Panel(d["sp5"], oracle.FRONT),
                           oracle.Panel(d["sp27"], oracle.BACK), d["blob"],
                           d["offsets"][:sub], d["lengths"][:sub], mode=1, threads=8)
    assert res[:sub].view(np.uint8).tobytes() == exp.view(np.uint8).tobytes()


def test_chunked_run_multi_rccl_counts(c2x24, monkeypatch):
    """dmx_run_multi over a one-device comm group with chunked shards: the RCCL all-reduce
    reduces the whole shard's counts."""
    d, p = c2x24
    res0, counts0, _, _ = _run(d, p, 0, monkeypatch)
    monkeypatch.setenv("DMX_RUN_CHUNK", "2500")
    ctxs = [lib.Context(0)]
    try:
        assert lib.comm_init_all(ctxs)
        _setup(ctxs[0], d)
        res, counts = lib.run_multi(ctxs, p)
    finally:
        for c in ctxs:
            c.close()
    assert res.tobytes() == res0.tobytes()
    assert counts.tolist() == counts0.tolist()


def test_even_chunk_count_then_mid_sized_load(c2x24, monkeypatch):
    """Capacities travel with their input sets: a one-shot load of the whole batch, a chunked
    dmx_run with an even number of chunks (the second set ends resident), then a load sized
    between the chunk and the first batch must reallocate, and match a fresh context."""
    d, p = c2x24
    n_mid = 12000
    q = lib.pack(d["blob"], d["offsets"][:n_mid], d["lengths"][:n_mid])
    monkeypatch.setenv("DMX_RUN_CHUNK", "5000")   # 20000 reads -> 4 chunks
    with lib.Context(0) as ctx:
        _setup(ctx, d)
        ctx.load(p)
        ctx.exec()
        ctx.sync()
        ctx.run(p)
        ctx.load(q)
        ctx.exec()
        got = ctx.fetch()
        got_counts = ctx.counts()
    with lib.Context(0) as ctx:
        _setup(ctx, d)
        ctx.load(q)
        ctx.exec()
        exp = ctx.fetch()
        exp_counts = ctx.counts()
    assert got.tobytes() == exp.tobytes()
    assert got_counts.tolist() == exp_counts.tolist()


def test_unaligned_batch_runs_one_shot(c2x24, monkeypatch):
    """A caller-packed batch whose offsets are not on dmx_pack's 32-nt grid is accepted at any
    size (it runs in one shot instead of chunks) with the same results."""
    d, p = c2x24
    n = 6000
    q = lib.pack(d["blob"], d["offsets"][:n], d["lengths"][:n])
    # shift every read by 16 nt (one u32 word) inside a buffer one word longer
    seq = np.concatenate([np.zeros(1, np.uint32), q.seq2b])
    nm = np.zeros(len(seq), np.uint32)
    bits = np.unpackbits(q.nmask.view(np.uint8), bitorder="little")
    sh = np.concatenate([np.zeros(16, np.uint8), bits, np.zeros(16, np.uint8)])
    nm[:] = np.packbits(sh, bitorder="little").view(np.uint32)[:len(nm)]
    shifted = lib.Packed(seq, nm, q.offsets + 16, q.lengths)
    monkeypatch.setenv("DMX_RUN_CHUNK", "1000")
    with lib.Context(0) as ctx:
        _setup(ctx, d)
        got = ctx.run(shifted)
    monkeypatch.setenv("DMX_RUN_CHUNK", "0")
    with lib.Context(0) as ctx:
        _setup(ctx, d)
        exp = ctx.run(q)
    assert got.tobytes() == exp.tobytes()


@pytest.mark.parametrize("chunk", [0, 4096])
def test_sparse_mask_run_matches_dense(c2x24, chunk, monkeypatch):
    """dmx_run_sparse (the no-match mask as its nonzero words, scattered on the device) equals
    dmx_run with the dense mask, one-shot and chunked, with N-heavy reads mixed in."""
    d, _ = c2x24
    blob = d["blob"].copy()
    rng = np.random.default_rng(4)
    blob[rng.random(len(blob)) < 0.003] = ord("N")
    p = lib.pack(blob, d["offsets"], d["lengths"])
    monkeypatch.setenv("DMX_RUN_CHUNK", str(chunk))
    with lib.Context(0) as ctx:
        _setup(ctx, d)
        dense = ctx.run(p)
        pinned = lib.host_register([p.seq2b, p.offsets, p.lengths] + list(p.exceptions()))
        try:
            sparse = ctx.run_sparse(p)
            c_sparse = ctx.counts()
        finally:
            lib.host_unregister(pinned)
        again = ctx.run(p)
    assert sparse.tobytes() == dense.tobytes() == again.tobytes()
    assert c_sparse.sum() > 0


def test_permuted_batch_runs_one_shot(c2x24, monkeypatch):
    """A dmx_pack batch whose reads are reordered (every offset aligned, but some below their
    chunk's first offset) must not be chunked: the device rebase by the chunk base would wrap.
    It runs in one shot and its results are the unpermuted run's, permuted."""
    d, p = c2x24
    perm = np.random.default_rng(7).permutation(p.n_reads)
    q = lib.Packed(p.seq2b, p.nmask, p.offsets[perm].copy(), p.lengths[perm].copy())
    monkeypatch.setenv("DMX_RUN_CHUNK", "3000")
    with lib.Context(0) as ctx:
        _setup(ctx, d)
        got = ctx.run(q)
        got_counts = ctx.counts()
        ctx.fetch()          # a one-shot run leaves its results fetchable (not chunked)
    monkeypatch.setenv("DMX_RUN_CHUNK", "0")
    with lib.Context(0) as ctx:
        _setup(ctx, d)
        exp = ctx.run(p)
        exp_counts = ctx.counts()
    assert got.tobytes() == exp[perm].tobytes()
    assert got_counts.tolist() == exp_counts.tolist()
