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
