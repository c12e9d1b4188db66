"""GPU parity: libdmx (HIP) vs the oracle (CPU restatement of cutadapt 4.9) on seeded inputs.

Bit-exact on every field of every read: bins, RC flags, trim coordinates, scores, errors.
"""
import numpy as np
import pytest

import oracle
from dmx import lib, synth

pytestmark = pytest.mark.gpu


def _oracle_two_round(d, rc=True, threads=8):
    p1 = oracle.Panel(d["sp5"], oracle.FRONT)
    p2 = oracle.Panel(d["sp27"], oracle.BACK)
    return oracle.run_batch(p1, p2, d["blob"], d["offsets"], d["lengths"], mode=1, use_rc=rc,
                            threads=threads)


def _gpu_two_round(ctx, d, rc=True):
    f = lib.DMX_RC if rc else 0
    ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | f)
    ctx.set_panel(1, d["sp27"], lib.DMX_BACK | f)
    ctx.set_mode(lib.MODE_TWO_ROUND)
    return ctx.run(lib.pack(d["blob"], d["offsets"], d["lengths"]))


def _assert_same(got, exp):
    got = got.view(np.uint8).reshape(len(got), -1)
    exp = exp.view(np.uint8).reshape(len(exp), -1)
    bad = np.nonzero((got != exp).any(axis=1))[0]
    assert len(bad) == 0, f"{len(bad)} reads differ, first {bad[:10]}"


@pytest.mark.parametrize("config,n", [("c1", 1000), ("c2", 20000), ("c2x24", 5000),
                                      ("c4", 5000)])
def test_two_round_matches_oracle(ctx, config, n):
    d = synth.generate(config, n=n)
    exp = _oracle_two_round(d)
    got = _gpu_two_round(ctx, d)
    got_v = got.view(oracle.RESULT_DTYPE)
    for f in ("bin1", "rc1", "bin2", "rc2"):
        assert np.array_equal(got_v[f], exp[f]), f
    _assert_same(got, exp)
