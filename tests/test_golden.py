"""Golden fixtures (tests/golden/, made by tests/golden/make_golden.py).

The vectors are the CPU restatements' answers (C oracle and full-matrix Python restatement, which
agreed on every vector when it was written); PARITY UNPINNED against cutadapt 4.9 itself, which
is absent here and ships no fixtures.  CPU tests re-derive them with the oracle;
GPU tests run libdmx.so on the same inputs through the C-ABI and compare every byte — the GPU
side never loads the oracle.
"""
import glob
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = sorted(os.path.splitext(os.path.basename(p))[0]
               for p in glob.glob(os.path.join(GOLD, "*.npz")))
FRONT, BACK = 11, 14   # oracle / pyref flag words (QUERY_START|QUERY_STOP|REF_START / REF_END)


def _load(name):
    z = np.load(os.path.join(GOLD, name + ".npz"))   # allow_pickle=False (default)
    d = {k: z[k] for k in z.files}
    d["panel1"] = [str(s) for s in d["panel1"]]
    d["panel2"] = [str(s) for s in d["panel2"]]
    return d


def _kats():
    with open(os.path.join(GOLD, "locate_kats.json")) as fh:
        return json.load(fh)["cases"]


def test_golden_inventory():
    assert {"c1_two_round", "c2x24_two_round", "c4_two_round", "c5_linked",
            "random_front_iupac", "random_back_iupac"} <= set(CASES)
    assert len(_kats()) > 600


@pytest.mark.parametrize("name", CASES)
def test_oracle_reproduces_golden(name):
    import oracle
    d = _load(name)
    e = float(d["max_errors"])
    p1 = oracle.Panel(d["panel1"], [int(w) for w in d["where1"]], max_errors=e)
    p2 = oracle.Panel(d["panel2"], oracle.BACK, max_errors=e) if d["panel2"] else None
    res = oracle.run_batch(p1, p2, d["blob"], d["offsets"], d["lengths"], mode=int(d["mode"]),
                           use_rc=bool(d["use_rc"]), threads=8)
    got = res.view(np.uint8).reshape(len(res), 40)
    bad = np.nonzero((got != d["expected"]).any(axis=1))[0]
    assert len(bad) == 0, f"{name}: {len(bad)} reads differ, first {bad[:10]}"


def test_locate_kats_oracle():
    import oracle
    for c in _kats():
        w = FRONT if c["where"] == "front" else BACK
        got = oracle.locate(c["adapter"], c["read"], c["max_error_rate"], w, c["min_overlap"])
        exp = tuple(c["expected"]) if c["expected"] is not None else None
        assert got == exp, c


def test_locate_kats_full_matrix_subset():
    """Every 8th KAT through the pure-Python full-matrix restatement (seconds)."""
    import pyref
    for c in _kats()[::8]:
        w = FRONT if c["where"] == "front" else BACK
        got = pyref.locate(c["adapter"], c["read"], c["max_error_rate"], w, c["min_overlap"])
        exp = tuple(c["expected"]) if c["expected"] is not None else None
        assert got == exp, c


# ---------------------------------------------------------------- GPU (libdmx.so, C-ABI) ----

def _where_flags(lib, w):
    return lib.DMX_FRONT if int(w) == FRONT else lib.DMX_BACK


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_gpu_reproduces_golden(ctx, name):
    from dmx import lib
    d = _load(name)
    e, rc, mode = float(d["max_errors"]), bool(d["use_rc"]), int(d["mode"])
    wh = [_where_flags(lib, w) for w in d["where1"]]
    if len(set(wh)) == 1:
        ctx.set_panel(0, d["panel1"], wh[0] | (lib.DMX_RC if rc else 0), e)
    else:
        ctx.set_panel_mixed(0, d["panel1"], wh, rc, e)
    if d["panel2"]:
        ctx.set_panel(1, d["panel2"], lib.DMX_BACK | (lib.DMX_RC if rc else 0), e)
    ctx.set_mode(mode)
    res = ctx.run(lib.pack(d["blob"], d["offsets"], d["lengths"]))
    got = res.view(np.uint8).reshape(len(res), 40)
    bad = np.nonzero((got != d["expected"]).any(axis=1))[0]
    assert len(bad) == 0, f"{name}: {len(bad)} reads differ, first {bad[:10]}"


@pytest.mark.gpu
def test_gpu_locate_kats(ctx):
    """Each KAT as a one-adapter, one-round call without --rc: bin 0 iff the KAT matched, and the
    match fields (read start/stop, adapter start/stop, score, errors) equal the KAT's."""
    from dmx import lib
    groups = {}
    for c in _kats():
        groups.setdefault((c["adapter"], c["where"], c["max_error_rate"], c["min_overlap"]),
                          []).append(c)
    ctx.set_mode(lib.MODE_SINGLE)
    for (ad, where, e, mo), cs in groups.items():
        ctx.set_panel(0, [ad], lib.DMX_FRONT if where == "front" else lib.DMX_BACK, e, mo)
        seqs = [c["read"] for c in cs]
        lens = np.array([len(s) for s in seqs], dtype=np.uint32)
        offs = np.zeros(len(seqs), dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        blob = np.frombuffer("".join(seqs).encode(), dtype=np.uint8)
        res = ctx.run(lib.pack(blob, offs, lens))
        for c, r in zip(cs, res):
            if c["expected"] is None:
                assert int(r["bin1"]) == -1, c
                continue
            rs, rt, qs, qt, score, err = c["expected"]
            assert int(r["bin1"]) == 0, c
            assert (int(r["m1_rstart"]), int(r["m1_rstop"]), int(r["m1_astart"]),
                    int(r["m1_astop"]), int(r["m1_score"]), int(r["m1_errors"])) == \
                (qs, qt, rs, rt, score, err), c
