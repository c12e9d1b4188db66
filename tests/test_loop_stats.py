"""The fused loop's round-2 report statistics (dmx/loop.py _round_stats) against a per-bin
boolean-mask restatement (the loop's earlier form): same counts, histograms and adjacent-base
tallies per SP5 bin on random two-round results, with and without the packed batch."""
from __future__ import annotations

import numpy as np
import pytest

from dmx import lib, loop, panel, report, synth
from dmx.report import Stats


def _masks_reference(st1, st2, res, lens, m1, m2, b1, b2, s1, s2w, e2w, bp2_out, n2_out,
                     packed=None):
    lens = lens.astype(np.int64)
    n = len(res)
    rc1 = res["rc1"] == 1
    st1.n_in += n
    st1.bp_in += int(lens.sum())
    st1.n_with_adapter += int(m1.sum())
    st1.n_rc += int(rc1.sum())
    st1.add_counts(b1[m1], rc1[m1], len(st1.adapters))
    st1.add_matches(b1[m1], "front", s1[m1], res["m1_errors"].astype(np.int64)[m1])
    len1 = lens - s1
    rc2 = (res["rc2"] == 1) & m1
    adj = None
    if packed is not None:
        hit_all = np.nonzero(m1 & m2)[0]
        p = res["m2_rstart"].astype(np.int64)[hit_all] - 1
        r1 = res["rc1"].astype(np.int64)[hit_all]
        two = res["rc2"].astype(np.int64)[hit_all] == 1
        codes = report.view_codes(packed, hit_all, np.where(two, 1 - r1, r1),
                                  np.where(two, p, np.where(p >= 0, s1[hit_all] + p, -1)))
        adj = np.full(n, 4, np.int64)
        adj[hit_all] = codes
    for i, s in enumerate(st2):
        sel = m1 & (b1 == i)
        if not sel.any():
            continue
        s.n_in += int(sel.sum())
        s.bp_in += int(len1[sel].sum())
        hit = sel & m2
        s.n_with_adapter += int(hit.sum())
        s.n_rc += int(rc2[sel].sum())
        s.add_counts(b2[hit], rc2[hit], len(s.adapters))
        s.add_matches(b2[hit], "back", len1[hit] - res["m2_rstart"].astype(np.int64)[hit],
                      res["m2_errors"].astype(np.int64)[hit])
        if adj is not None:
            s.add_adjacent(b2[hit], adj[hit])
        n2_out[i] += int(sel.sum())
        bp2_out[i] += int(np.where(m2, e2w - s2w, len1)[sel].sum())


def _state(s: Stats):
    return (s.n_in, s.bp_in, s.n_with_adapter, s.n_rc, dict(s.matches), dict(s.on_rc),
            {a: {p: dict(c) for p, c in parts.items()} for a, parts in s.hist.items()},
            {a: v.tolist() for a, v in s.adjacent.items()})


@pytest.mark.parametrize("with_packed", [False, True])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_round_stats_equals_per_bin_masks(seed, with_packed):
    rng = np.random.default_rng(seed)
    a1, a2 = panel.AdapterSet(), panel.AdapterSet()
    a1.add_spec(f"file:{panel.SP5_FASTA}", "front")
    a2.add_spec(f"file:{panel.SP27RC_FASTA}", "back")
    ads1, ads2 = a1.adapters, a2.adapters
    n = int(rng.integers(1, 3000))
    d = synth.generate("c2", n=n, seed=seed)
    lens = d["lengths"].astype(np.int64)
    res = np.zeros(n, lib.RESULT_DTYPE)
    # some SP5 bins stay empty (the grouping's empty slices)
    b1 = np.where(rng.random(n) < 0.1, -1, rng.choice([0, 2, 3, 7, 11], n))
    b2 = np.where((b1 >= 0) & (rng.random(n) < 0.8), rng.integers(0, len(ads2), n), -1)
    res["bin1"], res["bin2"] = b1, b2
    res["rc1"] = rng.integers(0, 2, n)
    res["rc2"] = rng.integers(0, 2, n)
    s1 = np.where(b1 >= 0, np.minimum(lens, rng.integers(0, 90, n)), 0)
    r2 = np.where(b2 >= 0, np.maximum(0, lens - s1 - rng.integers(0, 90, n)), 0)
    res["m1_rstop"], res["m2_rstart"] = s1, r2
    res["m1_errors"] = rng.integers(0, 4, n)
    res["m2_errors"] = rng.integers(0, 4, n)
    (s1p, e1, o1), (s2, e2, o2, nrc2) = loop.plan_rounds(res, lens)
    m1, m2 = b1 >= 0, b2 >= 0
    u2rc = ~m2 & (res["rc2"] == 1)
    s2w = np.where(m2, s2, np.where(u2rc, 0, s1p))
    e2w = np.where(m2, e2, np.where(u2rc, e1 - s1p, e1))
    packed = lib.pack(d["blob"], d["offsets"], d["lengths"]) if with_packed else None
    out = []
    for fn in (loop._round_stats, _masks_reference):
        st1, st2 = Stats(ads1), [Stats(ads2) for _ in ads1]
        bp2, n2 = np.zeros(len(ads1), np.int64), np.zeros(len(ads1), np.int64)
        fn(st1, st2, res, lens, m1, m2, b1.astype(np.int64), b2.astype(np.int64), s1p, s2w, e2w,
           bp2, n2, packed)
        out.append((_state(st1), [_state(s) for s in st2], bp2.tolist(), n2.tolist()))
    assert out[0] == out[1]
