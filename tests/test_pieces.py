"""GPU parity of the piece screen against the oracle.

Adversarial reads: every adapter of the 24 x 24 panels with exactly K edits, one in each of K of
its K + 1 pieces (so exactly one piece survives as an exact copy), for every surviving piece, in
both read orientations, at the read start, middle and end; partial adapters at both read ends;
N inside and around the pieces.  The flat scan (dmx_pack layouts, permuted read order, reads
that overlap in the packed batch), the per-part screen (DMX_NO_FLAT=1) and the full filter pass
(DMX_NO_PIECES=1) must all equal the oracle on every result byte.
"""
import numpy as np
import pytest

import oracle
from dmx import lib, synth
from test_pieces_host import _flank_cases, full_k, mutate, pieces_of, revcomp

pytestmark = pytest.mark.gpu


def _assert_same(got, exp):
    got = got.view(np.uint8).reshape(len(got), -1)
    exp = exp.view(np.uint8).reshape(len(exp), -1)
    bad = np.nonzero((got != exp).any(axis=1))[0]
    assert len(bad) == 0, f"{len(bad)} reads differ, first {bad[:10]}"


def _rand(rng, n, alphabet="ACGT", p=None):
    return "".join(rng.choice(list(alphabet), size=int(n), p=p))


def adversarial_reads(rng, panel, where, rate=0.1):
    """Reads holding one adapter copy with K edits (one surviving piece), plus partial copies at
    the read ends (a FRONT adapter's suffix at the start, a BACK adapter's prefix at the end)."""
    seqs = []
    for ad in panel:
        K = full_k(len(ad), rate)
        pcs = pieces_of(len(ad), K)
        for survive in range(K + 1):
            for place in ("start", "middle", "end"):
                copy = mutate(rng, ad, pcs, survive)
                L = int(rng.integers(150, 900))
                flank = int(rng.integers(0, 9))
                if place == "start":
                    s = _rand(rng, flank) + copy + _rand(rng, L)
                elif place == "end":
                    s = _rand(rng, L) + copy + _rand(rng, flank)
                else:
                    s = _rand(rng, L // 2) + copy + _rand(rng, L // 2)
                seqs.append(revcomp(s) if rng.random() < 0.5 else s)
        for _ in range(3):   # partial copies at the ends, with up to acc errors of their own
            cut = int(rng.integers(3, len(ad)))
            part = ad[len(ad) - cut:] if where == oracle.FRONT else ad[:cut]
            part = "".join(c if rng.random() > 0.05 else _rand(rng, 1) for c in part)
            s = part + _rand(rng, 300) if where == oracle.FRONT else _rand(rng, 300) + part
            seqs.append(revcomp(s) if rng.random() < 0.5 else s)
    # N inside and around the pieces of otherwise exact copies
    for _ in range(60):
        ad = panel[int(rng.integers(len(panel)))]
        s = list(_rand(rng, 200) + ad + _rand(rng, 200))
        for _ in range(int(rng.integers(1, 4))):
            s[200 + int(rng.integers(-8, len(ad) + 8))] = "N"
        s = "".join(s)
        seqs.append(revcomp(s) if rng.random() < 0.5 else s)
    return seqs + ["", "A", ad[:7], ad[-7:]]


def overlapping(seqs):
    """seqs plus, per read of >= 12 nt, the read without its first 3 and last 4 nt: packed as a
    view into the read's own nt (_run), so the batch holds reads that share nt."""
    return seqs + [s[3:len(s) - 4] for s in seqs if len(s) >= 12]


def _run(seqs, panel, where, layout="sorted", env=None, monkeypatch=None):
    perm = None
    if layout == "overlap":   # results for overlapping(seqs): the sub-reads point into their reads
        blob, offs, lens = oracle.pack_ascii(seqs)
        p = lib.pack(blob, offs, lens)
        src = [i for i in range(len(seqs)) if lens[i] >= 12]
        offs2 = np.concatenate([p.offsets, p.offsets[src] + 3]).astype(p.offsets.dtype)
        lens2 = np.concatenate([p.lengths, p.lengths[src] - 7]).astype(p.lengths.dtype)
        p = lib.Packed(p.seq2b, p.nmask, offs2, lens2)
    else:
        blob, offs, lens = oracle.pack_ascii(seqs)
        p = lib.pack(blob, offs, lens)
    if layout == "permuted":
        perm = np.random.default_rng(1).permutation(p.n_reads)
        p = lib.Packed(p.seq2b, p.nmask, p.offsets[perm].copy(), p.lengths[perm].copy())
    for k, v in (env or {}).items():
        monkeypatch.setenv(k, v)
    f = lib.DMX_FRONT if where == oracle.FRONT else lib.DMX_BACK
    with lib.Context(0) as c:
        c.set_panel(0, panel, f | lib.DMX_RC)
        c.set_mode(lib.MODE_SINGLE)
        got = c.run(p)
        tasks = c.stats()["filter_tasks"]
    for k in (env or {}):
        monkeypatch.delenv(k)
    if perm is not None:
        inv = np.empty_like(perm)
        inv[perm] = np.arange(len(perm))
        got = got[inv]
    return got, tasks


@pytest.mark.parametrize("rnd", [0, 1])
@pytest.mark.parametrize("variant", ["flat", "permuted", "overlap", "no_flat", "no_pieces"])
def test_one_surviving_piece(rnd, variant, monkeypatch):
    n1, s5, n2, s27 = synth.panels(24, 24)
    panel, where = (s5, oracle.FRONT) if rnd == 0 else (s27, oracle.BACK)
    rng = np.random.default_rng(100 + rnd)
    seqs = adversarial_reads(rng, panel, where)
    blob, offs, lens = oracle.pack_ascii(overlapping(seqs) if variant == "overlap" else seqs)
    exp = oracle.run_batch(oracle.Panel(panel, where), None, blob, offs, lens, mode=0,
                           use_rc=True, threads=8)
    assert (exp["bin1"] >= 0).mean() > 0.7
    layout = variant if variant in ("permuted", "overlap") else "sorted"
    env = {"no_flat": {"DMX_NO_FLAT": "1"}, "no_pieces": {"DMX_NO_PIECES": "1"}}.get(variant)
    got, tasks = _run(seqs, panel, where, layout, env, monkeypatch)
    _assert_same(got, exp)
    if variant == "no_pieces":
        assert tasks[0] == 0
    else:
        assert tasks[0] > 0   # the piece screen ran


def test_two_round_adversarial(ctx):
    """Both rounds on one batch: SP5 copies with one surviving piece at the read start, SP27rc
    copies with one surviving piece at the end, orientations mixed."""
    n1, s5, n2, s27 = synth.panels(24, 24)
    rng = np.random.default_rng(7)
    seqs = []
    for i in range(3000):
        a, b = s5[i % 24], s27[(i * 7) % 24]
        ka, kb = full_k(len(a), 0.1), full_k(len(b), 0.1)
        ca = mutate(rng, a, pieces_of(len(a), ka), int(rng.integers(ka + 1)))
        cb = mutate(rng, b, pieces_of(len(b), kb), int(rng.integers(kb + 1)))
        s = _rand(rng, rng.integers(0, 9)) + ca + _rand(rng, rng.integers(100, 1500)) + cb + \
            _rand(rng, rng.integers(0, 9))
        seqs.append(revcomp(s) if rng.random() < 0.3 else s)
    blob, offs, lens = oracle.pack_ascii(seqs)
    exp = oracle.run_batch(oracle.Panel(s5, oracle.FRONT), oracle.Panel(s27, oracle.BACK), blob,
                           offs, lens, mode=1, threads=8)
    assert (exp["bin2"] >= 0).mean() > 0.7
    ctx.set_panel(0, s5, lib.DMX_FRONT | lib.DMX_RC)
    ctx.set_panel(1, s27, lib.DMX_BACK | lib.DMX_RC)
    ctx.set_mode(lib.MODE_TWO_ROUND)
    got = ctx.run(lib.pack(blob, offs, lens))
    _assert_same(got, exp)
    assert all(t > 0 for t in ctx.stats()["filter_tasks"])


def test_iupac_panel_falls_back_to_the_full_filter(ctx):
    """A panel with a wildcard builds no pieces: the full filter pass runs (no filter tasks)."""
    rng = np.random.default_rng(9)
    suffix = _rand(rng, 20)
    panel = [_rand(rng, 20) + "N" + _rand(rng, 15) + suffix for _ in range(6)]
    seqs = []
    for _ in range(1500):
        ad = panel[int(rng.integers(6))].replace("N", "ACGT"[int(rng.integers(4))])
        s = _rand(rng, rng.integers(0, 300)) + ad + _rand(rng, rng.integers(0, 300))
        seqs.append(revcomp(s) if rng.random() < 0.5 else s)
    blob, offs, lens = oracle.pack_ascii(seqs)
    exp = oracle.run_batch(oracle.Panel(panel, oracle.BACK), None, blob, offs, lens, mode=0,
                           use_rc=True, threads=8)
    ctx.set_panel(0, panel, lib.DMX_BACK | lib.DMX_RC)
    ctx.set_mode(lib.MODE_SINGLE)
    got = ctx.run(lib.pack(blob, offs, lens))
    _assert_same(got, exp)
    assert ctx.stats()["filter_tasks"][0] == 0


@pytest.mark.parametrize("case", ["iupac_round1", "no_flat"])
def test_two_round_mixed_screens(case, monkeypatch):
    """Round 1 on the full filter pass (a wildcard panel) while round 2 takes the flat scan (its
    marks come from the one scan launched ahead of round 1), and both rounds on the per-part
    screen (DMX_NO_FLAT=1)."""
    n1, s5, n2, s27 = synth.panels(24, 24)
    rng = np.random.default_rng(11)
    p1 = [a[:10] + "N" + a[11:] for a in s5] if case == "iupac_round1" else s5
    seqs = []
    for i in range(2000):
        a = p1[i % 24].replace("N", "ACGT"[int(rng.integers(4))])
        b = s27[(i * 5) % 24]
        kb = full_k(len(b), 0.1)
        cb = mutate(rng, b, pieces_of(len(b), kb), int(rng.integers(kb + 1)))
        s = _rand(rng, rng.integers(0, 9)) + a + _rand(rng, rng.integers(100, 1200)) + cb
        seqs.append(revcomp(s) if rng.random() < 0.4 else s)
    blob, offs, lens = oracle.pack_ascii(seqs)
    exp = oracle.run_batch(oracle.Panel(p1, oracle.FRONT), oracle.Panel(s27, oracle.BACK), blob,
                           offs, lens, mode=1, threads=8)
    assert (exp["bin2"] >= 0).mean() > 0.6
    if case == "no_flat":
        monkeypatch.setenv("DMX_NO_FLAT", "1")
    with lib.Context(0) as c:
        c.set_panel(0, p1, lib.DMX_FRONT | lib.DMX_RC)
        c.set_panel(1, s27, lib.DMX_BACK | lib.DMX_RC)
        c.set_mode(lib.MODE_TWO_ROUND)
        got = c.run(lib.pack(blob, offs, lens))
        tasks = c.stats()["filter_tasks"]
    _assert_same(got, exp)
    assert tasks[1] > 0 and (tasks[0] == 0) == (case == "iupac_round1")


@pytest.mark.parametrize("variant", ["flat", "no_flat"])
@pytest.mark.parametrize("name,panel,where,rate", _flank_cases())
def test_shared_flank_panels(name, panel, where, rate, variant, monkeypatch):
    """Panels whose adapters share a constant prefix and suffix: pieces that straddle a shared
    block sample a window past offset 0 (the tools/parity_sweep.py seed-56 mismatches, when
    offsets 4 .. 8 overflowed the entries' 2-bit field)."""
    w = oracle.FRONT if where == lib.DMX_FRONT else oracle.BACK
    rng = np.random.default_rng(200 + len(name))
    seqs = adversarial_reads(rng, panel, w, rate)
    for ad in panel:   # exact copies at every start modulo the sampling stride
        for shift in range(4):
            s = _rand(rng, 40 + shift) + ad + _rand(rng, 60)
            seqs.append(revcomp(s) if rng.random() < 0.5 else s)
    blob, offs, lens = oracle.pack_ascii(seqs)
    exp = oracle.run_batch(oracle.Panel(panel, w, max_errors=rate), None, blob, offs, lens,
                           mode=0, use_rc=True, threads=8)
    assert (exp["bin1"] >= 0).mean() > 0.5
    if variant == "no_flat":
        monkeypatch.setenv("DMX_NO_FLAT", "1")
    with lib.Context(0) as c:
        c.set_panel(0, panel, where | lib.DMX_RC, rate)
        c.set_mode(lib.MODE_SINGLE)
        got = c.run(lib.pack(blob, offs, lens))
        tasks = c.stats()["filter_tasks"]
    _assert_same(got, exp)
    assert tasks[0] > 0
