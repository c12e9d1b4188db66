"""GPU parity: libdmx (HIP) vs the oracle (CPU restatement of cutadapt 4.9) on seeded inputs.

Bit-exact on every field of every read: bins, RC flags, trim coordinates, scores, errors.
"""
import os

import numpy as np
import pytest

import oracle
from dmx import lib, panel, synth
from helpers import amplicon_reads

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


def _random_panel(rng, n, lo, hi, wildcard=0.0):
    out = []
    for _ in range(n):
        L = int(rng.integers(lo, hi + 1))
        s = "".join(rng.choice(list("ACGT"), size=L))
        if wildcard:
            s = "".join(c if rng.random() > wildcard else rng.choice(list("NRYSWKMBDHV"))
                        for c in s)
        out.append(s)
    return out


def _reads_with(rng, panel, n, L=(0, 400), err=0.06):
    seqs = []
    for _ in range(n):
        Ln = int(rng.integers(L[0], L[1] + 1))
        s = "".join(rng.choice(list("ACGTN"), size=Ln, p=[0.249, 0.249, 0.249, 0.249, 0.004]))
        if panel and rng.random() < 0.8:
            a = panel[int(rng.integers(len(panel)))]
            a = "".join(c if c in "ACGT" else "ACGT"[int(rng.integers(4))] for c in a)
            frag = []
            for c in a:
                r = rng.random()
                if r < err * 0.6:
                    frag.append("ACGT"[int(rng.integers(4))])
                elif r < err * 0.8:
                    pass
                elif r < err:
                    frag += [c, "ACGT"[int(rng.integers(4))]]
                else:
                    frag.append(c)
            frag = "".join(frag)
            if rng.random() < 0.2:   # partial at either end
                cut = int(rng.integers(1, max(2, len(frag))))
                frag = frag[cut:] if rng.random() < 0.5 else frag[:cut]
            p = int(rng.integers(0, len(s) + 1))
            s = s[:p] + frag + s[p:]
        if rng.random() < 0.3:
            s = oracle_rc(s)
        seqs.append(s)
    return seqs


def oracle_rc(s):
    import pyref
    return pyref.revcomp(s)


@pytest.mark.parametrize("where", ["front", "back"])
@pytest.mark.parametrize("wild", [0.0, 0.15])
@pytest.mark.parametrize("rc", [True, False])
def test_single_round_random_panels(ctx, where, wild, rc):
    """Full-scan path (no shared suffix), mixed adapter lengths 3..64, IUPAC wildcards, N in
    reads, empty and short reads, partial adapters at both read ends."""
    rng = np.random.default_rng(11 + (where == "back") * 3 + int(wild * 100) + rc)
    panel = _random_panel(rng, 9, 3, 64, wild)
    seqs = _reads_with(rng, panel, 1500) + ["", "A", "ACG", panel[0][:5], panel[1][-4:]]
    blob, offs, lens = oracle.pack_ascii(seqs)
    ow = oracle.FRONT if where == "front" else oracle.BACK
    exp = oracle.run_batch(oracle.Panel(panel, ow), None, blob, offs, lens, mode=0, use_rc=rc,
                           threads=8)
    f = (lib.DMX_FRONT if where == "front" else lib.DMX_BACK) | (lib.DMX_RC if rc else 0)
    ctx.set_panel(0, panel, f)
    ctx.set_mode(lib.MODE_SINGLE)
    got = ctx.run(lib.pack(blob, offs, lens))
    _assert_same(got, exp)


@pytest.mark.parametrize("e", [0.1, 0.2, 2])
def test_error_rates_and_filter_toggle(ctx, e, monkeypatch):
    """-e as a rate and as an absolute count; index screen, prefix verification and shared-suffix
    filter each on vs off agree."""
    d = synth.generate("c4", n=3000, seed=5)
    p1 = oracle.Panel(d["sp5"], oracle.FRONT, max_errors=e)
    p2 = oracle.Panel(d["sp27"], oracle.BACK, max_errors=e)
    exp = oracle.run_batch(p1, p2, d["blob"], d["offsets"], d["lengths"], mode=1, threads=8)
    ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC, e)
    ctx.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC, e)
    ctx.set_mode(lib.MODE_TWO_ROUND)
    _assert_same(ctx.run(lib.pack(d["blob"], d["offsets"], d["lengths"])), exp)
    monkeypatch.setenv("DMX_NO_SCREEN", "1")
    with lib.Context(0) as c4:
        c4.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC, e)
        c4.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC, e)
        c4.set_mode(lib.MODE_TWO_ROUND)
        _assert_same(c4.run(lib.pack(d["blob"], d["offsets"], d["lengths"])), exp)
    monkeypatch.delenv("DMX_NO_SCREEN")
    monkeypatch.setenv("DMX_NO_VERIFY", "1")
    with lib.Context(0) as c3:
        c3.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC, e)
        c3.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC, e)
        c3.set_mode(lib.MODE_TWO_ROUND)
        _assert_same(c3.run(lib.pack(d["blob"], d["offsets"], d["lengths"])), exp)
    monkeypatch.setenv("DMX_NO_FILTER", "1")
    with lib.Context(0) as c2:
        c2.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC, e)
        c2.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC, e)
        c2.set_mode(lib.MODE_TWO_ROUND)
        _assert_same(c2.run(lib.pack(d["blob"], d["offsets"], d["lengths"])), exp)


@pytest.mark.parametrize("config,seed", [("c2x24", 3), ("c4", 4)])
def test_window_code_slots(config, seed, monkeypatch):
    """DMX_STAGE=1 (A/B): the screen, window scan and band read the codes of a
    verified window from its slot instead of the packed batch; every byte stays the same.  The
    slots are compiled only into the A/B build (make variant NAME=stage
    DEFS=-DDMX_STAGE_SLOTS=1): run with DMX_LIBDMX=.../dmx/libdmx_stage.so DMX_TEST_STAGE_SLOTS=1."""
    if os.environ.get("DMX_TEST_STAGE_SLOTS") != "1":
        pytest.skip("window code slots are an A/B build (DMX_STAGE_SLOTS=1)")
    monkeypatch.setenv("DMX_STAGE", "1")
    d = synth.generate(config, n=6000, seed=seed)
    exp = _oracle_two_round(d)
    with lib.Context(0) as c:
        _assert_same(_gpu_two_round(c, d), exp)
        _assert_same(_gpu_two_round(c, d, rc=False), _oracle_two_round(d, rc=False))


@pytest.mark.parametrize("mode", ["band", "ring"])
def test_resolve_kernels_agree(mode, monkeypatch):
    """Both resolve kernels (banded DP / LDS-ring traceback) reproduce the oracle."""
    if mode == "ring":
        monkeypatch.setenv("DMX_RESOLVE", "ring")
    d = synth.generate("c2", n=8000, seed=77)
    exp = _oracle_two_round(d)
    with lib.Context(0) as c:
        _assert_same(_gpu_two_round(c, d), exp)


def _linked_pairs(kind, rng):
    data = os.path.join(os.path.dirname(panel.SP5_FASTA))
    if kind in ("COI", "RNA"):
        return [(f, r) for _, f, r in panel.primer_pairs(os.path.join(data, f"{kind}_primers.fa"))]
    return [tuple(_random_panel(rng, 2, 12, 40, 0.1)) for _ in range(7)]


@pytest.mark.parametrize("kind", ["COI", "RNA", "random7"])
def test_linked_matches_oracle(ctx, kind):
    """Linked -g F...R (scripts/04_cleaning_primers.sh:377): per-pair front scan, back scan on
    read[front.rstop:], best pair by summed score then errors then pair order."""
    rng = np.random.default_rng({"COI": 1, "RNA": 2, "random7": 3}[kind])
    pairs = _linked_pairs(kind, rng)
    seqs = amplicon_reads(rng, pairs, 4000) + ["", "ACGT", pairs[0][0], pairs[0][0] + pairs[0][1]]
    blob, offs, lens = oracle.pack_ascii(seqs)
    exp = oracle.run_batch(oracle.Panel([p[0] for p in pairs], oracle.FRONT),
                           oracle.Panel([p[1] for p in pairs], oracle.BACK),
                           blob, offs, lens, mode=2, use_rc=False, threads=8)
    assert (exp["bin1"] >= 0).mean() > 0.5
    ctx.set_panel(0, [p[0] for p in pairs], lib.DMX_FRONT)
    ctx.set_panel(1, [p[1] for p in pairs], lib.DMX_BACK)
    ctx.set_mode(lib.MODE_LINKED)
    got = ctx.run(lib.pack(blob, offs, lens))
    _assert_same(got, exp)
    c = ctx.counts()
    A = len(pairs)
    for a in range(A):
        assert c[(a + 1) * (A + 1) + a + 1] == (exp["bin1"] == a).sum()
    assert c[0] == (exp["bin1"] < 0).sum()


def test_config5_linked_matches_oracle(ctx):
    """SURVEY.md §8d config 5 (synthetic COI consensuses, linked pairs, IUPAC instantiated,
    10% with one primer missing) on the GPU vs the oracle."""
    d = synth.generate("c5", n=20000)
    exp = oracle.run_batch(oracle.Panel(d["sp5"], oracle.FRONT), oracle.Panel(d["sp27"], oracle.BACK),
                           d["blob"], d["offsets"], d["lengths"], mode=2, use_rc=False, threads=8)
    untrimmed = (exp["bin1"] < 0).mean()
    assert 0.05 < untrimmed < 0.25
    ctx.set_panel(0, d["sp5"], lib.DMX_FRONT)
    ctx.set_panel(1, d["sp27"], lib.DMX_BACK)
    ctx.set_mode(lib.MODE_LINKED)
    _assert_same(ctx.run(lib.pack(d["blob"], d["offsets"], d["lengths"])), exp)


def test_linked_after_two_round_on_one_context():
    """Item list capacity across modes (parity sweep seed 43: illegal memory access).  A
    two-round batch of n1 reads sizes the winner slots for 2 n1 and the item list for n1; a later
    linked batch of n2 < n1 reads with P pairs needs n2 P items while n2 P <= 2 n1 slots still fit,
    so only the item list has to grow.  Every read here carries every pair, so the linked round 1
    has n2 P items; the results must equal the oracle's."""
    rng = np.random.default_rng(43)
    d = synth.generate("c2", n=2000, seed=9)
    pairs = [tuple(_random_panel(rng, 2, 20, 26, 0.0)) for _ in range(2)]
    seqs = []
    for _ in range(1900):
        s = ""
        for f, r in pairs:
            s += (rand_dna(rng, int(rng.integers(0, 15))) + f + rand_dna(rng, int(rng.integers(30, 120)))
                  + r)
        seqs.append(s + rand_dna(rng, int(rng.integers(0, 15))))
    blob, offs, lens = oracle.pack_ascii(seqs)
    exp = oracle.run_batch(oracle.Panel([p[0] for p in pairs], oracle.FRONT),
                           oracle.Panel([p[1] for p in pairs], oracle.BACK),
                           blob, offs, lens, mode=2, use_rc=False, threads=8)
    with lib.Context(0) as c:
        _assert_same(_gpu_two_round(c, d), _oracle_two_round(d))
        c.set_panel(0, [p[0] for p in pairs], lib.DMX_FRONT)
        c.set_panel(1, [p[1] for p in pairs], lib.DMX_BACK)
        c.set_mode(lib.MODE_LINKED)
        _assert_same(c.run(lib.pack(blob, offs, lens)), exp)
    assert (exp["bin1"] >= 0).mean() > 0.9


def rand_dna(rng, n):
    return "".join(rng.choice(list("ACGT"), size=n))


def test_run_multi_shards_equal_single_context(ctx):
    """dmx_run_multi: length-balanced contiguous shards over several contexts (here three on
    one GPU, each with its own stream and host thread) give the single-context results in
    input order, and the summed per-bin counts."""
    d = synth.generate("c2", n=20000, seed=31)
    exp = _gpu_two_round(ctx, d)
    exp_counts = ctx.counts()
    ctxs = [lib.Context(0) for _ in range(3)]
    try:
        for c in ctxs:
            c.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC)
            c.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC)
            c.set_mode(lib.MODE_TWO_ROUND)
        got, counts = lib.run_multi(ctxs, lib.pack(d["blob"], d["offsets"], d["lengths"]))
        _assert_same(got, exp)
        assert np.array_equal(counts, exp_counts)
        # more shards than reads: empty shards are skipped
        small = synth.generate("c2", n=2, seed=3)
        g2, _ = lib.run_multi(ctxs, lib.pack(small["blob"], small["offsets"], small["lengths"]))
        _assert_same(g2, _gpu_two_round(ctx, small))
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("where", ["front", "back", "mixed"])
@pytest.mark.parametrize("e,mo", [(0.1, 3), (0.25, 3), (3, 1), (4, 2)])
def test_tie_stress_short_adapters(ctx, where, e, mo):
    """Short adapters (3..14 nt, some IUPAC) against short reads give many equal-score matches
    on both strands and across adapters: every cutadapt tie rule (forward over RC on equal
    score whatever the errors, fewer errors, earlier adapter, earlier cell) is exercised.  With
    absolute error counts (-e 3 / 4) and short -O, accepted matches can score <= 0, and
    ReverseComplementer may take an orientation that matches nothing (its "no match" = 0)."""
    rng = np.random.default_rng({"front": 41, "back": 42, "mixed": 43}[where] + int(e * 100))
    panel = _random_panel(rng, 12, 3, 14, 0.1)
    seqs = _reads_with(rng, panel, 4000, L=(0, 60), err=0.1)
    blob, offs, lens = oracle.pack_ascii(seqs)
    if where == "mixed":
        wh = [oracle.FRONT if rng.random() < 0.5 else oracle.BACK for _ in panel]
    else:
        wh = [oracle.FRONT if where == "front" else oracle.BACK] * len(panel)
    exp = oracle.run_batch(oracle.Panel(panel, wh, max_errors=e, min_overlap=mo), None, blob,
                           offs, lens, mode=0, use_rc=True, threads=8)
    ctx.set_panel_mixed(0, panel, [lib.DMX_FRONT if w == oracle.FRONT else lib.DMX_BACK
                                   for w in wh], True, e, mo)
    ctx.set_mode(lib.MODE_SINGLE)
    _assert_same(ctx.run(lib.pack(blob, offs, lens)), exp)


@pytest.mark.parametrize("seed", [0, 1])
def test_windowed_path_orientation_ties(ctx, seed):
    """The shared-suffix window path (real SP5 / SP27rc panels) on reads built to tie across
    orientations and adapters: one adapter copy on the forward strand and another on the
    reverse strand (full, partial at a read end, or internal), with 0-8 % edits each."""
    rng = np.random.default_rng(900 + seed)
    _, sp5 = panel.load_panel(panel.SP5_FASTA)
    _, sp27 = panel.load_panel(panel.SP27RC_FASTA)
    seqs = []
    for _ in range(6000):
        body = "".join(rng.choice(list("ACGT"), size=int(rng.integers(60, 400))))
        pan = sp5 if rng.random() < 0.6 else sp27
        a = _mutate(rng, pan[int(rng.integers(len(pan)))], float(rng.choice([0, 0.03, 0.08])))
        b = _mutate(rng, pan[int(rng.integers(len(pan)))], float(rng.choice([0, 0.03, 0.08])))
        if rng.random() < 0.4:
            a = a[int(rng.integers(0, len(a) - 3)):]
        if rng.random() < 0.4:
            b = b[:int(rng.integers(3, len(b)))]
        u = rng.random()
        if u < 0.4:
            s = a + body + oracle_rc(b)
        elif u < 0.7:
            s = oracle_rc(b) + body + a
        else:
            s = body[:30] + a + body[30:] + oracle_rc(b)
        seqs.append(s)
    blob, offs, lens = oracle.pack_ascii(seqs)
    for p1, w in ((sp5, oracle.FRONT), (sp27, oracle.BACK)):
        exp = oracle.run_batch(oracle.Panel(p1, w), None, blob, offs, lens, mode=0, use_rc=True,
                               threads=8)
        ctx.set_panel(0, p1, (lib.DMX_FRONT if w == oracle.FRONT else lib.DMX_BACK) | lib.DMX_RC)
        ctx.set_mode(lib.MODE_SINGLE)
        _assert_same(ctx.run(lib.pack(blob, offs, lens)), exp)
    exp = oracle.run_batch(oracle.Panel(sp5, oracle.FRONT), oracle.Panel(sp27, oracle.BACK), blob,
                           offs, lens, mode=1, use_rc=True, threads=8)
    ctx.set_panel(0, sp5, lib.DMX_FRONT | lib.DMX_RC)
    ctx.set_panel(1, sp27, lib.DMX_BACK | lib.DMX_RC)
    ctx.set_mode(lib.MODE_TWO_ROUND)
    _assert_same(ctx.run(lib.pack(blob, offs, lens)), exp)


def _mutate(rng, a, err):
    out = []
    for c in a:
        r = rng.random()
        if r < err * 0.6:
            out.append("ACGT"[int(rng.integers(4))])
        elif r < err * 0.8:
            pass
        elif r < err:
            out += [c, "ACGT"[int(rng.integers(4))]]
        else:
            out.append(c)
    return "".join(out)


def test_two_round_nonpositive_scores(ctx):
    """Both rounds with per-orientation winners (-e 3 on the real panels' 17-nt index parts
    would not do: short random panels, -O 2): an unmatched read may be taken RC'd in either
    round, and round 2 runs on whatever round 1 chose."""
    rng = np.random.default_rng(77)
    p1, p2 = _random_panel(rng, 6, 4, 9), _random_panel(rng, 6, 4, 9)
    seqs = _reads_with(rng, p1 + p2, 5000, L=(0, 50), err=0.1)
    blob, offs, lens = oracle.pack_ascii(seqs)
    exp = oracle.run_batch(oracle.Panel(p1, oracle.FRONT, max_errors=3, min_overlap=2),
                           oracle.Panel(p2, oracle.BACK, max_errors=3, min_overlap=2), blob, offs,
                           lens, mode=1, use_rc=True, threads=8)
    assert ((exp["bin1"] >= 0) & (exp["bin2"] < 0) & (exp["rc2"] == 1)).any()
    ctx.set_panel(0, p1, lib.DMX_FRONT | lib.DMX_RC, 3, 2)
    ctx.set_panel(1, p2, lib.DMX_BACK | lib.DMX_RC, 3, 2)
    ctx.set_mode(lib.MODE_TWO_ROUND)
    _assert_same(ctx.run(lib.pack(blob, offs, lens)), exp)


def _pis_panel(rng, n, pre, suf, lmin, lmax):
    """P + I_a + S panels (shared prefix and suffix, index blocks of lmin..lmax nt): the shape the
    index screen runs on, including blocks longer than the packed screen's 16-bit
    halves (cut to their last 16 rows)."""
    P = "".join(rng.choice(list("ACGT"), pre))
    S = "".join(rng.choice(list("ACGT"), suf))
    return [P + "".join(rng.choice(list("ACGT"), int(rng.integers(lmin, lmax + 1)))) + S
            for _ in range(n)]


@pytest.mark.parametrize("seed,n,lmin,lmax,where", [
    (1, 24, 17, 17, "front"), (2, 24, 17, 17, "back"), (3, 13, 1, 16, "back"),
    (4, 30, 12, 32, "front"), (5, 7, 20, 32, "back"), (6, 32, 5, 24, "back")])
def test_packed_index_screen(ctx, seed, n, lmin, lmax, where, monkeypatch):
    """The packed index screen (four adapters per lane in 16-bit halves) against the oracle, the
    one-lane-per-adapter screen (DMX_SCREEN_V1) and no screen, on P + I_a + S panels with index
    blocks of 1..32 nt, two rounds (the other round's panel has the real M13 shape)."""
    rng = np.random.default_rng(seed)
    pre, suf = int(rng.integers(10, 21)), int(rng.integers(10, 21))
    lmax = min(lmax, 64 - pre - suf)
    pan = _pis_panel(rng, n, pre, suf, min(lmin, lmax), lmax)
    d = synth.generate("c2", n=1500, seed=seed)
    reads = synth.to_strings(d)
    extra = _reads_with(rng, pan, 3000, L=(0, 500), err=0.05)
    seqs = reads + extra
    blob, offs, lens = oracle.pack_ascii(seqs)
    if where == "front":
        p1, p2 = pan, d["sp27"]
    else:
        p1, p2 = d["sp5"], pan
    exp = oracle.run_batch(oracle.Panel(p1, oracle.FRONT), oracle.Panel(p2, oracle.BACK), blob,
                           offs, lens, mode=1, threads=8)
    packed = lib.pack(blob, offs, lens)
    tasks = {}
    for variant in ("packed", "v1", "none"):
        monkeypatch.delenv("DMX_SCREEN_V1", raising=False)
        monkeypatch.delenv("DMX_NO_SCREEN", raising=False)
        if variant == "v1":
            monkeypatch.setenv("DMX_SCREEN_V1", "1")
        if variant == "none":
            monkeypatch.setenv("DMX_NO_SCREEN", "1")
        with lib.Context(0) as c:
            c.set_panel(0, p1, lib.DMX_FRONT | lib.DMX_RC)
            c.set_panel(1, p2, lib.DMX_BACK | lib.DMX_RC)
            c.set_mode(lib.MODE_TWO_ROUND)
            c.load(packed)
            c.exec()
            _assert_same(c.fetch(), exp)
            tasks[variant] = c.stats()["tasks"]
    # the packed screen is the same kind of filter: it still prunes (blocks > 16 nt lose rows)
    r = 0 if where == "front" else 1
    assert tasks["packed"][r] >= tasks["v1"][r]
    assert tasks["packed"][r] <= 2 * tasks["v1"][r] + 100


def _run_mode(ctx, d, linked):
    f = 0 if linked else lib.DMX_RC
    ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | f)
    ctx.set_panel(1, d["sp27"], lib.DMX_BACK | f)
    ctx.set_mode(lib.MODE_LINKED if linked else lib.MODE_TWO_ROUND)
    return ctx.run(lib.pack(d["blob"], d["offsets"], d["lengths"])), ctx.counts()


def _sub(d, lo, hi):
    return dict(d, offsets=d["offsets"][lo:hi], lengths=d["lengths"][lo:hi])


@pytest.mark.parametrize("config", ["c2", "c5"])
def test_large_batch_equals_sub_batches(ctx, config):
    """Above 2048 x 256 reads the finalize kernels take several passes per block (block-stride,
    one bin-histogram flush per block, the round-2 item list claimed per pass). A 1.2 M-read
    batch gives the per-read results and per-bin counts of the same reads run as three 400 k
    sub-batches (one pass each), and a sample of its reads matches the oracle."""
    n = 1_200_000
    linked = config == "c5"
    d = synth.generate(config, n=n, seed=57)
    got, counts = _run_mode(ctx, d, linked)
    parts, csum = [], None
    for lo in range(0, n, 400_000):
        g, c = _run_mode(ctx, _sub(d, lo, lo + 400_000), linked)
        parts.append(g)
        csum = c if csum is None else csum + c
    _assert_same(got, np.concatenate(parts))
    assert np.array_equal(counts, csum)
    idx = np.sort(np.random.default_rng(5).choice(n, 3000, replace=False))
    exp = oracle.run_batch(oracle.Panel(d["sp5"], oracle.FRONT),
                           oracle.Panel(d["sp27"], oracle.BACK), d["blob"], d["offsets"][idx],
                           d["lengths"][idx], mode=2 if linked else 1, use_rc=not linked,
                           threads=8)
    _assert_same(got[idx], exp)


def test_screen_far_before_short_views(ctx):
    """The index screen of a 3' panel with a long shared prefix and suffix at -e 0.3 starts its
    warm-up up to m + k columns before the view, more than the 64-nt head pad for a short first
    read (a parity sweep, seed 46, faulted there): such positions are read at -64. Short and
    empty reads first and last, both strands, vs the oracle."""
    rng = np.random.default_rng(925)
    pre, suf = rand_dna(rng, 12), rand_dna(rng, 21)
    panel = [pre + rand_dna(rng, int(rng.integers(6, 28))) + suf for _ in range(15)]
    seqs = ["", "A", "ACG", rand_dna(rng, 5)]
    for _ in range(600):
        s = rand_dna(rng, int(rng.integers(0, 160)))
        if rng.random() < 0.5:
            a = panel[int(rng.integers(len(panel)))]
            cut = int(rng.integers(1, len(a) + 1))
            s = s + a[:cut]
        seqs.append(s)
    seqs += ["", "T", rand_dna(rng, 7)]
    blob, offs, lens = oracle.pack_ascii(seqs)
    for use_rc in (True, False):
        exp = oracle.run_batch(oracle.Panel(panel, oracle.BACK, max_errors=0.3, min_overlap=3),
                               None, blob, offs, lens, mode=0, use_rc=use_rc, threads=8)
        ctx.set_panel(0, panel, lib.DMX_BACK | (lib.DMX_RC if use_rc else 0), 0.3, 3)
        ctx.set_mode(lib.MODE_SINGLE)
        _assert_same(ctx.run(lib.pack(blob, offs, lens)), exp)


@pytest.mark.parametrize("n_rate,where", [(0.004, "spread"), (0.03, "spread"),
                                          (0.05, "adapters")])
def test_n_dense_reads_and_clean_flags(ctx, n_rate, where, monkeypatch):
    """the filter, the prefix verification and the index screen read a read's N
    as A (still necessary conditions), and the filter marks a window `clean` when the no-match
    mask is zero over every view position the window scan and the band DP read for it, which
    then skip the mask.  Reads with N sprinkled everywhere, or right at and before the adapters
    (inside the clean reach, where a wrong flag would turn an N into a match), two rounds on the
    24 x 24 panels with --rc: every result byte equals the oracle's, and equals the run with the
    clean flags off (DMX_NO_CLEAN) and with every stage reading the mask (no window is clean)."""
    d = synth.generate("c2x24", n=6000, seed=int(n_rate * 1000) + (7 if where == "adapters" else 0))
    seqs = synth.to_strings(d)
    rng = np.random.default_rng(int(n_rate * 1e4))
    out = []
    for s in seqs:
        b = bytearray(s.encode())
        if where == "spread":
            m = rng.random(len(b)) < n_rate
        else:   # the ends: adapters and the positions just before / after them
            m = np.zeros(len(b), bool)
            k = min(len(b), 160)
            m[:k] = rng.random(k) < 0.03
            m[len(b) - k:] |= rng.random(k) < 0.03
        for i in np.nonzero(m)[0]:
            b[i] = ord("N")
        out.append(b.decode())
    blob, offs, lens = oracle.pack_ascii(out)
    exp = oracle.run_batch(oracle.Panel(d["sp5"], oracle.FRONT),
                           oracle.Panel(d["sp27"], oracle.BACK), blob, offs, lens, mode=1,
                           threads=8)
    ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC)
    ctx.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC)
    ctx.set_mode(lib.MODE_TWO_ROUND)
    p = lib.pack(blob, offs, lens)
    got = ctx.run(p)
    _assert_same(got, exp)
    wins = ctx.debug_fetch(lib.DBG_VERIFIED, 1)
    assert len(wins) > 0 and (wins["strand"] & 2).any()   # some windows run clean
    monkeypatch.setenv("DMX_NO_CLEAN", "1")
    ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC)
    ctx.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC)
    got2 = ctx.run(p)
    assert (ctx.debug_fetch(lib.DBG_VERIFIED, 1)["strand"] & 2).sum() == 0
    assert got2.tobytes() == got.tobytes()


@pytest.mark.parametrize("variant", ["scan_band", "scan_ring", "filter_ring", "two_round"])
def test_empty_reads_accept_whole_adapter_deletion(ctx, variant, monkeypatch):
    """cutadapt's last-column scan runs i = first_i .. m: in an EMPTY read the cell (m, 0) of a
    3' adapter (every adapter character deleted: cost m, score -2m) is seen only there, and is
    accepted when the error allowance reaches m (an absolute -e >= m).  A parity sweep (seed 48,
    round 5) found the GPU skipping it (row loops ran i < m).  Empty reads among short ones,
    BACK panels with --rc, on the full scan with band or ring resolve, the windowed path, and
    the second round of a two-round run (empty round-1 tails)."""
    rng = np.random.default_rng(48)
    if variant == "filter_ring":
        suf = rand_dna(rng, 12)
        panel = [rand_dna(rng, int(rng.integers(0, 4))) + suf for _ in range(6)]
        e = 12.0
    else:
        panel = ["GACG", "AGCTG", "CCAA", "ACT", "GAC", "TTT", "CGTCC"]
        e = 3.0
    if variant == "scan_ring" or variant == "filter_ring":
        monkeypatch.setenv("DMX_RESOLVE", "ring")
    seqs = []
    for _ in range(400):
        u = rng.random()
        seqs.append("" if u < 0.3 else rand_dna(rng, int(rng.integers(1, 12))))
    seqs += ["", ""]
    blob, offs, lens = oracle.pack_ascii(seqs)
    with lib.Context(0) as c:
        if variant == "two_round":
            front = [rand_dna(rng, 9) for _ in range(3)]
            reads = [front[int(rng.integers(3))] + s if rng.random() < 0.7 else s for s in seqs]
            blob, offs, lens = oracle.pack_ascii(reads)
            exp = oracle.run_batch(oracle.Panel(front, oracle.FRONT),
                                   oracle.Panel(panel, oracle.BACK, max_errors=e), blob, offs,
                                   lens, mode=1, threads=8)
            c.set_panel(0, front, lib.DMX_FRONT | lib.DMX_RC)
            c.set_panel(1, panel, lib.DMX_BACK | lib.DMX_RC, e, 3)
            c.set_mode(lib.MODE_TWO_ROUND)
            got = c.run(lib.pack(blob, offs, lens))
            assert (exp["bin2"] >= 0).any()
        else:
            exp = oracle.run_batch(oracle.Panel(panel, oracle.BACK, max_errors=e), None, blob,
                                   offs, lens, mode=0, use_rc=True, threads=8)
            c.set_panel(0, panel, lib.DMX_BACK | lib.DMX_RC, e, 3)
            c.set_mode(lib.MODE_SINGLE)
            got = c.run(lib.pack(blob, offs, lens))
            empty = lens == 0
            assert (exp["bin1"][empty] >= 0).all()   # the whole-deletion cell is accepted
    _assert_same(got, exp)
