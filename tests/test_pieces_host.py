"""Piece screen tables on the host (no GPU).

The library's own piece table (dmx_panel_pieces) drives a pure-Python model of the screen: sample
an 8-mer every `step` positions, check every entry of a sampled 8-mer for an exact copy of its
piece, and mark the alignment end columns the entry allows.  Every alignment of all adapter rows
with at most K = acc[m] edits must end in a marked column of the view that holds the adapter —
the exactness argument the GPU kernels rest on (pigeonhole over K + 1 disjoint pieces).  Reads are
built with exactly K edits placed one per piece in K of the K + 1 pieces, so that exactly one piece
survives, for every surviving piece, in both orientations.
"""
import numpy as np
import pytest

from dmx import lib, synth

CODE = {"A": 0, "C": 1, "G": 2, "T": 3}
COMP = {"A": "T", "C": "G", "G": "C", "T": "A", "N": "N"}


def revcomp(s):
    return "".join(COMP[c] for c in reversed(s))


def full_k(m, rate):
    """acc[m]: the largest cost an alignment of all m rows may have (IEEE double, as the host)."""
    return max(c for c in range(128) if c <= m * rate)


def pieces_of(m, K):
    """The K + 1 row pieces build_pieces cuts (csrc/dmx_api.cpp): [r0, r0 + min(16, r1 - r0))."""
    np_ = K + 1
    out = []
    for p in range(np_):
        r0, r1 = p * m // np_, (p + 1) * m // np_
        out.append((r0, r0 + min(16, r1 - r0)))
    return out


def decode(val, ln):
    return "".join("ACGT"[(val >> (2 * i)) & 3] for i in range(ln))


def model_marks(read, ents, step, n_orient):
    """Columns (1-based alignment end columns) the screen marks in views 0 and 1 of `read`."""
    n = len(read)
    by_key = {}
    for e in ents:
        by_key.setdefault((e["val"] >> (2 * e["off"])) & 0xFFFF, []).append(e)
    marks = [set(), set()]
    codes = [CODE.get(c, 0) for c in read]   # N read as A (the screen's codes)
    for x in range(0, max(0, n - 7), step):
        k = 0
        for i in range(8):
            k |= codes[x + i] << (2 * i)
        for e in by_key.get(k, []):
            g = x - e["off"]
            ln = e["len"]
            if g < 0 or g + ln > n:
                continue
            v = 0
            for i in range(ln):
                v |= codes[g + i] << (2 * i)
            if v != e["val"]:
                continue
            if e["o"] == 0:
                pe = g + ln
            else:
                pe = n - g
            if e["o"] >= n_orient:
                continue
            for j in range(max(1, pe + e["dlo"]), min(n, pe + e["dhi"]) + 1):
                marks[e["o"]].add(j)
    return marks


def mutate(rng, adapter, pieces, survive):
    """adapter with one edit (sub / ins / del) inside each piece except `survive`; returns the
    sequenced copy (its full alignment has len(pieces) - 1 edits and ends at its last base)."""
    edits = {}
    for p, (r0, r1) in enumerate(pieces):
        if p != survive:
            edits[int(rng.integers(r0, r1))] = ("sub", "ins", "del")[int(rng.integers(3))]
    out = []
    for i, c in enumerate(adapter):
        t = edits.get(i)
        if t == "sub":
            out.append("ACGT".replace(c, "")[int(rng.integers(3))])
        elif t == "ins":
            out += ["ACGT"[int(rng.integers(4))], c]
        elif t == "del":
            pass
        else:
            out.append(c)
    return "".join(out)


def test_benchmark_panels_use_the_piece_screen():
    n1, s5, n2, s27 = synth.panels(24, 24)
    rc, info, ents = lib.panel_pieces(s5, lib.DMX_FRONT | lib.DMX_RC)
    assert rc == 0 and info["step"] == 2 and info["entries"] == len(ents) > 0
    assert info["front_reach"] == 59 + 5   # m + acc[m]: alignments entering at column 0
    rc, info2, _ = lib.panel_pieces(s27, lib.DMX_BACK | lib.DMX_RC)
    assert rc == 0 and info2["step"] == 2 and info2["front_reach"] == 0
    # every adapter's K + 1 pieces are in the table, both orientations, with their end range
    for s in s5:
        K = full_k(len(s), 0.1)
        for r0, r1 in pieces_of(len(s), K):
            for o, txt in ((0, s[r0:r1]), (1, revcomp(s[r0:r1]))):
                hit = [e for e in ents if e["o"] == o and e["len"] == r1 - r0 and
                       decode(e["val"], e["len"]) == txt]
                assert hit, (s, r0, r1, o)
                d = len(s) - r1
                assert min(e["dlo"] for e in hit) <= d - K and max(e["dhi"] for e in hit) >= d + K


@pytest.mark.parametrize("seqs,where,why", [
    (["ACGTNACGTACGTACGTACGTACGTACGT"] * 2, lib.DMX_FRONT, "IUPAC adapter"),
    (["ACGTAGCTAGCTAGGATCGA", "TTGACGTAGCTAGCATCGAT"], lib.DMX_BACK, "pieces < 8 nt"),
])
def test_piece_screen_off(seqs, where, why):
    rc, info, ents = lib.panel_pieces(seqs, where | lib.DMX_RC)
    assert rc == 0 and info["step"] == 0 and not ents, why


def test_no_pieces_switch(monkeypatch):
    n1, s5, n2, s27 = synth.panels(4, 4)
    monkeypatch.setenv("DMX_NO_PIECES", "1")
    rc, info, _ = lib.panel_pieces(s5, lib.DMX_FRONT | lib.DMX_RC)
    assert rc == 0 and info["step"] == 0


def _panels():
    n1, s5, n2, s27 = synth.panels(24, 24)
    rng = np.random.default_rng(5)
    suffix = "".join(rng.choice(list("ACGT"), size=20))   # the filter needs a shared suffix
    rand = ["".join(rng.choice(list("ACGT"), size=int(L))) + suffix
            for L in rng.integers(30, 45, size=8)]
    return [("sp5", s5, lib.DMX_FRONT), ("sp27", s27, lib.DMX_BACK), ("random", rand, lib.DMX_BACK)]


@pytest.mark.parametrize("name,seqs,where", _panels())
def test_every_k_edit_alignment_ends_in_a_marked_column(name, seqs, where):
    rc, info, ents = lib.panel_pieces(seqs, where | lib.DMX_RC)
    assert rc == 0 and info["step"] > 0, name
    rng = np.random.default_rng(len(name))
    checked = 0
    for a, ad in enumerate(seqs):
        K = full_k(len(ad), 0.1)
        pcs = pieces_of(len(ad), K)
        for survive in range(K + 1):
            for rc_read in (False, True):
                copy = mutate(rng, ad, pcs, survive)
                left = "".join(rng.choice(list("ACGT"), size=int(rng.integers(0, 90))))
                right = "".join(rng.choice(list("ACGT"), size=int(rng.integers(0, 90))))
                view0 = left + copy + right
                end = len(left) + len(copy)          # the K-edit alignment's end column
                read = revcomp(view0) if rc_read else view0
                marks = model_marks(read, ents, info["step"], 2)
                assert end in marks[1 if rc_read else 0], (name, a, survive, rc_read)
                checked += 1
    assert checked == sum((full_k(len(s), 0.1) + 1) * 2 for s in seqs)


def test_reads_with_n_only_add_marks():
    """N is read as A by the screen: a copy stays a copy, other 8-mers may turn into hits."""
    n1, s5, n2, s27 = synth.panels(24, 24)
    rc, info, ents = lib.panel_pieces(s5, lib.DMX_FRONT | lib.DMX_RC)
    rng = np.random.default_rng(3)
    for _ in range(40):
        ad = s5[int(rng.integers(len(s5)))]
        K = full_k(len(ad), 0.1)
        pcs = pieces_of(len(ad), K)
        survive = int(rng.integers(K + 1))
        copy = mutate(rng, ad, pcs, survive)
        left = "".join(rng.choice(list("ACGTN"), size=40, p=[.24, .24, .24, .24, .04]))
        read = left + copy
        marks = model_marks(read, ents, info["step"], 2)
        assert len(read) in marks[0]


def _shared_flank_panel(rng, n, pre, suf, lo, hi):
    """Adapters that share a constant prefix and suffix (as in the sweep's random panels): the
    pieces that straddle a shared block are the ones whose sampled window starts past offset 0."""
    p = "".join(rng.choice(list("ACGT"), size=pre))
    s = "".join(rng.choice(list("ACGT"), size=suf))
    return [p + "".join(rng.choice(list("ACGT"), size=int(L))) + s
            for L in rng.integers(lo, hi, size=n)]


# a panel of tools/parity_sweep.py seed 56 whose pieces took sampled windows at offsets 4 .. 8,
# beyond the entries' 2-bit offset field (read back as offsets 0 .. 3 with a shifted end range)
SWEEP56_PANEL = [
    "CGAAGACTCGCTCCTAGGTTTCGGACGGCCCGTGTTTACAACCCCTACGCC", "CGAAGACTCTAACCACAACCCCTACGCC",
    "CGAAGACTCCAACGGAACGGTCCCACAACCCCTACGCC", "CGAAGACTCGCTATCATTTTTTGCTAAACAACCCCTACGCC",
    "CGAAGACTCTCTCGCCAGTAGTTGGGGAATCCCCTTAACAACCCCTACGCC",
    "CGAAGACTCCCGACGGTTCTAAACTTCCTTACAACCCCTACGCC", "CGAAGACTCCCTATGGCGAATTTAGACAACCCCTACGCC",
    "CGAAGACTCCAGCCTGTTGAGTAAATTACAACCCCTACGCC", "CGAAGACTCGAATCCGCCAACAACCCCTACGCC",
    "CGAAGACTCAAGCCAGTACAACCCCTACGCC", "CGAAGACTCCGCGATACAACCCCTACGCC",
    "CGAAGACTCTAACGGCCGTGAAGAGGGGGTACACAACCCCTACGCC",
]


def _flank_cases():
    rng = np.random.default_rng(56)
    out = [("sweep56", SWEEP56_PANEL, lib.DMX_FRONT, 0.0)]
    for i, (where, rate) in enumerate([(lib.DMX_FRONT, 0.05), (lib.DMX_BACK, 0.0),
                                       (lib.DMX_BACK, 0.05), (lib.DMX_FRONT, 0.1)]):
        out.append((f"flank{i}", _shared_flank_panel(rng, 12, int(rng.integers(5, 14)),
                                                     int(rng.integers(8, 20)), 8, 35), where, rate))
    return out


@pytest.mark.parametrize("name,seqs,where,rate", _flank_cases())
def test_entries_keep_their_piece_end_range(name, seqs, where, rate):
    """Every entry of a piece carries the piece's own end range and an offset the screens can read
    back: the `step` sampled offsets of a piece are consecutive and start at 0 .. 4 - step."""
    rc, info, ents = lib.panel_pieces(seqs, where | lib.DMX_RC, rate)
    assert rc == 0 and info["step"] > 0, name
    by_piece = {}
    for e in ents:
        by_piece.setdefault((e["val"], e["len"], e["o"]), []).append(e)
    assert len(by_piece) == info["pieces"]
    for key, es in by_piece.items():
        assert len({(e["dlo"], e["dhi"]) for e in es}) == 1, (name, key)
        assert es[0]["dlo"] <= es[0]["dhi"]
        offs = sorted(e["off"] for e in es)
        assert offs == list(range(offs[0], offs[0] + info["step"])) and offs[-1] <= 3, (name, key)


@pytest.mark.parametrize("name,seqs,where,rate", _flank_cases())
def test_shared_flank_copies_end_in_marked_columns(name, seqs, where, rate):
    """Exact copies and K-edit copies (one surviving piece) of every adapter of a shared-flank
    panel, at every start modulo the sampling stride, end in a marked column."""
    rc, info, ents = lib.panel_pieces(seqs, where | lib.DMX_RC, rate)
    step = info["step"]
    rng = np.random.default_rng(len(name))
    for ad in seqs:
        K = full_k(len(ad), rate)
        pcs = pieces_of(len(ad), K)
        for survive in range(K + 1):
            for shift in range(step):
                copy = mutate(rng, ad, pcs, survive) if K else ad
                left = "".join(rng.choice(list("ACGT"), size=20 + shift))
                view0 = left + copy + "".join(rng.choice(list("ACGT"), size=30))
                for rc_read in (False, True):
                    read = revcomp(view0) if rc_read else view0
                    marks = model_marks(read, ents, step, 2)
                    assert len(left) + len(copy) in marks[1 if rc_read else 0], \
                        (name, ad, survive, shift, rc_read)


def test_entry_fields_on_random_panels():
    """The packed entry fields read back as built on 60 random panels (lengths 8..64, shared
    flanks or none, -e 0..0.3): per piece one end range, dlo <= dhi, `step` consecutive offsets
    <= 3, lengths 8..16; every key's 8-mer is the piece's codes at the entry's offset."""
    rng = np.random.default_rng(123)
    seen = 0
    for _ in range(60):
        n = int(rng.integers(1, 25))
        pre, suf = int(rng.integers(0, 16)), int(rng.integers(0, 24))
        lo = int(rng.integers(4, 30))
        seqs = [s[:64] for s in _shared_flank_panel(rng, n, pre, suf, lo, lo + 30)]
        seqs = [s for s in seqs if len(s) >= 8] or ["ACGTACGTACGTACGTAC"]
        where = lib.DMX_FRONT if rng.random() < 0.5 else lib.DMX_BACK
        rate = float(rng.choice([0.0, 0.05, 0.1, 0.1, 0.2, 0.3]))
        rc, info, ents = lib.panel_pieces(seqs, where | lib.DMX_RC, rate)
        assert rc == 0
        if not info["step"]:
            continue
        seen += 1
        by_piece = {}
        for e in ents:
            by_piece.setdefault((e["val"], e["len"], e["o"]), []).append(e)
        for es in by_piece.values():
            assert len({(e["dlo"], e["dhi"]) for e in es}) == 1
            assert es[0]["dlo"] <= es[0]["dhi"] and 8 <= es[0]["len"] <= 16
            offs = sorted(e["off"] for e in es)
            assert offs == list(range(offs[0], offs[0] + info["step"])) and offs[-1] <= 3
            assert offs[-1] + 8 <= es[0]["len"]
    assert seen >= 10
