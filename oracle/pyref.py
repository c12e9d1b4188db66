"""ORACLE — TEST INFRASTRUCTURE ONLY (pure-Python, small cases).

A second, independent CPU restatement of cutadapt 4.9's ``Aligner.locate`` semantics
(upstream ``cutadapt/_align.pyx``; call sites in the reference:
``scripts/02_cutadapt_loop.sh:64-72,91-103``, ``scripts/04_cleaning_primers.sh:371-388``).

Unlike ``cutadapt_oracle.c`` (a literal one-column DP with Ukkonen's cut-off and its stale
cells), this keeps the FULL (m+1) x (n+1) matrix and evaluates every cell, then scans the
candidates in cutadapt's order.  Agreement of the two formulations is the evidence that the
cut-off never changes an accepted result ("Why a full-column scan is exact").

PARITY UNPINNED: the reference holds no fixtures for this path.
Only for small inputs (pure Python loops).
"""
from __future__ import annotations

REF_START, QUERY_START, REF_END, QUERY_STOP = 1, 2, 4, 8
FRONT = QUERY_START | QUERY_STOP | REF_START
BACK = QUERY_START | QUERY_STOP | REF_END

_IUPAC = {"A": 1, "C": 2, "G": 4, "T": 8, "U": 8, "R": 5, "Y": 10, "S": 6, "W": 9, "K": 12,
          "M": 3, "B": 14, "D": 13, "H": 11, "V": 7, "N": 15}
_COMP = str.maketrans("ACGTUMRWSYKVHDBNacgtumrwsykvhdbn", "TGCAAKYWSRMBDHVNtgcaakywsrmbdhvn")


# The readings this restatement takes of the rules marked [UNVERIFIED] (cutadapt 4.9 source is
# not available here).  tests/test_oracle.py switches them to the alternative readings to show
# that every case of tools/unverified_cases.py (run against a real cutadapt 4.9 by
# tools/parity_vs_cutadapt.sh) tells the two readings apart.
DEFAULT_RULES = {
    "best_init": "none",         # locate's first best: any acceptable cell  | "zero": score 0
    "tie": "lower_cost",         # locate, equal score: lower cost wins     | "first": keep first
    "col0": "minus2i",           # BACK column 0: score -2 i                | "zero": score 0
    "besttie": "fewer_errors",   # best_match, equal score: fewer errors    | "first": file order
    "rc": "strict",              # --rc: reverse complement iff score >     | "geq": iff >=
    "linked": "both",            # -g F...R: both parts required            | "front": front alone
}
RULES = dict(DEFAULT_RULES)


class rules:
    """with rules(tie="first"): ... — evaluate under an alternative reading."""

    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        self.saved = dict(RULES)
        RULES.update(self.kw)

    def __exit__(self, *exc):
        RULES.clear()
        RULES.update(self.saved)


def revcomp(s: str) -> str:
    return s.translate(_COMP)[::-1]


def _acgt(c: str) -> int:
    v = _IUPAC.get(c.upper(), 0)
    return v if v in (1, 2, 4, 8) else 0


def locate(ref: str, query: str, max_error_rate: float, flags: int, min_overlap: int = 3):
    """Full-matrix restatement. Returns (ref_start, ref_stop, q_start, q_stop, score, errors)."""
    m, n = len(ref), len(query)
    wildcard_ref = not set(ref) <= set("ACGT")
    if wildcard_ref:
        r = [_IUPAC.get(c, 0) for c in ref]
        q = [_acgt(c) for c in query]
        eq = lambda a, b: (a & b) != 0  # noqa: E731
    else:
        r = list(ref)
        q = list(query.upper())
        eq = lambda a, b: a == b  # noqa: E731
    n_counts = [0] * (m + 1)
    nc = 0
    for i in range(m):
        n_counts[i] = nc
        nc += ref[i] in "Nn"
    n_counts[m] = nc
    eff_len = m - nc if wildcard_ref else m
    start_ref, start_q = bool(flags & REF_START), bool(flags & QUERY_START)
    stop_ref, stop_q = bool(flags & REF_END), bool(flags & QUERY_STOP)
    assert start_q and stop_q, "only FRONT/BACK-style flags are restated here"
    # cell = (cost, score, origin)
    C = [[None] * (n + 1) for _ in range(m + 1)]
    for i in range(m + 1):
        C[i][0] = (0, 0, -i) if start_ref else (i, -2 * i if RULES["col0"] == "minus2i" else 0,
                                                    0)
    for j in range(1, n + 1):
        C[0][j] = (0, 0, j)
        for i in range(1, m + 1):
            d, up, left = C[i - 1][j - 1], C[i - 1][j], C[i][j - 1]
            if eq(r[i - 1], q[j - 1]):
                C[i][j] = (d[0], d[1] + 1, d[2])
            elif d[0] + 1 <= left[0] + 1 and d[0] + 1 <= up[0] + 1:
                C[i][j] = (d[0] + 1, d[1] - 1, d[2])
            elif up[0] + 1 <= left[0] + 1:
                C[i][j] = (up[0] + 1, up[1] - 2, up[2])
            else:
                C[i][j] = (left[0] + 1, left[1] - 2, left[2])

    def acceptable(i, cell):
        length = i + min(cell[2], 0)
        eff = length
        if wildcard_ref:
            eff = length - n_counts[length] if length < m else eff_len
        return length >= min_overlap and cell[0] <= eff * max_error_rate

    # [UNVERIFIED] no initial score: any acceptable cell can win, also one scoring <= 0 (see
    # cutadapt_oracle.c "the initial best score"; tools/parity_vs_cutadapt.sh case "negscore")
    best = None  # (score, cost, origin, ref_stop, q_stop)
    if RULES["best_init"] == "zero":
        best = (0, m + n + 1, 0, m, n)
    lower_cost = RULES["tie"] == "lower_cost"

    def better(cell):
        return best is None or cell[1] > best[0] or (lower_cost and cell[1] == best[0]
                                                     and cell[0] < best[1])
    for j in range(1, n + 1):
        cell = C[m][j]
        if acceptable(m, cell) and better(cell):
            best = (cell[1], cell[0], cell[2], m, j)
    for i in range(0 if stop_ref else m, m + 1):
        cell = C[i][n]
        if acceptable(i, cell) and better(cell):
            best = (cell[1], cell[0], cell[2], i, n)
    if best is None or best[1] == m + n + 1:   # (the "zero" reading's seed: no match)
        return None
    score, cost, origin, rstop, qstop = best
    if origin >= 0:
        return (0, rstop, origin, qstop, score, cost)
    return (-origin, rstop, 0, qstop, score, cost)


def best_match(adapters, where, seq, e=0.1, min_overlap=3):
    """modifiers.AdapterCutter.best_match: (index, match) or (-1, None)."""
    best, bm = -1, None
    for a, ad in enumerate(adapters):
        rate = e / len(ad) if e >= 1 else e
        mt = locate(ad, seq, rate, where[a], min_overlap)
        if mt is None:
            continue
        if bm is None or mt[4] > bm[4] or (RULES["besttie"] == "fewer_errors" and
                                           mt[4] == bm[4] and mt[5] < bm[5]):
            best, bm = a, mt
    return best, bm


def demux_round(adapters, where, seq, use_rc=True, e=0.1, min_overlap=3):
    """ReverseComplementer: returns (index, is_rc, match, trimmed_seq)."""
    af, mf = best_match(adapters, where, seq, e, min_overlap)
    ar, mr = (-1, None)
    rc = revcomp(seq)
    if use_rc:
        ar, mr = best_match(adapters, where, rc, e, min_overlap)
    fs = mf[4] if mf else 0
    rs = mr[4] if mr else 0
    if use_rc and (rs > fs or (RULES["rc"] == "geq" and mr is not None and rs == fs)):
        a, mt, src, is_rc = ar, mr, rc, True
    else:
        a, mt, src, is_rc = af, mf, seq, False
    if a < 0:   # nothing matched in the chosen orientation (may still be the RC read)
        return -1, is_rc, None, src
    trimmed = src[mt[3]:] if where[a] == FRONT else src[:mt[2]]
    return a, is_rc, mt, trimmed


def two_round(sp5, sp27, seq, use_rc=True, e=0.1):
    a, rc1, m1, t1 = demux_round(sp5, [FRONT] * len(sp5), seq, use_rc, e)
    if a < 0:
        return (a, rc1, m1, -1, False, None, None)
    b, rc2, m2, t2 = demux_round(sp27, [BACK] * len(sp27), t1, use_rc, e)
    return (a, rc1, m1, b, rc2, m2, t2 if b >= 0 else None)


def linked(fronts, backs, seq, e=0.1):
    """-g F...R without anchoring: LinkedAdapter.match_to with both parts required (cutadapt 4.9
    adapters.py, LinkedAdapter; front on the read, back on read[front.rstop:]); the best pair is
    picked by AdapterCutter.best_match on LinkedMatch.score / .errors = summed parts.
    Returns (index, front_match, back_match, trimmed) or (-1, None, None, seq)."""
    best, bf, bb, bs, be = -1, None, None, 0, 0
    for a, (f, r) in enumerate(zip(fronts, backs)):
        mf = locate(f, seq, e / len(f) if e >= 1 else e, FRONT)
        if mf is None:
            continue
        rest = seq[mf[3]:]
        mb = locate(r, rest, e / len(r) if e >= 1 else e, BACK)
        if mb is None:
            if RULES["linked"] != "front":
                continue
            s, er = mf[4], mf[5]
        else:
            s, er = mf[4] + mb[4], mf[5] + mb[5]
        if best < 0 or s > bs or (s == bs and er < be):
            best, bf, bb, bs, be = a, mf, mb, s, er
    if best < 0:
        return -1, None, None, seq
    if bb is None:   # the "front" reading: the front part alone
        return best, bf, None, seq[bf[3]:]
    return best, bf, bb, seq[bf[3]:][:bb[2]]
