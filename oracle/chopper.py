"""ORACLE — TEST INFRASTRUCTURE ONLY.  CPU restatement of the pychopper-style read
reorientation of scripts/01_pychopper.sh:45-57:

    pychopper -b M13_seqs_for_pychopper.fa -c M13_config_for_pychopper.txt -k LSK114 -Q 10
              -w RESCUED -u UNCLASS -l SHORT -S STATS -p -t 24 -m edlib IN > PASS

pychopper v2.7.0 and edlib are not vendored in /root/reference and not installed here, and the
reference holds no pychopper output: PARITY UNPINNED.  The semantics are the build's definition
(DESIGN.md §8d), restated from edlib's HW ("infix") alignment mode and pychopper's documented
options:

  labels    primer p of the -b FASTA (file order; name = first header word) is label 2p
            ("NAME"), its reverse complement label 2p+1 ("-NAME", the config's notation)
  hits      per label, one edlib HW / TASK_LOC call with k = int(cutoff * m) (edlib 1.3.x,
            edlib.cpp edlibAlign): D(j) = least edit distance of the label ending at read column
            j (IUPAC codes; a read N matches anything); best = min over j of D(j); no hits when
            best > k, else one hit per stop j with D(j) == best (edlib's end locations), its
            start the smallest s with editdist(label, read[s:j)) == best (edlib takes the last
            position of its reverse SHW alignment: the longest optimal alignment) —
            oracle/chop_oracle.c (plain O(mn) DP) or `hits_py` (pure Python, tiny cases)
  segments  a read's hits sorted by (start, stop, label); every pair of consecutive hits (a, b)
            whose labels form a config rule (M13_config_for_pychopper.txt:1
            "+:SP5,-SP27|-:SP27,-SP5"; the first rule naming the pair) is a candidate segment on
            that rule's strand, span [a.start, b.stop) with -p (keep primers), else
            [a.stop, b.start) (empty if they overlap).  The read's segments are the best path
            over the candidates: no two chosen candidates share a hit, and the chosen set has
            the greatest summed length (pychopper's usable length); on a tie the earlier
            candidate is taken (right-to-left DP, `segments`)
  classes   FASTQ mean quality (-10 log10 of the mean error probability) < -Q -> qcfail;
            0 segments -> unclassified (record unchanged); 1 -> pass (short if < -z);
            >= 2 -> every segment rescued (short if < -z); '-' segments reverse-complemented;
            segment records named "{start}:{stop}|{id} strand=+|-" + the original comment
  autotune  without -q: over the grid linspace(0.1, 0.6, -L) (-L = 30 samples), the cutoff
            whose segments have the greatest summed length (usable bases) over the first -Y
            QC-passing reads (ties -> the smaller cutoff)

[UNVERIFIED] choices (RULES below; the build implements the first reading of each, the drop-in
and the kernels follow it): every choice pychopper v2.7.0's source would settle has a switch with
one alternative reading, and tools/pychopper_cases.py holds one small case per switch whose
outputs differ between the two readings (tests/test_chop.py checks that they do).
tools/parity_vs_pychopper.sh runs those cases through a real pychopper v2.7.0 wherever one is
installed and diffs the outputs against the drop-in's: a DIFF names the switch to flip.
  tune_grid    autotune grid: linspace(0.1, 0.6, -L) | "0.0-0.5": linspace(0.0, 0.5, -L)
  tune_sample  autotune reads: the first -Y QC-passing reads | "stride": -Y reads spread evenly
               over all QC-passing reads (every ceil(n / Y)-th), as a sample of the whole input
  tune_score   autotune criterion: most usable bases (summed segment length) | "reads": most
               reads with exactly one segment (the round-1/2 stand-in)
  seg_score    best path over a read's candidate segments: greatest summed length | "count":
               most segments, then greatest summed length
  naming       segment records: "{start}:{stop}|{id} strand=+|-{comment}" | "nostrand":
               "{start}:{stop}|{id}{comment}" (the strand only implied by the orientation)
Version target: pychopper v2.7.0, the version the reference pins (/root/reference/README.md:6).
Neither its source nor its documentation is available offline in this image, so no reading
above is settled by a v2.7.0 text: all five stay open switches until the parity hook runs on a
real v2.7.0 (tools/parity_vs_pychopper.sh refuses any other version unless told otherwise).
The `-k LSK114` kit is not a switch: with -b, -c, -m, -Q and -p given (01_pychopper.sh:45-57)
the restatement reads it as unused, and the reference holds no LSK114 primer or parameter file
that an alternative reading could draw on, so no case can separate it (parity unpinned).

Only tests/ (and bench.py's cpu_baseline leg, through `batch_hit_counts`) use this module, as
the checker of libdmx's `dmx_chop_*` (HIP) path and of the `bin/pychopper` drop-in.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np

import oracle as _orc

AUTOTUNE_SAMPLES = 30

# [UNVERIFIED] readings (module docstring); tests flip one at a time and restore it
DEFAULT_RULES = {"tune_grid": "0.1-0.6", "tune_sample": "first", "tune_score": "bases",
                 "seg_score": "length", "naming": "strand"}
ALT_RULES = {"tune_grid": "0.0-0.5", "tune_sample": "stride", "tune_score": "reads",
             "seg_score": "count", "naming": "nostrand"}
RULES = dict(DEFAULT_RULES)


def autotune_cutoffs(samples: int = AUTOTUNE_SAMPLES):
    """The -q grid tried without -q: `samples` values evenly spaced over [0.1, 0.6]
    (RULES["tune_grid"] "0.0-0.5": over [0.0, 0.5])."""
    lo, hi = (0.1, 0.6) if RULES["tune_grid"] == "0.1-0.6" else (0.0, 0.5)
    return [float(x) for x in np.linspace(lo, hi, num=samples)]

_COMP = str.maketrans("ACGTUMRWSYKVHDBNacgtumrwsykvhdbn", "TGCAAKYWSRMBDHVNtgcaakywsrmbdhvn")
_IUPAC = {"A": "A", "C": "C", "G": "G", "T": "T", "U": "T", "R": "AG", "Y": "CT", "S": "CG",
          "W": "AT", "K": "GT", "M": "AC", "B": "CGT", "D": "AGT", "H": "ACT", "V": "ACG",
          "N": "ACGT"}
_ready = False


def revcomp(s: str) -> str:
    return s.translate(_COMP)[::-1]


def labels(primers):
    """[(name, seq)] -> [(label name, seq)]: NAME, -NAME per primer, in file order."""
    out = []
    for name, seq in primers:
        s = seq.upper().replace("U", "T")
        out += [(name, s), ("-" + name, revcomp(s))]
    return out


def parse_config(text: str, names):
    """"+:SP5,-SP27|-:SP27,-SP5" -> [(left label, right label, strand 0 '+' / 1 '-')]."""
    idx = {}
    for p, nm in enumerate(names):
        idx[nm] = 2 * p
        idx["-" + nm] = 2 * p + 1
    rules = []
    for part in text.strip().split("|"):
        strand, pair = part.split(":", 1)
        a, b = (x.strip() for x in pair.split(","))
        rules.append((idx[a], idx[b], 0 if strand.strip() == "+" else 1))
    return rules


def _lib():
    global _ready
    L = _orc.lib()
    if not _ready:
        L.orc_chop_hits.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_double,
                                    ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        L.orc_chop_batch.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_int),
                                     ctypes.c_int, ctypes.c_double, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_int, ctypes.c_void_p]
        _ready = True
    return L


def hits_c(pat: str, read: str, cutoff: float):
    """[(start, stop, dist)] of one label in one read, in stop order (oracle/chop_oracle.c)."""
    L = _lib()
    cap = 64
    while True:
        buf = np.zeros(3 * cap, dtype=np.int32)
        nh = L.orc_chop_hits(pat.encode(), len(pat), float(cutoff), read.encode(), len(read),
                             buf.ctypes.data, cap)
        if nh < 0:
            raise ValueError(f"bad primer {pat!r}")
        if nh <= cap:
            break
        cap = nh
    return [(int(buf[3 * i + 1]), int(buf[3 * i]), int(buf[3 * i + 2])) for i in range(nh)]


def _eq(p: str, r: str) -> bool:
    return r not in "ACGT" or r in _IUPAC[p]


def _global(pat: str, txt: str) -> int:
    prev = list(range(len(pat) + 1))
    for t, ch in enumerate(txt, 1):
        cur = [t]
        for i in range(1, len(pat) + 1):
            cur.append(min(prev[i - 1] + (0 if _eq(pat[i - 1], ch) else 1), cur[i - 1] + 1,
                           prev[i] + 1))
        prev = cur
    return prev[-1]


def hits_py(pat: str, read: str, cutoff: float):
    """Pure-Python full-matrix version of hits_c (tiny cases only)."""
    m, n = len(pat), len(read)
    k = int(cutoff * m)
    R = read.upper()
    col = list(range(m + 1))
    D = [m]
    for j in range(1, n + 1):
        cur = [0]
        for i in range(1, m + 1):
            cur.append(min(col[i - 1] + (0 if _eq(pat[i - 1], R[j - 1]) else 1), cur[i - 1] + 1,
                           col[i] + 1))
        col = cur
        D.append(col[m])
    best = min(D[1:], default=m + 1)
    if best > k:
        return []
    out = []
    for stop in range(1, n + 1):
        if D[stop] == best:
            start = min(s for s in range(max(0, stop - m - best), stop + 1)
                        if _global(pat, R[s:stop]) == best)
            out.append((start, stop, best))
    return out


def read_hits(labs, read: str, cutoff: float, impl=None):
    """All hits of one read: [(start, stop, label, dist)] sorted by (start, stop, label)."""
    impl = impl or hits_c
    out = []
    for li, (_, pat) in enumerate(labs):
        out += [(s, e, li, d) for s, e, d in impl(pat, read, cutoff)]
    out.sort()
    return out


def segments(hits, rules, keep: bool):
    """Best path over the candidate segments of one read's sorted hits:
    [(start, stop, strand, rule)], left to right."""
    table = {}
    for r, (a, b, st) in enumerate(rules):
        table.setdefault((a, b), (r, st))
    c = len(hits)
    cand = [None] * c
    for i in range(c - 1):
        h1, h2 = hits[i], hits[i + 1]
        rs = table.get((h1[2], h2[2]))
        if rs is not None:
            a = h1[0] if keep else h1[1]
            b = h2[1] if keep else h2[0]
            cand[i] = (a, max(a, b), rs[1], rs[0])
    # best[i]: the best (segment count, summed length) using hits i.. only, compared by
    # summed length (RULES["seg_score"] "length") or by count, then length ("count")
    by_count = RULES["seg_score"] == "count"
    best = [(0, 0)] * (c + 2)
    take = [False] * c

    def key(v):
        return v if by_count else (v[1], v[0])

    for i in range(c - 2, -1, -1):
        best[i] = best[i + 1]
        if cand[i] is not None:
            t = (best[i + 2][0] + 1, cand[i][1] - cand[i][0] + best[i + 2][1])
            if key(t) >= key(best[i + 1]):
                best[i], take[i] = t, True
    segs, i = [], 0
    while i + 1 < c:
        if take[i]:
            segs.append(cand[i])
            i += 2
        else:
            i += 1
    return segs


def usable_length(segs) -> int:
    return sum(b - a for a, b, _, _ in segs)


def mean_qual(qual: str) -> float:
    """-10 log10 of the mean Phred+33 error probability, summed in read order."""
    if not qual:
        return 0.0
    s = 0.0
    for c in qual:
        s += 10.0 ** (-(ord(c) - 33) / 10.0)
    return -10.0 * math.log10(s / len(qual))


def seg_name(head: str, a: int, b: int, strand: int) -> str:
    cut = len(head)
    for i, ch in enumerate(head):
        if ch in " \t":
            cut = i
            break
    if RULES["naming"] == "nostrand":
        return f"{a}:{b}|{head[:cut]}{head[cut:]}"
    return f"{a}:{b}|{head[:cut]} strand={'-' if strand else '+'}{head[cut:]}"


def chop_records(records, primers, config: str, cutoff: float, keep: bool = True,
                 min_qual: float = 7.0, min_len: int = 50, fasta: bool = False):
    """records [(header, seq, qual-or-None)] -> {pass, rescued, unclass, short, qcfail}:
    lists of (header, seq, qual) in input order."""
    labs = labels(primers)
    rules = parse_config(config, [p[0] for p in primers])
    out = {k: [] for k in ("pass", "rescued", "unclass", "short", "qcfail")}
    for head, seq, qual in records:
        if not fasta and mean_qual(qual) < min_qual:
            out["qcfail"].append((head, seq, qual))
            continue
        segs = segments(read_hits(labs, seq, cutoff), rules, keep)
        if not segs:
            out["unclass"].append((head, seq, qual))
            continue
        dest = "pass" if len(segs) == 1 else "rescued"
        for a, b, st, _ in segs:
            s = seq[a:b]
            q = qual[a:b] if qual is not None else None
            if st:
                s = revcomp(s)
                q = q[::-1] if q is not None else None
            out[dest if b - a >= min_len else "short"].append((seg_name(head, a, b, st), s, q))
    return out


def autotune(records, primers, config: str, keep: bool = True, min_qual: float = 7.0,
             sample: int = 10000, fasta: bool = False, samples: int = AUTOTUNE_SAMPLES) -> float:
    """-q when not given: the grid value with the most usable bases (summed segment length)
    over the first `sample` QC-passing reads; ties -> the smaller cutoff."""
    labs = labels(primers)
    rules = parse_config(config, [p[0] for p in primers])
    pool = [s for _, s, q in records if fasta or mean_qual(q) >= min_qual]
    if RULES["tune_sample"] == "stride" and len(pool) > sample:
        step = -(-len(pool) // sample)
        pool = pool[::step]
    pool = pool[:sample]
    best, best_n = None, -1
    for q in autotune_cutoffs(samples):
        if RULES["tune_score"] == "reads":
            c = sum(1 for s in pool if len(segments(read_hits(labs, s, q), rules, keep)) == 1)
        else:
            c = sum(usable_length(segments(read_hits(labs, s, q), rules, keep)) for s in pool)
        if c > best_n:
            best, best_n = q, c
    return best


def batch_hit_counts(primers, cutoff: float, blob, offsets, lengths, threads: int):
    """Per-read hit counts over all labels, on `threads` pthreads (the bench's CPU baseline)."""
    labs = labels(primers)
    arr = (ctypes.c_char_p * len(labs))(*[s.encode() for _, s in labs])
    pl = (ctypes.c_int * len(labs))(*[len(s) for _, s in labs])
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = np.ascontiguousarray(lengths, dtype=np.uint32)
    out = np.zeros(len(lens), dtype=np.int32)
    _lib().orc_chop_batch(arr, pl, len(labs), float(cutoff), blob.ctypes.data, offs.ctypes.data,
                          lens.ctypes.data, len(lens), int(threads), out.ctypes.data)
    return out
