"""ORACLE — TEST INFRASTRUCTURE ONLY.  CPU restatement of `seqkit locate -d` (seqkit v2.x; not
vendored in /root/reference, not installed here), the residual-primer check of
scripts/04_cleaning_primers.sh:422 (`seqkit locate -d --pattern-file "$temp_primers"
"$temp_ends"`).  PARITY UNPINNED: restated from seqkit's documented behaviour, no seqkit
output exists to pin it to.

seqkit's published algorithm for -d: each pattern is turned into a regular expression in which
every IUPAC code becomes a character class of the bases it stands for (T and U together); the
regexp is searched on the sequence, and after each match the search restarts one position after
the match start (greedy mode, so overlapping matches are all reported).  The negative strand
(default on) is searched by running the same regexp on the reverse complement of the sequence;
hits are reported in positive-strand 1-based coordinates (start = len - e + 1, end = len - s
for a match [s, e) on the reverse complement) with the matched text as read on the reverse
complement.  Case-sensitive unless -i.

Only tests/ import this module, as the checker of libdmx's `dmx_locate` (HIP) path.
"""
from __future__ import annotations

import re

_CLASS = {"A": "A", "C": "C", "G": "G", "T": "TU", "U": "TU", "R": "AG", "Y": "CTU", "S": "CG",
          "W": "ATU", "K": "GTU", "M": "AC", "B": "CGTU", "D": "AGTU", "H": "ACTU", "V": "ACG",
          "N": "ACGTU"}
_COMP = str.maketrans("ACGTUMRWSYKVHDBNacgtumrwsykvhdbn", "TGCAAKYWSRMBDHVNtgcaakywsrmbdhvn")


def revcomp(s: str) -> str:
    return s.translate(_COMP)[::-1]


def pattern_regex(pattern: str, ignore_case: bool = False) -> re.Pattern:
    parts = []
    for ch in pattern:
        up = ch.upper()
        if up not in _CLASS:
            raise ValueError(f"non-IUPAC character {ch!r} in pattern {pattern!r}")
        cls = _CLASS[up] if ch.isupper() else _CLASS[up].lower()
        parts.append("[" + cls + "]")
    return re.compile("".join(parts), re.IGNORECASE if ignore_case else 0)


def _greedy(rx: re.Pattern, s: str):
    i = 0
    while True:
        m = rx.search(s, i)
        if m is None:
            return
        yield m.start(), m.end()
        i = m.start() + 1


def locate(records, patterns, ignore_case=False, only_positive=False):
    """records: [(seq_id, seq)], patterns: [(name, seq)] -> rows
    (seq_id, pattern_name, pattern, strand, start, end, matched) in seqkit's order."""
    rxs = [pattern_regex(p, ignore_case) for _, p in patterns]
    rows = []
    for sid, seq in records:
        rc = None
        n = len(seq)
        for (pname, pseq), rx in zip(patterns, rxs):
            for s, e in _greedy(rx, seq):
                rows.append((sid, pname, pseq, "+", s + 1, e, seq[s:e]))
            if only_positive:
                continue
            if rc is None:
                rc = revcomp(seq)
            for s, e in _greedy(rx, rc):
                rows.append((sid, pname, pseq, "-", n - e + 1, n - s, rc[s:e]))
    return rows
