"""cutadapt-style --json report and stdout report for one drop-in invocation.

Follows the layout of cutadapt 4.x's `--json` report (schema 0.3) and its human-readable
report (upstream report.py, not vendored — restated from its documentation and output format,
UNVERIFIED where marked): read counts, base-pair counts and, per adapter end, total matches,
matches on the reverse complement, the lengths at which one more error is allowed
(`error_lengths`), the bases preceding removed 3' adapters (`adjacent_bases`, with the dominant
one flagged) and the histogram of removed lengths by number of errors with the count expected
by chance.  The reference writes one report per cutadapt call (scripts/02_cutadapt_loop.sh:72,
102) and leaves the human report in the job log (:6).
"""
from __future__ import annotations

import json
import platform
import sys
from collections import Counter, defaultdict

import numpy as np

from . import __version__


ADJ_KEYS = ("A", "C", "G", "T", "")   # codes 0-3, then "no preceding base or not ACGT"


def effective_length(seq: str) -> int:
    """cutadapt's effective adapter length: N wildcards do not count (wildcard adapters only)."""
    wild = any(c not in "ACGT" for c in seq)
    return len(seq) - seq.count("N") if wild else len(seq)


def error_rate_of(seq: str, max_errors: float) -> float:
    """-e as a rate (< 1) or an absolute count (>= 1, converted per adapter)."""
    return max_errors if max_errors < 1.0 else max_errors / effective_length(seq)


def error_lengths(seq: str, max_errors: float) -> list:
    """Aligned lengths at which one more error becomes allowed: int(errors / rate) for
    errors = 1 .. int(rate * effective length) (the boundaries of the text report's "No. of
    allowed errors" ranges; UNVERIFIED against cutadapt's JSON)."""
    rate = error_rate_of(seq, max_errors)
    if rate <= 0.0:
        return []
    return [int(e / rate) for e in range(1, int(rate * effective_length(seq)) + 1)]


def allowed_errors_text(seq: str, max_errors: float) -> str:
    """The "No. of allowed errors:" line of cutadapt's text report (partial matches allowed)."""
    length = effective_length(seq)
    rate = error_rate_of(seq, max_errors)
    prev, parts = 1, []
    for e in range(1, int(rate * length) + 1):
        r = int(e / rate)
        parts.append(f"{prev}-{r - 1} bp: {e - 1}")
        prev = r
    last = f"{length} bp: {int(rate * length)}" if prev == length else \
        f"{prev}-{length} bp: {int(rate * length)}"
    return "; ".join(parts + [last])


def dominant_base(adj: dict):
    """A base preceding more than 80 % of the removed 3' adapters (cutadapt warns about it;
    threshold UNVERIFIED), else None."""
    total = sum(adj.values())
    for b in "ACGT":
        if total and adj.get(b, 0) > 0.8 * total:
            return b
    return None


def view_codes(packed, reads, strand, pos):
    """2-bit code (0-3) of view position `pos` of reads `reads` on `strand` (0 as given, 1 the
    reverse complement), 4 where that byte is not ACGT and where pos < 0 (no preceding base):
    read straight from the packed batch (include/dmx.h dmx_pack layout)."""
    reads = np.asarray(reads, np.int64)
    pos = np.asarray(pos, np.int64)
    strand = np.asarray(strand, np.int64)
    if not len(reads):
        return np.zeros(0, np.int64)
    offs = packed.offsets[reads].astype(np.int64)
    n = packed.lengths[reads].astype(np.int64)
    valid = (pos >= 0) & (pos < n)
    g = np.where(valid, np.where(strand == 0, offs + pos, offs + n - 1 - pos), offs)
    code = (packed.seq2b[g >> 4].astype(np.int64) >> (2 * (g & 15))) & 3
    code = np.where(strand == 1, 3 - code, code)
    nb = (packed.nmask[g >> 5].astype(np.int64) >> (g & 31)) & 1
    return np.where(valid & (nb == 0), code, 4)


class Stats:
    def __init__(self, adapters):
        self.adapters = adapters
        self.n_in = self.bp_in = 0
        self.n_out = self.bp_out = 0
        self.n_rc = 0
        self.n_with_adapter = 0
        self.n_discard_untrimmed = 0
        self.rc_mode = False      # --rc given: on_reverse_complement is reported (else null)
        self.matches = defaultdict(int)
        self.on_rc = defaultdict(int)
        # adapter index -> part ("front"/"back") -> Counter{(removed length, errors): count}
        self._hist = defaultdict(lambda: defaultdict(Counter))
        # adapter index -> counts of the base preceding a removed 3' adapter (ADJ_KEYS order)
        self._adjacent = defaultdict(lambda: np.zeros(5, np.int64))
        # per-batch additions not folded into the dicts yet: (part, keys, counts) and a dense
        # [adapter][5] count array (folding once per report instead of once per batch keeps
        # the fused loop's per-batch statistics in numpy)
        self._pend = []
        self._pend_n = 0
        self._adj_pend = None
        self.min_overlap = 3

    @property
    def hist(self):
        self._fold()
        return self._hist

    @property
    def adjacent(self):
        self._fold()
        return self._adjacent

    def _fold(self):
        if self._pend:
            for part in sorted({p for p, _, _ in self._pend}):
                ks = [k for p, k, _ in self._pend if p == part]
                cs = [c for p, _, c in self._pend if p == part]
                u, inv = np.unique(np.concatenate(ks), return_inverse=True)
                tot = np.zeros(len(u), np.int64)
                np.add.at(tot, inv, np.concatenate(cs).astype(np.int64))
                for k, n in zip(u.tolist(), tot.tolist()):
                    self._hist[k >> 40][part][((k >> 8) & ((1 << 32) - 1), k & 255)] += n
            self._pend = []
            self._pend_n = 0
        if self._adj_pend is not None:
            for a in np.nonzero(self._adj_pend.sum(axis=1))[0].tolist():
                self._adjacent[a] += self._adj_pend[a]
            self._adj_pend = None

    def add_match(self, a: int, rc: bool, part: str, removed: int, errors: int):
        self.add_matches(np.array([a]), part, np.array([removed]), np.array([errors]))

    def add_matches(self, a, part: str, removed, errors):
        """Vectorised add_match for arrays of adapter index / removed length / errors."""
        a = np.asarray(a, np.int64)
        if not len(a):
            return
        key = (a << 40) | (np.asarray(removed, np.int64) << 8) | np.asarray(errors, np.int64)
        u, c = np.unique(key, return_counts=True)
        self.add_match_counts(part, u, c)

    def add_match_counts(self, part: str, keys, counts):
        """Histogram entries as keys adapter << 40 | removed length << 8 | errors with their
        counts (folded into `hist` when it is read)."""
        self._pend.append((part, np.asarray(keys, np.int64), np.asarray(counts, np.int64)))
        self._pend_n += len(keys)
        if self._pend_n > (1 << 22):
            self._fold()

    def add_adjacent(self, a, codes):
        """Bases (view_codes) preceding removed 3' adapters of adapters `a`."""
        a = np.asarray(a, np.int64)
        if not len(a):
            return
        key = a * 5 + np.asarray(codes, np.int64)
        self.add_adjacent_counts(np.bincount(key, minlength=5 * len(self.adapters))
                                 .reshape(-1, 5))

    def add_adjacent_counts(self, counts):
        """A dense [adapter][5] array of preceding-base counts (ADJ_KEYS order)."""
        counts = np.asarray(counts, np.int64)
        if self._adj_pend is None:
            self._adj_pend = np.zeros((max(len(self.adapters), len(counts)), 5), np.int64)
        if len(counts) > len(self._adj_pend):
            grown = np.zeros((len(counts), 5), np.int64)
            grown[:len(self._adj_pend)] = self._adj_pend
            self._adj_pend = grown
        self._adj_pend[:len(counts)] += counts

    def add_counts(self, bins, rc, n_adapters: int):
        """Per-adapter totals from arrays of matched adapter index and RC flag."""
        bins = np.asarray(bins, np.int64)
        self.add_count_vectors(np.bincount(bins, minlength=n_adapters),
                               np.bincount(bins[np.asarray(rc, bool)], minlength=n_adapters))

    def add_count_vectors(self, m, r):
        """Per-adapter match and reverse-complement totals as count vectors."""
        for a in np.nonzero(m)[0].tolist():
            self.matches[a] += int(m[a])
        for a in np.nonzero(r)[0].tolist():
            self.on_rc[a] += int(r[a])

    def check_totals(self, totals):
        """Per-adapter match totals counted on the GPU(s) (dmx_counts, all-reduced over devices)
        must equal those derived from the per-read results."""
        got = [int(x) for x in totals]
        want = [self.matches[a] for a in range(len(self.adapters))]
        if got != want:
            raise RuntimeError(f"device bin counts {got} disagree with per-read results {want}")

    def to_json(self, argv, cores, in_path, error_rate):
        adapters = []
        for a, ad in enumerate(self.adapters):
            linked = hasattr(ad, "front")
            ends = {}
            for part in ("front", "back"):
                if linked:
                    seq = ad.front if part == "front" else ad.back
                elif ad.where != part:
                    ends[part] = None
                    continue
                else:
                    seq = ad.seq
                h = defaultdict(dict)
                for (L, e), cnt in self.hist[a][part].items():
                    h[L][e] = cnt
                adj = None
                if part == "back" and not linked:   # 3' adapters: the base before the match
                    v = self.adjacent[a]
                    adj = {k: int(v[i]) for i, k in enumerate(ADJ_KEYS)}
                ends[part] = {
                    "type": "regular", "sequence": seq, "error_rate": error_rate, "indels": True,
                    "error_lengths": error_lengths(seq, error_rate),
                    "matches": sum(sum(e.values()) for e in h.values()),
                    "adjacent_bases": adj,
                    "dominant_adjacent_base": dominant_base(adj) if adj else None,
                    "trimmed_lengths": [
                        {"len": L, "expect": round(self.n_in * 0.25 ** min(L, len(seq)), 1),
                         "counts": [h[L].get(e, 0) for e in range(max(h[L]) + 1)]}
                        for L in sorted(h)],
                }
            adapters.append({
                "name": ad.name, "total_matches": self.matches[a],
                "on_reverse_complement": self.on_rc[a] if (self.rc_mode or self.on_rc) else None,
                "linked": linked,
                "five_prime_end": ends.get("front"), "three_prime_end": ends.get("back"),
            })
        return {
            "tag": "Cutadapt report", "schema_version": [0, 3],
            "cutadapt_version": f"dmx {__version__} (cutadapt 4.9 compatible)",
            "python_version": platform.python_version(),
            "command_line_arguments": list(argv), "cores": cores,
            "input": {"path1": in_path, "path2": None, "paired": False, "interleaved": None},
            "read_counts": {
                "input": self.n_in,
                "filtered": {"too_short": None, "too_long": None, "too_many_n": None,
                             "too_many_expected_errors": None, "casava_filtered": None,
                             "discard_trimmed": None,
                             "discard_untrimmed": self.n_discard_untrimmed or None},
                "output": self.n_out, "reverse_complemented": self.n_rc,
                "read1_with_adapter": self.n_with_adapter, "read2_with_adapter": None},
            "basepair_counts": {"input": self.bp_in, "input_read1": self.bp_in,
                                "input_read2": None, "quality_trimmed": None,
                                "quality_trimmed_read1": None, "quality_trimmed_read2": None,
                                "poly_a_trimmed": None, "poly_a_trimmed_read1": None,
                                "poly_a_trimmed_read2": None, "output": self.bp_out,
                                "output_read1": self.bp_out, "output_read2": None},
            "adapters_read1": adapters, "adapters_read2": None,
            "poly_a_trimmed_read1": None, "poly_a_trimmed_read2": None,
        }

    def write_json(self, path, **kw):
        with open(path, "w") as fh:
            json.dump(self.to_json(**kw), fh, indent=2)
            fh.write("\n")

    def summary(self, out=sys.stdout, error_rate: float = 0.1):
        """cutadapt's human-readable report: the summary block, then per adapter its sequence,
        type, length and match counts, the allowed errors by length, the bases preceding removed
        3' adapters and the table of removed lengths (count, expected count, maximum and
        observed errors).  Layout restated from cutadapt 4.x output (UNVERIFIED in detail)."""
        def pct(x, tot):
            return f"({100.0 * x / tot:.1f}%)" if tot else "(0.0%)"
        p = lambda *a: print(*a, file=out)   # noqa: E731
        p("=== Summary ===\n")
        p(f"Total reads processed:           {self.n_in:>12,}")
        p(f"Reads with adapters:             {self.n_with_adapter:>12,} "
          f"{pct(self.n_with_adapter, self.n_in)}")
        if self.rc_mode:
            p(f"Reverse-complemented:            {self.n_rc:>12,} {pct(self.n_rc, self.n_in)}")
        if self.n_discard_untrimmed:
            p(f"Reads discarded as untrimmed:    {self.n_discard_untrimmed:>12,} "
              f"{pct(self.n_discard_untrimmed, self.n_in)}")
        p(f"Reads written (passing filters): {self.n_out:>12,} {pct(self.n_out, self.n_in)}")
        p("")
        p(f"Total basepairs processed: {self.bp_in:>14,} bp")
        p(f"Total written (filtered):  {self.bp_out:>14,} bp {pct(self.bp_out, self.bp_in)}")
        for a, ad in enumerate(self.adapters):
            linked = hasattr(ad, "front")
            p(f"\n=== Adapter {ad.name} ===\n")
            if linked:
                parts = [("front", ad.front, "5'"), ("back", ad.back, "3'")]
                p(f"Sequence: {ad.front}...{ad.back}; Type: linked; "
                  f"Length: {len(ad.front)}+{len(ad.back)}; Trimmed: {self.matches[a]} times")
            else:
                parts = [(ad.where, ad.seq, "5'" if ad.where == "front" else "3'")]
                rc = (f"; Reverse-complemented: {self.on_rc[a]} times" if self.rc_mode else "")
                p(f"Sequence: {ad.seq}; Type: regular {parts[0][2]}; Length: {len(ad.seq)}; "
                  f"Trimmed: {self.matches[a]} times{rc}")
            for part, seq, kind in parts:
                if linked:
                    p(f"\n{'First' if part == 'front' else 'Second'} adapter ({kind}):")
                p(f"\nMinimum overlap: {self.min_overlap}")
                p("No. of allowed errors:")
                p(allowed_errors_text(seq, error_rate))
                if part == "back" and not linked:
                    v = self.adjacent[a]
                    tot = int(v.sum())
                    p("\nBases preceding removed adapters:")
                    for i, b in enumerate("ACGT"):
                        p(f"  {b}: {100.0 * v[i] / tot if tot else 0.0:.1f}%")
                    p(f"  none/other: {100.0 * v[4] / tot if tot else 0.0:.1f}%")
                    dom = dominant_base({k: int(v[i]) for i, k in enumerate(ADJ_KEYS)})
                    if dom:
                        p(f"WARNING:\n    The adapter is preceded by '{dom}' extremely often.")
                p("\nOverview of removed sequences")
                p("length\tcount\texpect\tmax.err\terror counts")
                h = defaultdict(dict)
                for (L, e), cnt in self.hist[a][part].items():
                    h[L][e] = cnt
                rate = error_rate_of(seq, error_rate)
                for L in sorted(h):
                    cnts = [h[L].get(e, 0) for e in range(max(h[L]) + 1)]
                    p(f"{L}\t{sum(cnts)}\t{self.n_in * 0.25 ** min(L, len(seq)):.1f}\t"
                      f"{int(min(L, len(seq)) * rate)}\t{' '.join(str(c) for c in cnts)}")
