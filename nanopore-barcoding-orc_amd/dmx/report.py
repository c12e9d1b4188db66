"""cutadapt-style --json report and stdout summary for one drop-in invocation.

Follows the layout of cutadapt 4.x's `--json` report (schema 0.3; upstream report.py, not
vendored — field set restated from its documentation, UNVERIFIED where marked): read counts,
base-pair counts and, per adapter, total matches, matches on the reverse complement, and the
histogram of removed lengths by number of errors.  The reference writes one report per
cutadapt call (scripts/02_cutadapt_loop.sh:72,102).
"""
from __future__ import annotations

import json
import platform
import sys
from collections import Counter, defaultdict

import numpy as np

from . import __version__


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
        self.hist = defaultdict(lambda: defaultdict(Counter))

    def add_match(self, a: int, rc: bool, part: str, removed: int, errors: int):
        self.hist[a][part][(int(removed), int(errors))] += 1

    def add_matches(self, a, part: str, removed, errors):
        """Vectorised add_match for arrays of adapter index / removed length / errors."""
        a = np.asarray(a, np.int64)
        if not len(a):
            return
        key = (a << 40) | (np.asarray(removed, np.int64) << 8) | np.asarray(errors, np.int64)
        u, c = np.unique(key, return_counts=True)
        for k, n in zip(u.tolist(), c.tolist()):
            self.hist[k >> 40][part][((k >> 8) & ((1 << 32) - 1), k & 255)] += n

    def add_counts(self, bins, rc, n_adapters: int):
        """Per-adapter totals from arrays of matched adapter index and RC flag."""
        bins = np.asarray(bins, np.int64)
        m = np.bincount(bins, minlength=n_adapters)
        r = np.bincount(bins[np.asarray(rc, bool)], minlength=n_adapters)
        for a in range(n_adapters):
            if m[a]:
                self.matches[a] += int(m[a])
            if r[a]:
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
                ends[part] = {
                    "type": "regular", "sequence": seq, "error_rate": error_rate, "indels": True,
                    "error_lengths": None,   # UNVERIFIED layout; not produced
                    "matches": sum(sum(e.values()) for e in h.values()),
                    "adjacent_bases": None, "dominant_adjacent_base": None,
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

    def summary(self, out=sys.stdout):
        pct = (100.0 * self.n_with_adapter / self.n_in) if self.n_in else 0.0
        print("=== Summary ===\n", file=out)
        print(f"Total reads processed:           {self.n_in:>12,}", file=out)
        print(f"Reads with adapters:             {self.n_with_adapter:>12,} ({pct:.1f}%)",
              file=out)
        if self.n_rc:
            print(f"Reverse-complemented:            {self.n_rc:>12,}", file=out)
        print(f"Reads written (passing filters): {self.n_out:>12,}", file=out)
        print(f"Total basepairs processed: {self.bp_in:>14,} bp", file=out)
        print(f"Total written (filtered):  {self.bp_out:>14,} bp", file=out)
        for a, ad in enumerate(self.adapters):
            print(f"\n=== Adapter {ad.name} ===\n\nTrimmed: {self.matches[a]} times", file=out)
