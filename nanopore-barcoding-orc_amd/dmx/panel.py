"""Adapter panels: FASTA parsing and cutadapt-style adapter specifications.

Restates cutadapt 4.9's parser behaviour for the forms the reference uses
(scripts/02_cutadapt_loop.sh:69 `-g file:SP5.fa`, :99 `-a file:SP27rc.fa`;
scripts/04_cleaning_primers.sh:377 `-g FWD...REV`, :476-498 `-g SEQ` / `-a SEQ`):
  * `file:PATH`: one adapter per FASTA record; name = first word of the header line;
  * `NAME=SEQ` or `SEQ`: a literal adapter, auto-named "1", "2", ... in command-line order;
  * `A...B`: a linked adapter (front A, back B);
  * sequences uppercased with U -> T (upstream parser.py; UNVERIFIED).
The panels in the reference have no trailing newline (M13_amplicon_indices_forward.fa:24) and
blank lines (RNA_primers.fa:5); both are tolerated.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass, field

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
SP5_FASTA = os.path.join(DATA_DIR, "M13_amplicon_indices_forward.fa")
SP27RC_FASTA = os.path.join(DATA_DIR, "M13_amplicon_indices_reverse_rc.fa")
COI_FASTA = os.path.join(DATA_DIR, "COI_primers.fa")
RNA_FASTA = os.path.join(DATA_DIR, "RNA_primers.fa")

IUPAC = set("ACGTURYSWKMBDHVN")


def normalize(seq: str) -> str:
    s = seq.strip().upper().replace("U", "T")
    bad = set(s) - IUPAC
    if bad:
        raise ValueError(f"adapter {seq!r} contains non-IUPAC characters {sorted(bad)}")
    if not s:
        raise ValueError("empty adapter sequence")
    return s


def read_fasta(path: str) -> list[tuple[str, str]]:
    """Parse a FASTA file into (header, sequence) records (whitespace inside sequences dropped)."""
    recs: list[tuple[str, str]] = []
    header, parts = None, []
    with open(path, "r") as fh:
        for line in fh:
            line = line.rstrip("\r\n")
            if not line.strip():
                continue
            if line.startswith(">"):
                if header is not None:
                    recs.append((header, "".join(parts)))
                header, parts = line[1:], []
            else:
                if header is None:
                    raise ValueError(f"{path}: sequence before the first '>' header")
                parts.append("".join(line.split()))
    if header is not None:
        recs.append((header, "".join(parts)))
    return recs


@dataclass
class Adapter:
    name: str
    seq: str
    where: str            # "front" (-g) or "back" (-a)


@dataclass
class LinkedAdapter:
    name: str
    front: str
    back: str


@dataclass
class AdapterSet:
    adapters: list = field(default_factory=list)   # Adapter or LinkedAdapter, command-line order
    _counter: int = 0

    def _auto_name(self) -> str:
        self._counter += 1
        return str(self._counter)

    def add_spec(self, spec: str, where: str):
        """Add one -g/-a argument."""
        if spec.startswith("file:"):
            for header, seq in read_fasta(spec[5:]):
                name = header.split()[0] if header.split() else self._auto_name()
                self._add(name, seq, where)
            return
        name = None
        if "=" in spec:
            name, spec = spec.split("=", 1)
            name = name.strip()
        if "..." in spec:
            a, b = spec.split("...", 1)
            if where != "front":
                # -a A...B is also linked in cutadapt (front optional by default); not used by
                # the reference scripts.
                raise NotImplementedError("linked adapters are supported with -g only")
            self.adapters.append(LinkedAdapter(name or self._auto_name(), normalize(a),
                                               normalize(b)))
            return
        self._add(name or self._auto_name(), spec, where)

    def _add(self, name: str, seq: str, where: str):
        s = seq.strip()
        if s.startswith("^") or s.endswith("$") or s.endswith("X") or s.startswith("X"):
            raise NotImplementedError("anchored / non-internal adapters are not on the hot path")
        self.adapters.append(Adapter(name, normalize(s), where))

    @property
    def linked(self) -> bool:
        return any(isinstance(a, LinkedAdapter) for a in self.adapters)


def load_panel(path: str) -> tuple[list[str], list[str]]:
    """(names, sequences) of a FASTA panel."""
    recs = read_fasta(path)
    return [h.split()[0] for h, _ in recs], [normalize(s) for _, s in recs]


_PAIR_ID = re.compile(r"_([A-Z])(?=\s|$|_)")


def primer_pairs(path: str) -> list[tuple[str, str, str]]:
    """Linked primer pairs [(pair_id, forward, reverse)] from a round-1 primer FASTA.

    Restates the header convention of scripts/04_cleaning_primers.sh:184-270: a header holding
    "Forward" / "Reverse" assigns its sequence to every pair id `_X` it carries (X one capital
    letter followed by whitespace, `_` or the end); pair order = first appearance; a later
    record for the same (id, orientation) replaces the earlier one; incomplete pairs are skipped
    (:380-385).  The sequences are used as written (the script does not reverse-complement)."""
    fwd: dict[str, str] = {}
    rev: dict[str, str] = {}
    order: list[str] = []
    for head, seq in read_fasta(path):
        seq = "".join(seq.split())
        if not seq:
            continue
        ids = _PAIR_ID.findall(">" + head)
        if "Forward" in head:
            dst = fwd
        elif "Reverse" in head:
            dst = rev
        else:
            continue
        for pid in ids:
            dst[pid] = seq
            if pid not in order:
                order.append(pid)
    return [(p, fwd[p], rev[p]) for p in order if p in fwd and p in rev]
