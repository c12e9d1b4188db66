"""Drop-in `seqkit` for the residual-primer failsafe of scripts/04_cleaning_primers.sh:397-460.

The script runs (after `source activate seqkit`):

    seqkit subseq -r 1:100   trimmed.fasta >  ends          (:414)
    seqkit subseq -r -100:-1 trimmed.fasta >> ends          (:416)
    seqkit locate -d --pattern-file primers.fa ends > loc   (:422)
    seqkit grep -v -f ids trimmed.fasta > cleanest          (:436)

`locate` is the compute: it runs on the GPU (libdmx `dmx_locate`, a Shift-And kernel per
(record, pattern) over both strands).  `subseq -r` and `grep -f` are record plumbing done here.
Output formats follow seqkit v2 (not vendored; restated, parity unpinned): FASTA wrapped at 60
columns (`-w 0` disables wrapping), headers kept as read, `locate` prints the TSV header
`seqID patternName pattern strand start end matched` and one row per hit.

Any other subcommand or flag is handed to the next `seqkit` found on PATH after this one; if
there is none, it exits with status 2 and says so (never silently ignored).
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys

import numpy as np

from . import fastx, lib

SUPPORTED = ("subseq", "locate", "grep")


def _records(path):
    """[(header bytes, sequence bytes)] of a FASTA/FASTQ(.gz) file ('-' = stdin)."""
    out = []
    for b in fastx.read_batches(path):
        for i in range(len(b)):
            out.append((b.header(i), b.sequence(i)))
    return out


def _seq_id(header: bytes) -> bytes:
    return header.split(None, 1)[0] if header.strip() else b""


def _write_fasta(fh, header: bytes, seq: bytes, width: int):
    fh.write(b">" + header + b"\n")
    if width <= 0:
        fh.write(seq + b"\n")
        return
    for i in range(0, len(seq), width):
        fh.write(seq[i:i + width] + b"\n")


def _region(spec: str):
    try:
        a, b = spec.split(":")
        a, b = int(a), int(b)
    except ValueError:
        raise SystemExit(f"seqkit (dmx): bad region {spec!r}, expected START:END") from None
    if a == 0 or b == 0:
        raise SystemExit("seqkit (dmx): region positions are 1-based and non-zero")
    return a, b


def region_slice(n: int, a: int, b: int):
    """1-based inclusive region with negative positions counted from the end (-1 = last),
    clipped to the sequence: (start, stop) as a Python slice (may be empty)."""
    s = a - 1 if a > 0 else n + a
    e = b if b > 0 else n + b + 1
    s, e = min(max(s, 0), n), min(e, n)
    return s, max(s, e)


def _out(path):
    return sys.stdout.buffer if path in (None, "-") else open(path, "wb")


def cmd_subseq(args):
    a, b = _region(args.region)
    fh = _out(args.out_file)
    for path in args.files or ["-"]:
        for h, s in _records(path):
            lo, hi = region_slice(len(s), a, b)
            _write_fasta(fh, h, s[lo:hi], args.line_width)
    fh.flush()


def _read_patterns(args):
    pats = []
    for path in args.pattern_file or []:
        for h, s in _records(path):
            pats.append((_seq_id(h).decode(), s.decode("ascii")))
    for i, p in enumerate(args.pattern or []):
        pats.append((p, p))
    if not pats:
        raise SystemExit("seqkit (dmx): locate needs -p/--pattern or -f/--pattern-file")
    return pats


def cmd_locate(args):
    if args.max_mismatch:
        raise SystemExit("seqkit (dmx): locate -m > 0 is not supported (exact matching only)")
    pats = _read_patterns(args)
    if not args.degenerate:
        for name, p in pats:
            if set(p.upper()) - set("ACGTU"):
                raise SystemExit(f"seqkit (dmx): pattern {name} has degenerate bases; pass -d")
    recs = []
    for path in args.files or ["-"]:
        recs.extend(_records(path))
    lens = np.array([len(s) for _, s in recs], dtype=np.uint32)
    offs = np.zeros(len(recs), dtype=np.uint64)
    if len(recs) > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    blob = np.frombuffer(b"".join(s for _, s in recs), dtype=np.uint8)
    dev = int(os.environ.get("DMX_DEVICE", "0"))
    with lib.Context(dev) as ctx:
        hits = ctx.locate([p for _, p in pats], blob, offs, lens, ignore_case=args.ignore_case,
                          only_positive=args.only_positive_strand)
    fh = _out(args.out_file)
    fh.write(b"seqID\tpatternName\tpattern\tstrand\tstart\tend\tmatched\n")
    for h in hits:
        i = int(h["seq"])
        head, seq = recs[i]
        st, en = int(h["start"]), int(h["end"])
        m = seq[st - 1:en]
        if int(h["strand"]):
            m = fastx.revcomp(m)
        name, pseq = pats[int(h["pattern"])]
        fh.write(b"\t".join([_seq_id(head), name.encode(), pseq.encode(),
                             b"-" if int(h["strand"]) else b"+", str(st).encode(),
                             str(en).encode(), m]) + b"\n")
    fh.flush()


def cmd_grep(args):
    if not args.pattern_file and not args.pattern:
        raise SystemExit("seqkit (dmx): grep needs -p/--pattern or -f/--pattern-file")
    keys = set()
    for path in args.pattern_file or []:
        with open(path, "rb") as fh:
            for line in fh:
                line = line.rstrip(b"\r\n")
                if line:
                    keys.add(line)
    keys.update(p.encode() for p in args.pattern or [])
    fh = _out(args.out_file)
    for path in args.files or ["-"]:
        for h, s in _records(path):
            key = h if args.by_name else _seq_id(h)
            if (key in keys) != args.invert_match:
                _write_fasta(fh, h, s, args.line_width)
    fh.flush()


def _parser():
    ap = argparse.ArgumentParser(prog="seqkit", add_help=True)
    sub = ap.add_subparsers(dest="cmd")

    def common(p):
        p.add_argument("-o", "--out-file", default="-")
        p.add_argument("-w", "--line-width", type=int, default=60)
        p.add_argument("-j", "--threads", type=int, default=4)
        p.add_argument("files", nargs="*")

    p = sub.add_parser("subseq")
    p.add_argument("-r", "--region", required=True)
    common(p)
    p = sub.add_parser("locate")
    p.add_argument("-d", "--degenerate", action="store_true")
    p.add_argument("-f", "--pattern-file", action="append")
    p.add_argument("-p", "--pattern", action="append")
    p.add_argument("-i", "--ignore-case", action="store_true")
    p.add_argument("-P", "--only-positive-strand", action="store_true")
    p.add_argument("-m", "--max-mismatch", type=int, default=0)
    common(p)
    p = sub.add_parser("grep")
    p.add_argument("-f", "--pattern-file", action="append")
    p.add_argument("-p", "--pattern", action="append")
    p.add_argument("-v", "--invert-match", action="store_true")
    p.add_argument("-n", "--by-name", action="store_true")
    common(p)
    return ap


def _forward(argv):
    """Hand an unsupported command to the next `seqkit` on PATH (not this one)."""
    me = os.path.realpath(sys.argv[0]) if sys.argv and sys.argv[0] else ""
    for d in os.environ.get("PATH", "").split(os.pathsep):
        cand = os.path.join(d, "seqkit")
        if os.path.isfile(cand) and os.access(cand, os.X_OK) and os.path.realpath(cand) != me:
            return subprocess.call([cand] + argv)
    sys.stderr.write("seqkit (dmx): only `subseq -r`, `locate` and `grep -f/-p` are provided "
                     f"here and no other seqkit is on PATH: {' '.join(argv)}\n")
    return 2


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    # a region such as -100:-1 would read as an option to argparse: bind it to its flag
    argv = [f"--region={argv[i + 1]}" if a in ("-r", "--region") and i + 1 < len(argv) else a
            for i, a in enumerate(argv) if not (i > 0 and argv[i - 1] in ("-r", "--region"))]
    if not argv or argv[0] not in SUPPORTED:
        sys.exit(_forward(argv))
    ap = _parser()
    try:
        args, extra = ap.parse_known_args(argv)
    except SystemExit as e:
        sys.exit(2 if e.code else 0)
    if extra:
        sys.exit(_forward(argv))
    try:
        {"subseq": cmd_subseq, "locate": cmd_locate, "grep": cmd_grep}[args.cmd](args)
    except BrokenPipeError:
        pass
    except (ValueError, lib.DmxError) as e:
        sys.stderr.write(f"seqkit (dmx): {e}\n")
        sys.exit(1)


__all__ = ["main", "region_slice"]
