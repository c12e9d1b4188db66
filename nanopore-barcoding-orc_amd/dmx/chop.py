"""`pychopper`-compatible read reorientation (scripts/01_pychopper.sh:45-57) on the GPU.

Drop-in for the reference's one pychopper call:
  pychopper -b M13_seqs_for_pychopper.fa -c M13_config_for_pychopper.txt -k LSK114 -Q 10
            -w RESCUED.fastq -u UNCLASS.fastq -l SHORT.fastq -S STATS.out -p -t 24 -m edlib
            IN.fastq.gz > PASS.fastq
pychopper v2.7.0 (edlib backend) is not vendored in /root/reference and not installed here: the
semantics are the build's restatement, checked against oracle/chopper.py, parity
unpinned.  Primer hits and segments come from libdmx (`dmx_chop_*`, HIP; no CPU fallback).
Per QC-passing read:
  0 segments            -> unclassified (-u), the record unchanged
  1 segment             -> PASS (stdout, or the second positional) if its length >= -z, else -l
  >= 2 segments (fused) -> every segment to the rescued output (-w) if >= -z, else -l
Segment records are oriented (strand '-' reverse-complemented, qualities reversed) and named
"{start}:{stop}|{id} strand=+|-" followed by the original comment ([start, stop) on the read as
given).  QC: a FASTQ read whose mean quality (-10 log10 of the mean error probability, Phred+33)
is below -Q goes to -K if given, else is dropped.  Cutoff -q: maximum edit distance as a
fraction of the primer length (k = int(q * m)); without -q it is tuned on the first -Y
QC-passing reads of the first batch over -L values evenly spaced on [0.1, 0.6] (the value whose
segments have the most usable bases, i.e. the greatest summed segment length; ties -> the
smaller).  A read's segments are the best path over its candidate segments (consecutive primer
hits forming a config rule; no shared hit, greatest summed length).  -k is accepted and unused
(-b and -c define primers and layout); only -m edlib is implemented.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

from . import __version__, lib, nio, panel

PRIMERS_FASTA = os.path.join(panel.DATA_DIR, "M13_seqs_for_pychopper.fa")
CONFIG_FILE = os.path.join(panel.DATA_DIR, "M13_config_for_pychopper.txt")
AUTOTUNE_SAMPLES = 30
PASS, RESCUED, UNCLASS, SHORT, QCFAIL = range(5)


def load_primers(path: str):
    """-b FASTA -> [(name, seq)]: name = first word of the header, sequence upper-cased, U -> T
    (adapters_primers/M13_seqs_for_pychopper.fa: SP5 and SP27 with N for the variable index)."""
    out = []
    for head, seq in panel.read_fasta(path):
        words = head.split()
        out.append((words[0] if words else head, panel.normalize(seq)))
    if not out:
        raise ValueError(f"{path}: no primers")
    return out


def parse_config(text: str, names):
    """pychopper layout ("+:SP5,-SP27|-:SP27,-SP5", M13_config_for_pychopper.txt:1) -> rules
    (left label, right label, strand 0 '+' / 1 '-') over labels NAME = 2p, -NAME = 2p + 1."""
    idx = {}
    for p, nm in enumerate(names):
        idx[nm] = 2 * p
        idx["-" + nm] = 2 * p + 1
    rules = []
    for part in text.strip().split("|"):
        part = part.strip()
        if not part:
            continue
        try:
            strand, pair = part.split(":", 1)
            a, b = (x.strip() for x in pair.split(","))
            rules.append((idx[a], idx[b], {"+": 0, "-": 1}[strand.strip()]))
        except (ValueError, KeyError) as e:
            raise ValueError(f"bad pychopper config rule {part!r}") from e
    return rules


def autotune_cutoffs(samples: int = AUTOTUNE_SAMPLES):
    """The -q grid tried without -q (-L samples evenly spaced over [0.1, 0.6])."""
    return [float(x) for x in np.linspace(0.1, 0.6, num=samples)]


def plan_rows(nseg, segs, lens, qc_ok, min_len: int, outs):
    """Output rows of one batch (read, out, start, stop, rc, name_mode), in read order.
    outs[kind] = output index or -1 (not written) for PASS, RESCUED, UNCLASS, SHORT, QCFAIL."""
    ns = nseg.astype(np.int64)
    sread = segs["read"].astype(np.int64)
    sstart = segs["start"].astype(np.int64)
    sstop = segs["stop"].astype(np.int64)
    single = ns[sread] == 1
    s_out = np.where(sstop - sstart >= min_len, np.where(single, outs[PASS], outs[RESCUED]),
                     outs[SHORT])
    s_out = np.where(qc_ok[sread], s_out, -1)
    w_read = np.nonzero(~qc_ok | (ns == 0))[0]
    w_out = np.where(qc_ok[w_read], outs[UNCLASS], outs[QCFAIL])
    read = np.concatenate([sread, w_read])
    out = np.concatenate([s_out, w_out])
    start = np.concatenate([sstart, np.zeros(len(w_read), np.int64)])
    stop = np.concatenate([sstop, lens[w_read].astype(np.int64)])
    rc = np.concatenate([segs["strand"].astype(np.uint8), np.zeros(len(w_read), np.uint8)])
    mode = np.concatenate([np.ones(len(sread), np.uint8), np.zeros(len(w_read), np.uint8)])
    order = np.argsort(read, kind="stable")
    order = order[out[order] >= 0]
    return (read[order].astype(np.uint32), out[order].astype(np.int32),
            start[order].astype(np.int32), stop[order].astype(np.int32), rc[order], mode[order])


class ChopStats:
    """The -S statistics file (tab-separated Category / Name / Value)."""

    def __init__(self):
        self.n_in = self.n_qcfail = self.n_unclass = self.n_found = self.n_rescue = 0
        self.strand = [0, 0]
        self.n_short = 0
        self.cutoff = None

    def add(self, nseg, segs, qc_ok, min_len: int):
        ns = nseg.astype(np.int64)
        self.n_in += len(ns)
        self.n_qcfail += int((~qc_ok).sum())
        self.n_unclass += int((qc_ok & (ns == 0)).sum())
        self.n_found += int((qc_ok & (ns == 1)).sum())
        self.n_rescue += int((qc_ok & (ns >= 2)).sum())
        if len(segs):
            ok = qc_ok[segs["read"].astype(np.int64)]
            long_ = (segs["stop"].astype(np.int64) - segs["start"]) >= min_len
            for st in (0, 1):
                self.strand[st] += int((ok & long_ & (segs["strand"] == st)).sum())
            self.n_short += int((ok & ~long_).sum())

    def rows(self):
        return [("Classification", "Primers_found", self.n_found),
                ("Classification", "Rescue", self.n_rescue),
                ("Classification", "Unusable", self.n_unclass),
                ("Classification", "QC_fail", self.n_qcfail),
                ("Strand", "+", self.strand[0]), ("Strand", "-", self.strand[1]),
                ("Segments", "Short", self.n_short), ("Reads", "Input", self.n_in),
                ("Parameters", "cutoff", "NA" if self.cutoff is None else repr(self.cutoff))]

    def write(self, path: str):
        with open(path, "w") as fh:
            fh.write("Category\tName\tValue\n")
            for a, b, v in self.rows():
                fh.write(f"{a}\t{b}\t{v}\n")


class Chopper:
    """A device context set up for one primer panel and layout (include/dmx.h dmx_chop_*)."""

    def __init__(self, ctx, primers, rules, keep: bool):
        self.ctx = ctx
        self.seqs = [p[1] for p in primers]
        self.rules = rules
        self.keep = keep
        self.cutoff = None

    def set_cutoff(self, q: float):
        if q != self.cutoff:
            self.ctx.chop_set(self.seqs, self.rules, q, self.keep)
            self.cutoff = q

    def run(self):
        """Segments of the resident batch: (segments per read, CHOP_SEG_DTYPE records)."""
        self.ctx.chop_exec()
        nseg, _, segs, _ = self.ctx.chop_fetch()
        return nseg, segs

    def autotune(self, sample_idx, samples: int = AUTOTUNE_SAMPLES) -> float:
        """The grid cutoff whose segments over the sampled reads have the greatest summed length
        (usable bases; ties -> the smaller)."""
        grid = autotune_cutoffs(samples)
        best, best_n = grid[0], -1
        sel = np.zeros(self.ctx._n_loaded, dtype=bool)
        sel[sample_idx] = True
        for q in grid:
            self.set_cutoff(q)
            nseg, segs = self.run()
            ok = sel[segs["read"].astype(np.int64)]
            c = int((segs["stop"].astype(np.int64)[ok] - segs["start"][ok]).sum())
            if c > best_n:
                best, best_n = q, c
        return best


def sample_packed(p: lib.Packed, idx: np.ndarray) -> lib.Packed:
    """The reads `idx` of a packed batch as a batch of their own (same packed words, truncated
    after the last sampled read): the autotune runs over the sample only."""
    offs = np.ascontiguousarray(p.offsets[idx])
    lens = np.ascontiguousarray(p.lengths[idx])
    end = int((offs + lens).max()) if len(idx) else 0
    words = min(p.n_words, (end + lib.PACK_PAD + 31) // 32 * 2 + 4)
    return lib.Packed(p.seq2b[:words], p.nmask[:words], offs, lens)


def build_parser():
    p = argparse.ArgumentParser(prog="pychopper",
                                description="dmx: MI355X drop-in for pychopper (-m edlib)")
    p.add_argument("--version", action="version",
                   version=f"dmx {__version__} (pychopper 2.7 compatible reorientation subset)")
    p.add_argument("-b", dest="primers", required=True, help="primer FASTA")
    p.add_argument("-c", dest="config", required=True, help="layout, e.g. +:SP5,-SP27|-:SP27,-SP5")
    p.add_argument("-k", dest="kit", default=None, help="accepted; -b/-c define the primers")
    p.add_argument("-q", dest="cutoff", type=float, default=None)
    p.add_argument("-Q", dest="min_qual", type=float, default=7.0)
    p.add_argument("-z", dest="min_len", type=int, default=50)
    p.add_argument("-Y", dest="autotune_n", type=int, default=10000)
    p.add_argument("-L", dest="autotune_samples", type=int, default=AUTOTUNE_SAMPLES,
                   help="cutoff values tried when tuning -q (evenly spaced on [0.1, 0.6])")
    p.add_argument("-w", dest="rescued")
    p.add_argument("-u", dest="unclass")
    p.add_argument("-l", dest="short")
    p.add_argument("-K", dest="qcfail")
    p.add_argument("-S", dest="stats")
    p.add_argument("-p", dest="keep_primers", action="store_true")
    p.add_argument("-t", dest="threads", type=int, default=8)
    p.add_argument("-m", dest="method", default="edlib")
    p.add_argument("--device", type=int, default=None)
    p.add_argument("--batch-mb", type=int, default=0,
                   help="reader batch size (default: 256, less under a memory budget)")
    p.add_argument("input")
    p.add_argument("output", nargs="?", default="-")
    return p


def _err(msg: str):
    print(f"pychopper (dmx): error: {msg}", file=sys.stderr)
    raise SystemExit(2)


def run(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = build_parser().parse_args(argv)
    if args.method != "edlib":
        _err("only -m edlib is implemented (the pHMM backend is not on this path)")
    if args.cutoff is not None and not 0.0 <= args.cutoff < 1.0:
        _err("-q must be in [0, 1)")
    if args.autotune_samples < 1:
        _err("-L must be at least 1")
    primers = load_primers(args.primers)
    with open(args.config) as fh:
        rules = parse_config(fh.read(), [p[0] for p in primers])
    dev = args.device if args.device is not None else int(os.environ.get("DMX_DEVICE", "0") or 0)
    ctx = lib.Context(dev)
    ch = Chopper(ctx, primers, rules, args.keep_primers)
    paths, outs = [], [-1] * 5
    for kind, pth in ((PASS, args.output), (RESCUED, args.rescued), (UNCLASS, args.unclass),
                      (SHORT, args.short), (QCFAIL, args.qcfail)):
        if pth:
            outs[kind] = len(paths)
            paths.append(pth)
    stats = ChopStats()
    cutoff = args.cutoff
    sink = None
    t0 = time.perf_counter()
    try:
        batch = (args.batch_mb << 20) if args.batch_mb > 0 else nio.batch_bytes_for_budget()
        with nio.Reader(args.input, batch, threads=args.threads) as reader:
            for batch in reader:
                try:
                    if sink is None:
                        sink = nio.Sink(paths, batch.fasta, 1, threads=args.threads)
                    n = len(batch)
                    if not n:
                        continue
                    qc_ok = (np.ones(n, dtype=bool) if batch.fasta
                             else batch.mean_qual() >= args.min_qual)
                    if cutoff is None:   # tune on the -Y sample alone, then load the batch
                        ctx.load(sample_packed(batch.packed,
                                               np.nonzero(qc_ok)[0][:args.autotune_n]))
                        cutoff = ch.autotune(np.arange(ctx._n_loaded), args.autotune_samples)
                    ctx.load(batch.packed)
                    ch.set_cutoff(cutoff)
                    nseg, segs = ch.run()
                    sink.write_rows(batch, *plan_rows(nseg, segs, batch.lens, qc_ok,
                                                      args.min_len, outs))
                    stats.add(nseg, segs, qc_ok, args.min_len)
                finally:
                    batch.free()
        if sink is None:   # empty input: the outputs still exist
            sink = nio.Sink(paths, False, 1, threads=args.threads)
    finally:
        if sink is not None:
            sink.close()
    stats.cutoff = cutoff
    if args.stats:
        stats.write(args.stats)
    print(f"pychopper (dmx {__version__}, MI355X): {stats.n_in} reads in "
          f"{time.perf_counter() - t0:.3f} s, cutoff {cutoff}: {stats.n_found} with primers, "
          f"{stats.n_rescue} rescued, {stats.n_unclass} unclassified, {stats.n_qcfail} QC fail",
          file=sys.stderr)
    ctx.close()
    return 0


def main():
    try:
        sys.exit(run())
    except lib.DmxError as e:
        print(f"pychopper (dmx): GPU error: {e}", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
