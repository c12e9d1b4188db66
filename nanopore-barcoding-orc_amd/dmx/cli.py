"""`cutadapt`-compatible command line for the reference's demultiplexing calls.

Drop-in for the executable the reference's scripts call (boundary = the cutadapt CLI):
  scripts/02_cutadapt_loop.sh:64-72   cutadapt --action=trim -e 0.1 -j 24 --rc
                                      -g file:SP5.fa -o SP5/{name}_DS.fastq.gz IN --json=J
  scripts/02_cutadapt_loop.sh:94-102  cutadapt ... --rc -a file:SP27rc.fa -o SP27/{name}_ID_DS...
  scripts/04_cleaning_primers.sh:377  cutadapt -j N -g F...R [-g F...R] --untrimmed-output=U -o O IN
  scripts/04_cleaning_primers.sh:507  cutadapt -j N -g F -a R ... -o O IN
Supported subset: --action=trim, -e, -O, -j, --rc, -g/-a (file:, NAME=SEQ,
SEQ, linked A...B with -g), -o (with {name} demultiplexing), --untrimmed-output,
--discard-untrimmed, --json, -Z/--compression-level, FASTQ/FASTA(.gz) in and out.
All matching runs on the GPU through libdmx (no CPU fallback): a missing extension or GPU is
an error exit, so `set -euo pipefail` in the calling script aborts.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

from . import __version__
from . import fastx, lib, panel
from .report import Stats


class _AdapterAction(argparse.Action):
    """Keep -g/-a in command-line order (adapter order = tie-break order in best_match)."""

    def __call__(self, parser, ns, values, option_string=None):
        lst = getattr(ns, "adapters", None) or []
        lst.append(("front" if self.dest == "front" else "back", values))
        ns.adapters = lst


def build_parser():
    p = argparse.ArgumentParser(prog="cutadapt", add_help=True,
                                description="dmx: MI355X drop-in for cutadapt (demux subset)")
    p.add_argument("--version", action="version",
                   version=f"dmx {__version__} (cutadapt 4.9 compatible demux subset)")
    p.add_argument("-g", "--front", dest="front", action=_AdapterAction, metavar="ADAPTER")
    p.add_argument("-a", "--adapter", dest="back", action=_AdapterAction, metavar="ADAPTER")
    p.add_argument("-b", "--anywhere", dest="anywhere", action="append")
    p.add_argument("-e", "--error-rate", "--errors", dest="error_rate", type=float, default=0.1)
    p.add_argument("-O", "--overlap", type=int, default=3)
    p.add_argument("-j", "--cores", type=int, default=1)
    p.add_argument("--rc", "--revcomp", dest="rc", action="store_true")
    p.add_argument("--action", default="trim")
    p.add_argument("-o", "--output")
    p.add_argument("--untrimmed-output")
    p.add_argument("--discard-untrimmed", "--trimmed-only", dest="discard_untrimmed",
                   action="store_true")
    p.add_argument("--json")
    p.add_argument("-Z", dest="zlevel1", action="store_true")
    p.add_argument("--compression-level", type=int, default=1)
    p.add_argument("--quiet", action="store_true")
    p.add_argument("--report", default="full")
    p.add_argument("--no-indels", action="store_true")
    p.add_argument("-N", "--no-match-adapter-wildcards", dest="no_adapter_wildcards",
                   action="store_true")
    p.add_argument("--match-read-wildcards", action="store_true")
    p.add_argument("--device", type=int, default=int(os.environ.get("DMX_DEVICE", "0")))
    p.add_argument("--batch-mb", type=int, default=256)
    p.add_argument("input")
    return p


def _unsupported(msg: str):
    print(f"cutadapt (dmx): error: {msg}", file=sys.stderr)
    raise SystemExit(2)


def run(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = build_parser().parse_args(argv)
    if args.action != "trim":
        _unsupported("only --action=trim is implemented")
    if args.anywhere:
        _unsupported("-b (anywhere adapters) is not on the demultiplexing hot path")
    if args.no_indels or args.no_adapter_wildcards or args.match_read_wildcards:
        _unsupported("--no-indels / -N / --match-read-wildcards are not implemented")
    if not getattr(args, "adapters", None):
        _unsupported("at least one -g/-a adapter is required")
    if not args.output:
        _unsupported("-o is required")
    aset = panel.AdapterSet()
    for where, spec in args.adapters:
        aset.add_spec(spec, where)
    ads = aset.adapters
    linked = aset.linked
    if linked and not all(isinstance(a, panel.LinkedAdapter) for a in ads):
        _unsupported("mixing linked and single adapters in one call is not implemented")
    if linked and args.rc:
        _unsupported("--rc with linked adapters is not implemented")
    level = 1 if args.zlevel1 else args.compression_level

    ctx = lib.Context(args.device)
    if linked:
        ctx.set_panel(0, [a.front for a in ads], lib.DMX_FRONT, args.error_rate, args.overlap)
        ctx.set_panel(1, [a.back for a in ads], lib.DMX_BACK, args.error_rate, args.overlap)
        ctx.set_mode(lib.MODE_LINKED)
    else:
        wheres = [lib.DMX_FRONT if a.where == "front" else lib.DMX_BACK for a in ads]
        if len(set(wheres)) == 1:
            ctx.set_panel(0, [a.seq for a in ads], wheres[0] | (lib.DMX_RC if args.rc else 0),
                          args.error_rate, args.overlap)
        else:
            ctx.set_panel_mixed(0, [a.seq for a in ads], wheres, args.rc, args.error_rate,
                                args.overlap)
        ctx.set_mode(lib.MODE_SINGLE)

    demux = "{name}" in args.output
    fasta_out = fastx.is_fasta_path(args.output.replace("{name}", "x"))
    writers: dict[str, fastx.Writer] = {}

    def writer(key: str, path: str) -> fastx.Writer:
        w = writers.get(key)
        if w is None:
            w = writers[key] = fastx.Writer(path, fasta_out, level)
        return w

    names = [a.name for a in ads]
    if demux:   # cutadapt creates every demultiplexed output, also when it stays empty
        for nm in names + ["unknown"]:
            writer(nm, args.output.replace("{name}", nm))
    else:
        writer("__main__", args.output)
        if args.untrimmed_output:
            writer("__untrimmed__", args.untrimmed_output)

    stats = Stats(ads)
    t0 = time.perf_counter()
    for batch in fastx.read_batches(args.input, args.batch_mb << 20):
        n = len(batch)
        if n == 0:
            continue
        blob, offs, lens = batch.seq_offsets()
        res = ctx.run(lib.pack(blob, offs, lens))
        _emit(batch, res, ads, linked, demux, args, writer, stats, fasta_out, lens)
    for w in writers.values():
        w.close()
    if args.json:
        stats.write_json(args.json, argv=argv, cores=args.cores, in_path=args.input,
                         error_rate=args.error_rate)
    if not args.quiet:
        print(f"This is dmx {__version__} (cutadapt 4.9-compatible demultiplexer on MI355X)")
        print(f"Command line parameters: {' '.join(argv)}")
        print(f"Finished in {time.perf_counter() - t0:.3f} s\n")
        stats.summary()
    ctx.close()
    return 0


def _emit(batch, res, ads, linked, demux, args, writer, stats, fasta_out, lens):
    n = len(batch)
    lens = lens.astype(np.int64)
    bin1 = res["bin1"].astype(np.int64)
    matched = bin1 >= 0
    if linked:
        # front part on the read, back part on read[front.rstop:] (LinkedAdapter.match_to)
        start = np.where(matched, res["m1_rstop"], 0).astype(np.int64)
        stop = np.where(matched, start + res["m2_rstart"], lens)
        rc = np.zeros(n, dtype=bool)
    else:
        is_front = np.array([a.where == "front" for a in ads] + [False])[bin1]
        rc = (res["rc1"] == 1) & matched
        start = np.where(matched & is_front, res["m1_rstop"], 0).astype(np.int64)
        stop = np.where(matched & ~is_front, res["m1_rstart"], lens).astype(np.int64)
    stats.n_in += n
    stats.bp_in += int(lens.sum())
    stats.n_with_adapter += int(matched.sum())
    stats.n_rc += int(rc.sum())
    for a in np.unique(bin1[matched]):
        sel = bin1 == a
        stats.matches[int(a)] += int(sel.sum())
        if args.rc:
            stats.on_rc[int(a)] += int((sel & rc).sum())
    for i in np.flatnonzero(matched):
        a = int(bin1[i])
        if linked:
            stats.add_match(a, False, "front", int(res["m1_rstop"][i]), int(res["m1_errors"][i]))
            blen = int(lens[i] - res["m1_rstop"][i])
            stats.add_match(a, False, "back", blen - int(res["m2_rstart"][i]),
                            int(res["m2_errors"][i]))
        elif ads[a].where == "front":
            stats.add_match(a, bool(rc[i]), "front", int(res["m1_rstop"][i]),
                            int(res["m1_errors"][i]))
        else:
            stats.add_match(a, bool(rc[i]), "back", int(lens[i] - res["m1_rstart"][i]),
                            int(res["m1_errors"][i]))

    groups: dict[str, list] = {}
    out_bp = 0
    out_n = 0
    for i in range(n):
        if matched[i]:
            key = ads[int(bin1[i])].name if demux else "__main__"
            rec = fastx.render(batch, i, int(start[i]), int(stop[i]), bool(rc[i]),
                               b" rc" if rc[i] else b"", fasta_out)
            out_bp += int(stop[i] - start[i])
        else:
            if demux:
                key = "unknown"
            elif args.untrimmed_output:
                key = "__untrimmed__"
            elif args.discard_untrimmed:
                stats.n_discard_untrimmed += 1
                continue
            else:
                key = "__main__"
            rec = fastx.render(batch, i, 0, int(lens[i]), False, b"", fasta_out)
            out_bp += int(lens[i])
        out_n += 1
        groups.setdefault(key, []).append(rec)
    stats.n_out += out_n
    stats.bp_out += out_bp
    for key, recs in groups.items():
        writer(key, "").write_chunks(recs)


def main():
    try:
        sys.exit(run())
    except lib.DmxError as e:
        print(f"cutadapt (dmx): GPU error: {e}", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
