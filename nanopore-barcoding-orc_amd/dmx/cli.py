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
from . import fastx, lib, nio, panel
from . import report
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
    p.add_argument("-j", "--cores", type=int, default=1)   # host I/O threads (0 = all)
    p.add_argument("--rc", "--revcomp", dest="rc", action="store_true")
    p.add_argument("--action", default="trim")
    p.add_argument("-o", "--output")
    p.add_argument("--untrimmed-output")
    p.add_argument("--discard-untrimmed", "--trimmed-only", dest="discard_untrimmed",
                   action="store_true")
    p.add_argument("--json")
    # cutadapt 4.9: --compression-level defaults to 5; -Z selects level 1 (here Huffman-only
    # DEFLATE, the fastest stream any inflater reads).  DMX_COMPRESSION_LEVEL changes the
    # default for an unchanged calling script.
    p.add_argument("-Z", dest="zlevel1", action="store_true")
    p.add_argument("--compression-level", type=int,
                   default=int(os.environ.get("DMX_COMPRESSION_LEVEL", "5") or 5))
    p.add_argument("--quiet", action="store_true")
    p.add_argument("--report", default="full")
    p.add_argument("--no-indels", action="store_true")
    p.add_argument("-N", "--no-match-adapter-wildcards", dest="no_adapter_wildcards",
                   action="store_true")
    p.add_argument("--match-read-wildcards", action="store_true")
    p.add_argument("--device", type=int, default=None)
    p.add_argument("--batch-mb", type=int, default=None)
    p.add_argument("input")
    return p


def _unsupported(msg: str):
    print(f"cutadapt (dmx): error: {msg}", file=sys.stderr)
    raise SystemExit(2)


_T_IMPORT = time.perf_counter()


def _since_exec() -> float:
    """Seconds since this process started (Linux /proc, 10 ms resolution; -1 elsewhere)."""
    try:
        with open("/proc/self/stat") as fh:
            start = int(fh.read().rsplit(")", 1)[1].split()[19])
        with open("/proc/uptime") as fh:
            up = float(fh.read().split()[0])
        return up - start / os.sysconf("SC_CLK_TCK")
    except (OSError, ValueError, IndexError):
        return -1.0


_EXEC_TO_IMPORT = _since_exec()


def _phase(name: str, marks: list):
    """DMX_PROFILE_CLI=1: phase timestamps of this call (seconds since the module import)."""
    if marks is not None:
        marks.append((name, time.perf_counter() - _T_IMPORT))


_CTX_CACHE: dict = {}   # (devices, open-time settings) -> contexts kept by the resident server
# the DMX_* switches dmx_open reads once per context (csrc/dmx_api.cpp dmx_open): a cached
# context is reused only by calls with the same values
OPEN_TIME_ENV = ("DMX_NO_FILTER", "DMX_NO_VERIFY", "DMX_RESOLVE", "DMX_NO_SCREEN",
                 "DMX_SCREEN_V1")


def close_cached_contexts():
    for ctxs in _CTX_CACHE.values():
        for c in ctxs:
            c.close()
    _CTX_CACHE.clear()
    nio.drop_retained()


def cached_group(devices) -> list:
    """The resident server's contexts for these devices, opened under the current dmx_open-time
    switches; one set (device memory) is kept at a time."""
    key = (tuple(devices), tuple(os.environ.get(k, "") for k in OPEN_TIME_ENV))
    if key not in _CTX_CACHE:
        close_cached_contexts()
        _CTX_CACHE[key] = lib.open_group(devices)
    return _CTX_CACHE[key]


def run(argv=None, keep_contexts: bool = False) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    marks = [] if os.environ.get("DMX_PROFILE_CLI") == "1" else None
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
    if "{name1}" in args.output or "{name2}" in args.output:
        _unsupported("{name1}/{name2} (cutadapt's combinatorial demultiplexing of paired-end "
                     "reads) needs paired input; single-end demultiplexing takes {name}.  The "
                     "two-round SP5 x SP27 layout {name1}_{name2} is `dmx-demux-loop IN "
                     "--template '{name1}_{name2}.fastq.gz'` (default: the script's "
                     "'{name2}_{name1}_{ds}.fastq.gz')")
    aset = panel.AdapterSet()
    for where, spec in args.adapters:
        aset.add_spec(spec, where)
    ads = aset.adapters
    linked = aset.linked
    if linked and not all(isinstance(a, panel.LinkedAdapter) for a in ads):
        _unsupported("mixing linked and single adapters in one call is not implemented")
    if linked and args.rc:
        _unsupported("--rc with linked adapters is not implemented")

    _phase("args", marks)
    # the reader's producer thread starts on the first batch while the device contexts open
    reader = nio.Reader(args.input, _batch_bytes(args), threads=args.cores)
    try:
        devices = _devices(args)
        if keep_contexts:   # the server's contexts (panels and mode are set again below)
            ctxs = cached_group(devices)
        else:
            ctxs = lib.open_group(devices)
        _phase("open", marks)
        for ctx in ctxs:
            _configure(ctx, ads, linked, args)
        _phase("panel", marks)
        level = 1 if args.zlevel1 else args.compression_level

        demux = "{name}" in args.output
        fasta_out = fastx.is_fasta_path(args.output.replace("{name}", "x"))
        names = [a.name for a in ads]
        if demux:   # cutadapt creates every demultiplexed output, also when it stays empty
            paths = [args.output.replace("{name}", nm) for nm in names]
            if not args.discard_untrimmed:
                paths.append(args.output.replace("{name}", "unknown"))
            unmatched_to = -1 if args.discard_untrimmed else len(names)
        else:
            paths = [args.output] + ([args.untrimmed_output] if args.untrimmed_output else [])
            unmatched_to = 1 if args.untrimmed_output else (-1 if args.discard_untrimmed else 0)

        stats = Stats(ads)
        stats.rc_mode = bool(args.rc)
        stats.min_overlap = args.overlap
        t0 = time.perf_counter()
        a1 = len(ads) if linked else 0
        totals = np.zeros((len(ads) + 1, a1 + 1), dtype=np.int64)
        # the resident server keeps gzip outputs' text for the script's next calls, which read the
        # round-1 bins back (02_cutadapt_loop.sh:91-103); retain_plan says which outputs
        untrimmed = len(names) if demux and not args.discard_untrimmed else None
        retain, keep = retain_plan(paths, untrimmed, reader.in_memory, keep_contexts)
        sink = nio.Sink(paths, fasta_out, level, threads=args.cores, retain_bytes=retain)
    except BaseException:
        reader.close()
        raise
    for o, k in enumerate(keep):
        if retain and not k:
            sink.retain_output(o, False)
    _phase("sink", marks)
    tw = [0.0, 0.0, 0.0]   # read wait, GPU, plan + write enqueue
    try:
        with reader:
            _phase("reader", marks)
            t = time.perf_counter()
            for batch in reader:
                tw[0] += time.perf_counter() - t
                try:
                    if len(batch):
                        t = time.perf_counter()
                        res, cnt = lib.run_batch(ctxs, batch.packed)
                        tw[1] += time.perf_counter() - t
                        t = time.perf_counter()
                        totals += lib.bin_totals(cnt, len(ads), len(ads) if linked else 0)
                        plan = _plan(res, ads, linked, demux, unmatched_to, batch.lens, stats,
                                     batch.packed)
                        sink.write(batch, *plan)
                        tw[2] += time.perf_counter() - t
                finally:
                    batch.free()
                t = time.perf_counter()
        _phase("loop", marks)
    finally:
        sink.close()
    _phase("drain", marks)
    if marks is not None:
        marks.extend([("read_wait", tw[0]), ("gpu", tw[1]), ("plan_write", tw[2])])
    # per-adapter totals: the devices' bin counts (summed over GPUs by RCCL) must agree with the
    # per-read results the outputs were written from
    dev = np.diagonal(totals[1:, 1:]) if linked else totals[1:, 0]
    stats.check_totals(dev)
    stats.n_out = int(sink.n_written.sum())
    stats.bp_out = int(sink.bp_written.sum())
    if args.json:
        stats.write_json(args.json, argv=argv, cores=args.cores, in_path=args.input,
                         error_rate=args.error_rate)
    if not args.quiet:
        print(f"This is dmx {__version__} (cutadapt 4.9-compatible demultiplexer on MI355X)")
        print(f"Command line parameters: {' '.join(argv)}")
        print(f"Finished in {time.perf_counter() - t0:.3f} s on {len(ctxs)} GPU(s)\n")
        stats.summary(error_rate=args.error_rate)
    if not keep_contexts:
        for ctx in ctxs:
            ctx.close()
    _phase("close", marks)
    if marks is not None:
        print("dmx cli phases: " + " ".join(f"{k}={v:.3f}" for k, v in marks) +
              f" exec_to_import={_EXEC_TO_IMPORT:.2f} peak_rss_mb={nio.peak_rss_mb():.0f}",
              file=sys.stderr)
    return 0


def retain_plan(paths, untrimmed, input_in_memory: bool, resident: bool):
    """(cap in bytes, keep flag per output) of the round-2 cache for one call; `untrimmed` is
    the index of the demultiplexed `unknown` output, or None.

    Only outputs a later call reads back are kept: in 02_cutadapt_loop.sh those are round 1's
    SP5 bins (read by the round-2 calls, :91-103).  Not kept: the `unknown` bin (the identifier
    scan at :79 skips it), every output of a call whose input itself came from the cache (a
    round-2 call: its SP27 bins are never read again), and everything outside the resident
    server.  The cap is nio.default_retain_bytes(): DMX_RETAIN_MB, else a quarter of the memory
    still available to the job, at most 8 GiB."""
    if not resident or input_in_memory:
        return 0, [False] * len(paths)
    cap = nio.default_retain_bytes()
    if cap <= 0:
        return 0, [False] * len(paths)
    keep = [p.endswith(".gz") for p in paths]
    if untrimmed is not None:   # the demultiplexed untrimmed bin ({name} -> "unknown")
        keep[untrimmed] = False
    return cap, keep


def _batch_bytes(args) -> int:
    """Reader batch size: --batch-mb / DMX_BATCH_MB, else about a quarter of the input (32..256
    MB), so that a round-2 call's ~200 MB bin is read, demultiplexed and written as a pipeline
    of batches (reading batch i+1 while batch i is written) instead of one batch in series.
    Large inputs keep 256 MB batches (fewer per-batch thread fan-outs)."""
    mb = args.batch_mb or int(os.environ.get("DMX_BATCH_MB", "0") or 0)
    if mb > 0:
        return mb << 20
    cap = nio.batch_bytes_for_budget(256 << 20)   # a memory budget (a SLURM --mem) lowers it
    try:
        size = os.path.getsize(args.input)
    except OSError:
        return cap
    if args.input.endswith(".gz"):
        size *= 2                     # FASTQ deflates to about half
    return int(min(cap, max(32 << 20, size // 4)))


def _devices(args) -> list:
    """GPUs for this call: DMX_GPUS ("all", a count, or a comma list) shards every batch over
    several devices (-j is host I/O threads, the GPU count comes from the
    environment).  An explicit --device / DMX_DEVICE pins one GPU; the default is every
    visible GPU."""
    spec = os.environ.get("DMX_GPUS", "").strip()
    if not spec:
        if args.device is not None:
            return [args.device]
        if os.environ.get("DMX_DEVICE", "").strip():
            return [int(os.environ["DMX_DEVICE"])]
        spec = "all"
    if spec == "all":
        n = lib.device_count()
        if n <= 0:
            raise lib.DmxError("DMX_GPUS=all but no HIP device is visible")
        return list(range(n))
    if "," in spec:
        return [int(x) for x in spec.split(",") if x.strip()]
    n = int(spec)
    if n <= 0:
        raise lib.DmxError("DMX_GPUS must be positive")
    return list(range(n))


def _configure(ctx, ads, linked, args):
    if linked:
        ctx.set_panel(0, [a.front for a in ads], lib.DMX_FRONT, args.error_rate, args.overlap)
        ctx.set_panel(1, [a.back for a in ads], lib.DMX_BACK, args.error_rate, args.overlap)
        ctx.set_mode(lib.MODE_LINKED)
        return
    wheres = [lib.DMX_FRONT if a.where == "front" else lib.DMX_BACK for a in ads]
    if len(set(wheres)) == 1:
        ctx.set_panel(0, [a.seq for a in ads], wheres[0] | (lib.DMX_RC if args.rc else 0),
                      args.error_rate, args.overlap)
    else:
        ctx.set_panel_mixed(0, [a.seq for a in ads], wheres, args.rc, args.error_rate,
                            args.overlap)
    ctx.set_mode(lib.MODE_SINGLE)


def _plan(res, ads, linked, demux, unmatched_to, lens, stats, packed=None):
    """Per-read output index, trim coordinates and orientation (vectorised), and statistics.

    -g (FRONT): RemoveBeforeMatch keeps seq[rstop:]; -a (BACK): RemoveAfterMatch keeps
    seq[:rstart]; linked: read[front.rstop:][:back.rstart]; coordinates of RC hits are on the
    reverse complement, which the sink renders (with " rc" appended to the name)."""
    n = len(res)
    lens = lens.astype(np.int64)
    bin1 = res["bin1"].astype(np.int64)
    matched = bin1 >= 0
    m1_rstart = res["m1_rstart"].astype(np.int64)
    m1_rstop = res["m1_rstop"].astype(np.int64)
    if linked:
        start = np.where(matched, m1_rstop, 0)
        stop = np.where(matched, start + res["m2_rstart"].astype(np.int64), lens)
        rc = np.zeros(n, dtype=bool)
    else:
        is_front = np.array([a.where == "front" for a in ads] + [False])[bin1]
        # ReverseComplementer may pick the reverse complement of a read that matches nothing
        # there (its forward best scored < 0): the unmatched record is then written reversed
        rc = res["rc1"] == 1
        start = np.where(matched & is_front, m1_rstop, 0)
        stop = np.where(matched & ~is_front, m1_rstart, lens)
    if demux:
        out_idx = np.where(matched, bin1, unmatched_to)
    else:
        out_idx = np.where(matched, 0, unmatched_to)

    stats.n_in += n
    stats.bp_in += int(lens.sum())
    stats.n_with_adapter += int(matched.sum())
    stats.n_rc += int(rc.sum())
    if not matched.all() and unmatched_to < 0:
        stats.n_discard_untrimmed += int((~matched).sum())
    bm = bin1[matched]
    stats.add_counts(bm, rc[matched], len(ads))
    e1 = res["m1_errors"].astype(np.int64)[matched]
    if linked:
        stats.add_matches(bm, "front", m1_rstop[matched], e1)
        blen = (lens - m1_rstop)[matched]
        stats.add_matches(bm, "back", blen - res["m2_rstart"].astype(np.int64)[matched],
                          res["m2_errors"].astype(np.int64)[matched])
    else:
        fr = is_front[matched]
        stats.add_matches(bm[fr], "front", m1_rstop[matched][fr], e1[fr])
        stats.add_matches(bm[~fr], "back", (lens - m1_rstart)[matched][~fr], e1[~fr])
        if packed is not None:   # 3' adapters: the base before the match, on the matched view
            ib = np.nonzero(matched & ~is_front)[0]
            stats.add_adjacent(bin1[ib], report.view_codes(packed, ib, rc[ib].astype(np.int64),
                                                           m1_rstart[ib] - 1))
    rc8 = rc.astype(np.uint8)
    return out_idx.astype(np.int32), start.astype(np.int32), stop.astype(np.int32), rc8, rc8


def main():
    try:
        sys.exit(run())
    except lib.DmxError as e:
        print(f"cutadapt (dmx): GPU error: {e}", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
