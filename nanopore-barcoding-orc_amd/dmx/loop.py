"""Fused replacement for scripts/02_cutadapt_loop.sh: both demultiplexing rounds in one pass
(and, with --reorient, scripts/01_pychopper.sh's pychopper step in front of them).

The reference runs cutadapt 13 times per sample (round 1 `-g file:SP5 --rc` at :64-72, then one
`-a file:SP27rc --rc` call per SP5 bin at :91-103), re-reading and re-compressing every read,
and then deletes the `unknown` and SP27_009..012 outputs (:107-119).  This driver reads the
input once, runs DMX_MODE_TWO_ROUND on the GPU(s) (round 2 on the round-1-trimmed, oriented
view of every read, no host round trip) and writes the files the script leaves behind:

  demuxed/SP5/{SP5_i}_{dataset}.fastq.gz            round-1 output per SP5 bin (:70)
  demuxed/SP5/cutadapt_SP5_{dataset}.json           round-1 report (:72)
  demuxed/SP27/{SP27_j}_{SP5_i}_{dataset}.fastq.gz  round-2 output, j <= 8 (:100, :114-118)
  demuxed/SP27/{SP5_i}_{dataset}.json               round-2 report per SP5 bin (:102)

The round-2 names are the two-name layout `{name2}_{name1}_{ds}.fastq.gz` (name1 = the SP5 bin,
name2 = the SP27 bin; the script's `-o SP27/{name}_<id>_<ds>` with <id> = the SP5 bin).
`--template` sets another layout under demuxed/SP27/ (e.g. '{name1}_{name2}.fastq.gz' or
'{name1}/{name2}.fastq'); a name without .gz is written uncompressed.

with the same record content and order as the 13 cutadapt calls (tests/test_cli_gpu.py checks
it against the per-call CLI and the oracle).  `--reorient` takes the RAW reads instead: per
batch it finds the primer segments on the GPU (bin/pychopper's semantics, dmx/chop.py), writes
pychopper's outputs (pychopped/<base>_{pass,rescued,unclass,short}.fastq, <base>_stats.out;
01_pychopper.sh:45-57) and demultiplexes the PASS records straight from the resident batch —
packed from the batch as oriented views (dmx_batch_pack_views), never written and read back —
with the same outputs as bin/pychopper followed by this loop on its PASS file.  `--no-cleanup` also writes the `unknown` and
SP27_009..012 files the script deletes.  Options mirror the script's variables (e_rate,
threads, adapter FASTAs); GPUs as in the CLI (DMX_GPUS / DMX_DEVICE, default all visible).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

from . import __version__, lib, nio, panel
from .cli import _EXEC_TO_IMPORT, _T_IMPORT, _devices
from . import report
from .report import Stats

INVALID_SP27 = ("SP27_009", "SP27_010", "SP27_011", "SP27_012")   # 02_cutadapt_loop.sh:114-118
# 02_cutadapt_loop.sh:100: `-o demuxed/SP27/{name}_${identifier}_${dataset}.fastq.gz` per SP5 bin
DEFAULT_TEMPLATE = "{name2}_{name1}_{ds}.fastq.gz"


def round2_path(outdir: str, template: str, name1: str, name2: str, ds: str) -> str:
    """A round-2 output path: `template` with {name1} (SP5 bin), {name2} (SP27 bin) and {ds}
    (dataset) substituted, under <outdir>/SP27/."""
    rel = template.replace("{name1}", name1).replace("{name2}", name2).replace("{ds}", ds)
    return os.path.join(outdir, "SP27", rel)


def check_template(template: str) -> str | None:
    """Why a --template cannot name every (SP5, SP27) bin apart, or None."""
    if "{name1}" not in template or "{name2}" not in template:
        return "--template needs both {name1} and {name2} (one file per (SP5, SP27) bin)"
    rest = template.replace("{name1}", "").replace("{name2}", "").replace("{ds}", "")
    if "{" in rest or "}" in rest:
        return "--template knows only {name1}, {name2} and {ds}"
    if os.path.isabs(template) or ".." in template.split("/"):
        return "--template is a path under <outdir>/SP27/"
    return None


def dataset_name(infile: str) -> str:
    """02_cutadapt_loop.sh:26-35."""
    ds = os.path.basename(infile)
    if ds.startswith("pychopped_"):
        ds = ds[len("pychopped_"):]
    for suf in (".fastq.gz", ".fastq", ".fq.gz", ".fq", ".gz", "_pass"):
        if ds.endswith(suf):
            ds = ds[:-len(suf)]
    return ds


def build_parser():
    p = argparse.ArgumentParser(prog="dmx-demux-loop",
                                description="fused scripts/02_cutadapt_loop.sh on MI355X")
    p.add_argument("infile")
    p.add_argument("-e", "--e-rate", type=float, default=0.1)
    p.add_argument("-j", "--threads", type=int, default=24)
    p.add_argument("--sp5", default=panel.SP5_FASTA, help="adapters_SP5 FASTA (:43)")
    p.add_argument("--sp27", default=panel.SP27RC_FASTA, help="adapters_SP27 FASTA (:44)")
    p.add_argument("--outdir", default=None, help="default: $(dirname $(dirname IN))/demuxed")
    p.add_argument("--no-cleanup", action="store_true",
                   help="keep the unknown and SP27_009..012 outputs (:107-119 delete them)")
    p.add_argument("--template", default=DEFAULT_TEMPLATE,
                   help="round-2 output names under <outdir>/SP27/: {name1} = SP5 bin, {name2} "
                        "= SP27 bin ('unknown' for the --no-cleanup round-2 unknown files), "
                        "{ds} = dataset (default: the script's " + DEFAULT_TEMPLATE + ")"),
    # cutadapt's defaults (the script's calls pass neither): level 5; -Z = level 1
    p.add_argument("--compression-level", type=int,
                   default=int(os.environ.get("DMX_COMPRESSION_LEVEL", "5") or 5))
    p.add_argument("-Z", dest="zlevel1", action="store_true")
    p.add_argument("--batch-mb", type=int, default=int(os.environ.get("DMX_BATCH_MB", "0") or 0),
                   help="reader batch size (default: 256, less under a memory budget: "
                        "nio.batch_bytes_for_budget)")
    p.add_argument("--device", type=int, default=None)
    # 01 -> 02 fused: INFILE is the raw reads; reorient them as 01_pychopper.sh does, write its
    # outputs, and demultiplex its PASS records straight from the resident batch
    p.add_argument("--reorient", action="store_true",
                   help="INFILE = raw reads: run 01_pychopper.sh's pychopper step first (its "
                        "outputs in --pychopper-dir) and demultiplex its PASS records")
    p.add_argument("--pychopper-dir", default=None, help="default: $(dirname IN)/pychopped")
    p.add_argument("--primers", default=None, help="pychopper -b (M13_seqs_for_pychopper.fa)")
    p.add_argument("--layout", default=None, help="pychopper -c (M13_config_for_pychopper.txt)")
    p.add_argument("-Q", dest="min_qual", type=float, default=10.0, help="pychopper -Q (:17)")
    p.add_argument("-z", dest="min_len", type=int, default=50, help="pychopper -z")
    p.add_argument("-q", dest="cutoff", type=float, default=None, help="pychopper -q")
    p.add_argument("-Y", dest="autotune_n", type=int, default=10000, help="pychopper -Y")
    p.add_argument("-L", dest="autotune_samples", type=int, default=None, help="pychopper -L")
    p.add_argument("--no-keep-primers", action="store_true", help="pychopper without -p")
    return p


def view_coords(vs, ve, vst, a, b, o):
    """Sub-range [a, b) of orient(P, o), P = orient(read[vs:ve], vst) (a pychopper segment), as
    (start, stop, orientation) on the read itself: with t = vst ^ o, orient(read[vs:ve], t)[a:b]
    is read[vs + a : vs + b] (t = 0) or the reverse complement of read[ve - b : ve - a]."""
    t = (vst.astype(np.uint8) ^ o.astype(np.uint8)).astype(np.uint8)
    vs, ve = vs.astype(np.int64), ve.astype(np.int64)
    a, b = a.astype(np.int64), b.astype(np.int64)
    return np.where(t == 1, ve - b, vs + a), np.where(t == 1, ve - a, vs + b), t


def base_name(infile: str) -> str:
    """01_pychopper.sh:21-26: the input's file name without .gz, then .fastq / .fq."""
    b = os.path.basename(infile)
    for suf in (".gz",):
        if b.endswith(suf):
            b = b[:-len(suf)]
    for suf in (".fastq", ".fq"):
        if b.endswith(suf):
            b = b[:-len(suf)]
            break
    return b


def plan_rounds(res, lens):
    """Composite trim coordinates of both rounds on the original read.

    Round 1 (FRONT, --rc): T1 = orient(read, rc1)[s1:] with s1 = m1.rstop.  Round 2 (BACK, --rc)
    on T1: keep orient(T1, rc2)[:r2] with r2 = m2.rstart.  With revcomp(orient(x, o)[a:b]) =
    orient(x, !o)[n-b:n-a] the round-2 output is orient(read, rc1)[s1 : s1 + r2] if rc2 == 0
    and orient(read, !rc1)[0 : r2] if rc2 == 1; its name carries one " rc" per RC'd round."""
    lens = lens.astype(np.int64)
    rc1 = res["rc1"].astype(np.uint8)
    rc2 = res["rc2"].astype(np.uint8)
    s1 = res["m1_rstop"].astype(np.int64)
    r2 = res["m2_rstart"].astype(np.int64)
    start2 = np.where(rc2 == 1, 0, s1)
    stop2 = np.where(rc2 == 1, r2, s1 + r2)
    orient2 = (rc1 ^ rc2).astype(np.uint8)
    return (s1, lens, rc1), (start2, stop2, orient2, (rc1 + rc2).astype(np.uint8))


def run(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = build_parser().parse_args(argv)
    infile = args.infile
    base = pych_dir = None
    if args.reorient:   # 01_pychopper.sh:21-31 names; 02 reads pychopped/pychopped_<base>
        base = base_name(infile)
        pych_dir = args.pychopper_dir or os.path.join(os.path.dirname(os.path.abspath(infile)),
                                                      "pychopped")
        ds = base
        demux_in = os.path.join(pych_dir, f"pychopped_{base}.gz")
    else:
        ds = dataset_name(infile)
        demux_in = infile
    why = check_template(args.template)
    if why:
        print(f"dmx-demux-loop: error: {why}", file=sys.stderr)
        return 2
    outdir = args.outdir or os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(demux_in))), "demuxed")
    print("=========================================")
    print(f"Processing: {infile}")
    print(f"Dataset name: {ds}")
    print(f"Output directory: {outdir}")
    print("=========================================")
    chop_files = ()
    if args.reorient:
        from . import chop
        args.primers = args.primers or chop.PRIMERS_FASTA
        args.layout = args.layout or chop.CONFIG_FILE
        chop_files = (args.primers, args.layout)
    for f in (infile, args.sp5, args.sp27) + chop_files:
        if not os.path.isfile(f):
            print(f"Error: Required file not found: {f}")
            return 1
    os.makedirs(os.path.join(outdir, "SP5"), exist_ok=True)
    os.makedirs(os.path.join(outdir, "SP27"), exist_ok=True)
    aset1, aset2 = panel.AdapterSet(), panel.AdapterSet()
    aset1.add_spec(f"file:{args.sp5}", "front")
    aset2.add_spec(f"file:{args.sp27}", "back")
    ads1, ads2 = aset1.adapters, aset2.adapters
    n1, n2 = [a.name for a in ads1], [a.name for a in ads2]

    # outputs: round 1 = one file per SP5 adapter (+ unknown); round 2 = per (SP5, SP27) pair
    keep2 = [j for j, nm in enumerate(n2) if args.no_cleanup or nm not in INVALID_SP27]
    p1 = [f"{outdir}/SP5/{nm}_{ds}.fastq.gz" for nm in n1]
    if args.no_cleanup:
        p1.append(f"{outdir}/SP5/unknown_{ds}.fastq.gz")
    out2 = np.full((len(n1), len(n2) + 1), -1, dtype=np.int32)   # [bin1, bin2 + 1] -> output
    p2 = []
    for i, ident in enumerate(n1):
        if args.no_cleanup:
            out2[i, 0] = len(p2)
            p2.append(round2_path(outdir, args.template, ident, "unknown", ds))
        for j in keep2:
            out2[i, j + 1] = len(p2)
            p2.append(round2_path(outdir, args.template, ident, n2[j], ds))
    if len(set(p2)) != len(p2):
        print("dmx-demux-loop: error: --template gives two bins the same file", file=sys.stderr)
        return 2
    for d in sorted({os.path.dirname(x) for x in p2}):
        os.makedirs(d, exist_ok=True)

    marks = [("setup", time.perf_counter() - _T_IMPORT)]   # DMX_PROFILE_IO phase marks
    # the reader's producer thread starts on the first batch while the device contexts open
    batch = (args.batch_mb << 20) if args.batch_mb > 0 else nio.batch_bytes_for_budget()
    reader = nio.Reader(infile, batch, threads=args.threads)
    ctxs = []
    try:   # from the reader on: any failure closes whatever is open
        return _loop_body(args, argv, infile, outdir, ds, demux_in, pych_dir, base, ads1, ads2,
                          n1, n2, out2, p1, p2, marks, reader, ctxs)
    except BaseException:
        reader.close()
        for ctx in ctxs:
            ctx.close()
        raise


def _loop_body(args, argv, infile, outdir, ds, demux_in, pych_dir, base, ads1, ads2, n1, n2,
               out2, p1, p2, marks, reader, ctxs):
    """The fused loop after the reader is open; `ctxs` is filled in place so that the caller can
    close the device contexts when anything here raises (sinks and the reorienter are closed
    below on every path)."""
    ctxs.extend(lib.open_group(_devices(args)))
    reo = sink1 = sink2 = None
    marks.append(("open", time.perf_counter() - _T_IMPORT))
    for ctx in ctxs:
        ctx.set_panel(0, [a.seq for a in ads1], lib.DMX_FRONT | lib.DMX_RC, args.e_rate, 3)
        ctx.set_panel(1, [a.seq for a in ads2], lib.DMX_BACK | lib.DMX_RC, args.e_rate, 3)
        ctx.set_mode(lib.MODE_TWO_ROUND)

    st1 = Stats(ads1)
    st1.rc_mode = True
    st2 = []
    for _ in n1:
        s = Stats(ads2)
        s.rc_mode = True
        st2.append(s)
    try:
        if args.reorient:
            reo = Reorienter(args, pych_dir, base)
        t0 = time.perf_counter()
        marks.append(("outputs", t0 - _T_IMPORT))
        print("Round 1: Demultiplexing with SP5 adapters...")
        print("Round 2: Demultiplexing with SP27 adapters (fused with round 1)...")
        level = 1 if args.zlevel1 else args.compression_level
        sink1 = nio.Sink(p1, False, level, threads=args.threads)
        sink2 = nio.Sink(p2, False, level, threads=args.threads)
        marks.append(("sinks", time.perf_counter() - _T_IMPORT))
    except BaseException:
        for x in (sink1, sink2, reo):
            if x is not None:
                try:
                    x.close()
                except Exception:   # the original error is the one to report
                    pass
        raise
    bp2_out = np.zeros(len(n1), np.int64)
    prof = dict(read_wait=0.0, gpu=0.0, plan_write=0.0, drain=0.0)
    # parts of plan_write: coordinates, the two sink hand-offs (each waits for that sink's
    # previous batch to be rendered, compressed and written), the report statistics
    prof.update(pw_plan=0.0, pw_write1=0.0, pw_write2=0.0, pw_stats=0.0)
    if reo is not None:   # parts of "gpu": pychopper step, view packing
        prof.update(reo=0.0, pack=0.0)
    n2_out = np.zeros(len(n1), np.int64)
    totals = np.zeros((len(n1) + 1, len(n2) + 1), dtype=np.int64)   # device bin counts
    try:
        while True:
            tw = time.perf_counter()
            batch = reader.next()
            prof["read_wait"] += time.perf_counter() - tw
            if batch is None:
                break
            try:
                if not len(batch):
                    continue
                tw = time.perf_counter()
                views = None
                packed, lens = batch.packed, batch.lens
                if reo is not None:   # the PASS records of 01_pychopper.sh, as views
                    views = reo.batch(batch)
                    tp = time.perf_counter()
                    prof["reo"] += tp - tw
                    packed = batch.pack_views(views[0], views[1], views[2], views[3],
                                              threads=args.threads)
                    prof["pack"] += time.perf_counter() - tp
                    lens = packed.lengths
                    if not len(lens):
                        continue
                res, cnt = lib.run_batch(ctxs, packed)
                totals += lib.bin_totals(cnt, len(n1), len(n2))
                prof["gpu"] += time.perf_counter() - tw
                tw = time.perf_counter()
                (s1, e1, o1), (s2, e2, o2, nrc2) = plan_rounds(res, lens)
                b1 = res["bin1"].astype(np.int64)
                b2 = res["bin2"].astype(np.int64)
                m1 = b1 >= 0
                idx1 = np.where(m1, b1, len(n1) if args.no_cleanup else -1)
                # unmatched in round 1 is written untrimmed to unknown (--no-cleanup only)
                s1w = np.where(m1, s1, 0)
                o1w = o1.astype(np.uint8)   # an unmatched read may still be taken RC'd
                tq = time.perf_counter()
                prof["pw_plan"] += tq - tw
                if views is None:
                    sink1.write(batch, idx1, s1w, e1, o1w, o1w)
                else:
                    x, y, t = view_coords(views[1], views[2], views[3], s1w, e1, o1w)
                    sink1.write_rows2(batch, views[0], idx1, x, y, t, views[1], views[2],
                                      views[3], o1w)
                tr = time.perf_counter()
                prof["pw_write1"] += tr - tq
                idx2 = np.where(m1, out2[np.maximum(b1, 0), b2 + 1], -1)
                # round-2 unknown: the round-1 output record, untrimmed by round 2
                m2 = b2 >= 0
                # unmatched in round 2 but taken reverse-complemented: RC of the round-1
                # record T1 = orient(read, rc1)[s1:n], i.e. orient(read, !rc1)[0 : n - s1]
                u2rc = ~m2 & (res["rc2"] == 1)
                s2w = np.where(m2, s2, np.where(u2rc, 0, s1))
                e2w = np.where(m2, e2, np.where(u2rc, e1 - s1, e1))
                o2w = np.where(m2, o2, np.where(u2rc, 1 - o1, o1)).astype(np.uint8)
                n2w = np.where(m2, nrc2, o1 + u2rc).astype(np.uint8)
                tq = time.perf_counter()
                prof["pw_plan"] += tq - tr
                if views is None:
                    sink2.write(batch, idx2, s2w, e2w, o2w, n2w)
                else:
                    x, y, t = view_coords(views[1], views[2], views[3], s2w, e2w, o2w)
                    sink2.write_rows2(batch, views[0], idx2, x, y, t, views[1], views[2],
                                      views[3], n2w)
                tr = time.perf_counter()
                prof["pw_write2"] += tr - tq
                _round_stats(st1, st2, res, lens, m1, m2, b1, b2, s1, s2w, e2w,
                             bp2_out, n2_out, packed)
                tq = time.perf_counter()
                prof["pw_stats"] += tq - tr
                prof["plan_write"] += tq - tw
            finally:
                tf = time.perf_counter()
                batch.free()
                prof["free"] = prof.get("free", 0.0) + time.perf_counter() - tf
    finally:
        tw = time.perf_counter()
        marks.append(("loop", tw - _T_IMPORT))
        reader.close()
        sink1.close()
        sink2.close()
        if reo is not None:
            reo.close()
        prof["drain"] += time.perf_counter() - tw
        marks.append(("drain", time.perf_counter() - _T_IMPORT))
    if reo is not None:
        prof.update({"reo_" + k: v for k, v in reo.prof.items()})
    # the devices' (SP5, SP27) bin counts (RCCL-summed over GPUs) vs the per-read results
    st1.check_totals(totals[1:, :].sum(axis=1))
    for i, s in enumerate(st2):
        s.check_totals(totals[i + 1, 1:])
    st1.n_out = int(sink1.n_written.sum())
    st1.bp_out = int(sink1.bp_written.sum())
    for i, s in enumerate(st2):
        s.n_out, s.bp_out = int(n2_out[i]), int(bp2_out[i])
    st1.write_json(f"{outdir}/SP5/cutadapt_SP5_{ds}.json", argv=["dmx-demux-loop"] + argv,
                   cores=args.threads, in_path=demux_in, error_rate=args.e_rate)
    print(f"Found {len(n1)} identifiers from SP5 demultiplexing")
    for i, ident in enumerate(n1):
        st2[i].write_json(f"{outdir}/SP27/{ident}_{ds}.json",
                          argv=["dmx-demux-loop"] + argv, cores=args.threads,
                          in_path=f"{outdir}/SP5/{ident}_{ds}.fastq.gz", error_rate=args.e_rate)
    marks.append(("reports", time.perf_counter() - _T_IMPORT))
    for ctx in ctxs:
        ctx.close()
    marks.append(("close", time.perf_counter() - _T_IMPORT))
    if os.environ.get("DMX_PROFILE_IO"):   # phases: seconds since the module import
        print("io profile (s): " + ", ".join(f"{k} {v:.3f}" for k, v in prof.items()) +
              f"; peak_rss_mb {nio.peak_rss_mb():.0f}; phases " +
              " ".join(f"{k}={v:.3f}" for k, v in marks) +
              f" exec_to_import={_EXEC_TO_IMPORT:.2f}", file=sys.stderr)
    print("Demultiplexing complete!")
    print(f"Finished in {time.perf_counter() - t0:.3f} s on {len(ctxs)} GPU(s): "
          f"{st1.n_in:,} reads, {st1.n_with_adapter:,} with an SP5 adapter")
    print("Pipeline complete!")
    print(f"Results in: {outdir}")
    return 0


class Reorienter:
    """The pychopper step of 01_pychopper.sh:45-57 inside the fused loop (dmx/chop.py semantics,
    its own device context): per batch, primer hits and segments on the GPU, pychopper's five
    outputs written, and the PASS records (one segment, QC pass, >= -z nt) returned as views
    (read, start, stop, strand) for the demultiplexer."""

    def __init__(self, args, pych_dir: str, base: str):
        from . import chop
        self.chop = chop
        self.args = args
        os.makedirs(pych_dir, exist_ok=True)
        primers = chop.load_primers(args.primers)
        with open(args.layout) as fh:
            rules = chop.parse_config(fh.read(), [p[0] for p in primers])
        dev = args.device if args.device is not None else int(os.environ.get("DMX_DEVICE", "0")
                                                               or 0)
        self.ctx = lib.Context(dev)
        self.ch = chop.Chopper(self.ctx, primers, rules, not args.no_keep_primers)
        # 01_pychopper.sh:47-57: -w rescued, -u unclass, -l short, -S stats, PASS to stdout
        self.paths = [os.path.join(pych_dir, f"{base}_{k}.fastq")
                      for k in ("pass", "rescued", "unclass", "short")]
        self.stats_path = os.path.join(pych_dir, f"{base}_stats.out")
        self.outs = [0, 1, 2, 3, -1]   # PASS, RESCUED, UNCLASS, SHORT, QCFAIL (no -K)
        self.sink = None
        self.stats = chop.ChopStats()
        self.cutoff = args.cutoff
        self.t0 = time.perf_counter()
        self.prof = dict(qual=0.0, tune=0.0, chop=0.0, rows=0.0)   # parts of the io profile's "reo"

    def _tick(self, key, t):
        now = time.perf_counter()
        self.prof[key] += now - t
        return now

    def batch(self, b):
        chop, a = self.chop, self.args
        if self.sink is None:
            self.sink = nio.Sink(self.paths, b.fasta, 1, threads=a.threads)
        n = len(b)
        t = time.perf_counter()
        qc_ok = np.ones(n, dtype=bool) if b.fasta else b.mean_qual() >= a.min_qual
        t = self._tick("qual", t)
        if self.cutoff is None:   # tuned on the first -Y QC-passing reads (bin/pychopper's rule)
            self.ctx.load(chop.sample_packed(b.packed, np.nonzero(qc_ok)[0][:a.autotune_n]))
            self.cutoff = self.ch.autotune(np.arange(self.ctx._n_loaded),
                                           a.autotune_samples or chop.AUTOTUNE_SAMPLES)
            t = self._tick("tune", t)
        self.ctx.load(b.packed)
        self.ch.set_cutoff(self.cutoff)
        nseg, segs = self.ch.run()
        t = self._tick("chop", t)
        self.sink.write_rows(b, *chop.plan_rows(nseg, segs, b.lens, qc_ok, a.min_len, self.outs))
        self.stats.add(nseg, segs, qc_ok, a.min_len)
        self._tick("rows", t)
        sread = segs["read"].astype(np.int64)
        sstart = segs["start"].astype(np.int64)
        sstop = segs["stop"].astype(np.int64)
        ok = (qc_ok[sread] & (nseg.astype(np.int64)[sread] == 1) & (sstop - sstart >= a.min_len))
        # plan_rows's PASS rows, in read order (segments come in read order)
        return (sread[ok].astype(np.uint32), sstart[ok].astype(np.int32),
                sstop[ok].astype(np.int32), segs["strand"][ok].astype(np.uint8))

    def close(self):
        if self.sink is None:   # empty input: the outputs still exist
            self.sink = nio.Sink(self.paths, False, 1, threads=self.args.threads)
        self.sink.close()
        self.stats.cutoff = self.cutoff
        self.stats.write(self.stats_path)
        s = self.stats
        print(f"pychopper (dmx {__version__}, MI355X, fused): {s.n_in} reads in "
              f"{time.perf_counter() - self.t0:.3f} s, cutoff {self.cutoff}: {s.n_found} with "
              f"primers, {s.n_rescue} rescued, {s.n_unclass} unclassified, {s.n_qcfail} QC fail",
              file=sys.stderr)
        self.ctx.close()


def _round_stats(st1, st2, res, lens, m1, m2, b1, b2, s1, s2w, e2w, bp2_out, n2_out,
                 packed=None):
    lens = lens.astype(np.int64)
    n = len(res)
    rc1 = res["rc1"] == 1
    st1.n_in += n
    st1.bp_in += int(lens.sum())
    st1.n_with_adapter += int(m1.sum())
    st1.n_rc += int(rc1.sum())
    st1.add_counts(b1[m1], rc1[m1], len(st1.adapters))
    st1.add_matches(b1[m1], "front", s1[m1], res["m1_errors"].astype(np.int64)[m1])
    # round 2, one report per SP5 bin: its input is that bin's round-1 output
    len1 = lens - s1
    rc2 = (res["rc2"] == 1) & m1
    adj = None
    if packed is not None:
        # base before each round-2 (3') match, on the round-2 view: the round-1 output
        # T1 = orient(read, rc1)[s1:], reverse-complemented when rc2 — position p of it is
        # orient(read, rc1)[s1 + p], or orient(read, 1 - rc1)[p] on the reverse complement
        hit_all = np.nonzero(m1 & m2)[0]
        p = res["m2_rstart"].astype(np.int64)[hit_all] - 1
        r1 = res["rc1"].astype(np.int64)[hit_all]
        two = res["rc2"].astype(np.int64)[hit_all] == 1
        codes = report.view_codes(packed, hit_all, np.where(two, 1 - r1, r1),
                                  np.where(two, p, np.where(p >= 0, s1[hit_all] + p, -1)))
        adj = np.full(n, 4, np.int64)
        adj[hit_all] = codes
    # every SP5 bin at once: per-bin sums are bincounts over the round-1 bin, the round-2
    # histograms one unique over (bin1, adapter2, removed, errors) keys, sliced per bin (the
    # statistics of a bin are those of the reads a boolean mask of the bin would select)
    nb1, nb2 = len(st2), len(st2[0].adapters) if st2 else 0
    sel = np.nonzero(m1)[0]
    bsel = b1[sel]

    def per_bin(v):
        w = np.asarray(v, np.int64)[sel]
        return np.bincount(bsel, weights=w, minlength=nb1).round().astype(np.int64)

    n_in = np.bincount(bsel, minlength=nb1)
    bp_in = per_bin(len1)
    n_rc = per_bin(rc2)
    bp_out = per_bin(np.where(m2, e2w - s2w, len1))
    r2 = res["m2_rstart"].astype(np.int64)
    err2 = res["m2_errors"].astype(np.int64)
    hit = np.nonzero(m1 & m2)[0]
    hb1, hb2 = b1[hit], b2[hit]
    pair = hb1 * nb2 + hb2
    cnt2 = np.bincount(pair, minlength=nb1 * nb2).reshape(nb1, nb2)
    rcnt2 = np.bincount(pair[rc2[hit]], minlength=nb1 * nb2).reshape(nb1, nb2)
    key = (hb1 << 48) | (hb2 << 40) | ((len1 - r2)[hit] << 8) | err2[hit]
    u, c = np.unique(key, return_counts=True)
    ue = np.searchsorted(u >> 48, np.arange(nb1 + 1))
    adjc = None
    if adj is not None:
        adjc = np.bincount(pair * 5 + adj[hit], minlength=nb1 * nb2 * 5).reshape(nb1, nb2, 5)
    low = (1 << 48) - 1
    for i, s in enumerate(st2):
        if not n_in[i]:
            continue
        s.n_in += int(n_in[i])
        s.bp_in += int(bp_in[i])
        s.n_with_adapter += int(cnt2[i].sum())
        s.n_rc += int(n_rc[i])
        s.add_count_vectors(cnt2[i], rcnt2[i])
        if ue[i] < ue[i + 1]:
            s.add_match_counts("back", u[ue[i]:ue[i + 1]] & low, c[ue[i]:ue[i + 1]])
        if adjc is not None and cnt2[i].any():
            s.add_adjacent_counts(adjc[i])
        # reads the per-call cutadapt would write (all of them: unknown included), before the
        # script's cleanup deletes files
        n2_out[i] += int(n_in[i])
        bp2_out[i] += int(bp_out[i])


def main():
    try:
        sys.exit(run())
    except lib.DmxError as e:
        print(f"dmx-demux-loop: GPU error: {e}", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
