"""End-to-end wall time of the demultiplexing step on a synthetic FASTQ(.gz) (not the bench line).

SURVEY.md §8d asks for kernel time on resident reads (bench.py) and, separately, the
end-to-end wall time including gzip and parse.  This tool generates `--reads` reads of a
workload (default c2: 12x12 panel, lognormal ~1.2 kb) with random qualities, writes them as
FASTQ.gz (level 1, parallel members, via libdmx_io), then times
  fused : bin/dmx-demux-loop IN       (one pass, both rounds; what 02_cutadapt_loop.sh leaves)
          on plain FASTQ (01_pychopper.sh:57 writes *_pass.fastq uncompressed), on our
          multi-member .gz (member-parallel inflate) and on an ordinary single-member .gz
          (speculative chunk-parallel inflate; DMX_E2E_SEQ_A_B=1 adds zlib's sequential path)
  calls : the 13 bin/cutadapt calls of 02_cutadapt_loop.sh:64-103 (per-call drop-in)
  pychopper (--pychopper): bin/pychopper with 01_pychopper.sh:45-57's flags on the .gz input
  reorient (--reorient): 01 -> 02 on the raw single-member .gz, two ways: bin/pychopper then
          bin/dmx-demux-loop on its PASS file (the two scripts), and bin/dmx-demux-loop
          --reorient (one pass); both at the default level 5
and prints one JSON line with reads/s for each.  Usage:
  python tools/e2e_bench.py --reads 1000000 [--workload c2] [--threads 16] [--skip-calls]
                            [--skip-fused] [--pychopper] [--reorient]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import tempfile
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nanopore-barcoding-orc_amd")
sys.path.insert(0, PKG)

from dmx import chop, nio, panel, synth  # noqa: E402


def write_fastq(path_plain: str, d: dict, seed: int, chunk: int = 100_000) -> int:
    """FASTQ text assembled with numpy (names r<i>, Phred 5..40), chunk by chunk."""
    rng = np.random.default_rng(seed)
    blob, offs, lens = d["blob"], d["offsets"].astype(np.int64), d["lengths"].astype(np.int64)
    n = len(lens)
    with open(path_plain, "wb") as fh:
        for lo in range(0, n, chunk):
            hi = min(n, lo + chunk)
            names = [f"@r{i} ch={i % 512}\n".encode() for i in range(lo, hi)]
            nl = np.array([len(x) for x in names], np.int64)
            L = lens[lo:hi]
            size = nl + L + 3 + L + 1
            rec = np.zeros(hi - lo + 1, np.int64)
            rec[1:] = np.cumsum(size)
            out = np.empty(int(rec[-1]), np.uint8)
            name_blob = np.frombuffer(b"".join(names), np.uint8)
            nstart = np.concatenate([[0], np.cumsum(nl)[:-1]])
            idx = np.repeat(rec[:-1] - nstart, nl) + np.arange(len(name_blob))
            out[idx] = name_blob
            s0 = rec[:-1] + nl
            tot = int(L.sum())
            rel = np.arange(tot) - np.repeat(np.cumsum(L) - L, L)
            sidx = np.repeat(s0, L) + rel
            out[sidx] = blob[np.repeat(offs[lo:hi], L) + rel]
            out[s0 + L] = 10
            out[s0 + L + 1] = 43
            out[s0 + L + 2] = 10
            out[sidx + np.repeat(L + 3, L)] = rng.integers(38, 74, tot, dtype=np.uint8)
            out[rec[1:] - 1] = 10
            fh.write(out.tobytes())
    return n


def gzip_native(src: str, dst: str, threads: int):
    sink = nio.Sink([dst], False, 1, threads=threads)
    with nio.Reader(src, 256 << 20, threads=threads) as r:
        for b in r:
            n = len(b)
            z = np.zeros(n, np.uint8)
            sink.write(b, np.zeros(n, np.int32), np.zeros(n, np.int32), b.lens.astype(np.int32),
                       z, z)
            b.free()
    sink.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--skip-calls", action="store_true")
    ap.add_argument("--skip-fused", action="store_true")
    ap.add_argument("--pychopper", action="store_true")
    ap.add_argument("--reorient", action="store_true")
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--single-level", type=int, default=1,
                    help="zlib level of the single-member .gz (default strategy: LZ77 + "
                         "dynamic Huffman blocks, as `gzip -N` writes)")
    ap.add_argument("--calls-input", choices=["single", "members"], default="single",
                    help="round-1 input of the 13 calls: the single-member .gz (what "
                         "02_cutadapt_loop.sh reads, pychopped_<ds>.gz) or our multi-member .gz")
    ap.add_argument("--mem-budget-mb", type=int, default=0,
                    help="DMX_MEM_BUDGET_MB for the timed commands (a SLURM job's --mem: 4096 "
                         "for 02_cutadapt_loop.sh, 2048 for 01_pychopper.sh)")
    a = ap.parse_args()
    if a.mem_budget_mb:
        os.environ["DMX_MEM_BUDGET_MB"] = str(a.mem_budget_mb)
    wd = a.workdir or tempfile.mkdtemp(prefix="dmx_e2e_")
    pych = os.path.join(wd, "pychopped")
    os.makedirs(pych, exist_ok=True)
    t = time.perf_counter()
    d = synth.generate(a.workload, n=a.reads, seed=77)
    plain = os.path.join(pych, "pychopped_e2e.fastq")
    gz = plain + ".gz"
    write_fastq(plain, d, seed=5)
    gzip_native(plain, gz, a.threads)
    # an ordinary single-member gzip (`gzip -1`-like: LZ77 + dynamic blocks, no size fields):
    # the reader inflates it in speculative parallel chunks (csrc/dmx_inflate.h)
    gz1 = os.path.join(wd, "single", "pychopped_e2e.fastq.gz")
    os.makedirs(os.path.dirname(gz1), exist_ok=True)
    with open(plain, "rb") as fi, open(gz1, "wb") as fo:
        c = zlib.compressobj(a.single_level, zlib.DEFLATED, 31, 8, zlib.Z_DEFAULT_STRATEGY)
        while True:
            chunk = fi.read(64 << 20)
            if not chunk:
                break
            fo.write(c.compress(chunk))
        fo.write(c.flush())
    gen_s = time.perf_counter() - t
    raw_bytes, gz_bytes = os.path.getsize(plain), os.path.getsize(gz)
    env = dict(os.environ)
    res = {"workload": a.workload, "reads": a.reads, "threads": a.threads,
           "mem_budget_mb": a.mem_budget_mb or None,
           "input_fastq_bytes": raw_bytes, "input_gz_bytes": gz_bytes, "gen_s": round(gen_s, 1)}

    if a.pychopper:   # 01_pychopper.sh:45-57, PASS to a file as the script's redirect does
        po = os.path.join(wd, "pychopper_out")
        os.makedirs(po, exist_ok=True)
        cmd = [os.path.join(PKG, "bin", "pychopper"), "-b", chop.PRIMERS_FASTA,
               "-c", chop.CONFIG_FILE, "-k", "LSK114", "-Q", "10", "-w", f"{po}/rescued.fastq",
               "-u", f"{po}/unclass.fastq", "-l", f"{po}/short.fastq", "-S", f"{po}/stats.out",
               "-p", "-t", str(a.threads), "-m", "edlib", gz]
        t = time.perf_counter()
        with open(f"{po}/pass.fastq", "wb") as fh:
            p = subprocess.run(cmd, check=True, stdout=fh, stderr=subprocess.PIPE, text=True)
        ps = time.perf_counter() - t
        res["pychopper_gz_s"] = round(ps, 3)
        res["pychopper_gz_reads_per_s"] = round(a.reads / ps, 1)
        res["pychopper_report"] = p.stderr.strip().splitlines()[-1] if p.stderr.strip() else ""
    res["input_gz_single_bytes"] = os.path.getsize(gz1)
    res["input_gz_single_level"] = a.single_level
    # outputs at cutadapt's default level 5 (libdeflate members) and at -Z (Huffman-only)
    fused = [("fused_plain", plain), ("fused_plain_Z", plain), ("fused_gz_members_Z", gz),
             ("fused_gz_single", gz1), ("fused_gz_single_Z", gz1)]
    if os.environ.get("DMX_E2E_SEQ_A_B") == "1":   # the same file through zlib's sequential path
        fused.append(("fused_gz_single_Z_seq_inflate", gz1))
    if a.reorient:   # 01 -> 02: the two scripts vs the fused pass, on the raw single member
        ro = os.path.join(wd, "reorient")
        os.makedirs(ro, exist_ok=True)
        chop_cmd = [os.path.join(PKG, "bin", "pychopper"), "-b", chop.PRIMERS_FASTA,
                    "-c", chop.CONFIG_FILE, "-k", "LSK114", "-Q", "10",
                    "-w", f"{ro}/rescued.fastq", "-u", f"{ro}/unclass.fastq",
                    "-l", f"{ro}/short.fastq", "-S", f"{ro}/stats.out", "-p", "-t",
                    str(a.threads), "-m", "edlib", gz1]
        t = time.perf_counter()
        with open(f"{ro}/pychopped_pass.fastq", "wb") as fh:
            subprocess.run(chop_cmd, check=True, stdout=fh, stderr=subprocess.DEVNULL, env=env)
        t_chop = time.perf_counter() - t
        subprocess.run([os.path.join(PKG, "bin", "dmx-demux-loop"), f"{ro}/pychopped_pass.fastq",
                        "-j", str(a.threads), "--outdir", f"{ro}/demuxed_two_step"], check=True,
                       env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        t_two = time.perf_counter() - t
        t = time.perf_counter()
        p = subprocess.run([os.path.join(PKG, "bin", "dmx-demux-loop"), gz1, "--reorient",
                            "--pychopper-dir", f"{ro}/fused_pychopped", "-j", str(a.threads),
                            "--outdir", f"{ro}/demuxed_fused"], check=True,
                           env=dict(env, DMX_PROFILE_IO="1"), stdout=subprocess.DEVNULL,
                           stderr=subprocess.PIPE, text=True)
        t_fused = time.perf_counter() - t
        res.update({"reorient_two_step_s": round(t_two, 3),
                    "reorient_two_step_pychopper_s": round(t_chop, 3),
                    "reorient_fused_s": round(t_fused, 3),
                    "reorient_fused_reads_per_s": round(a.reads / t_fused, 1),
                    "reorient_fused_profile": (p.stderr.strip().splitlines()[-1]
                                               if p.stderr.strip() else "")})
    for tag, path in (() if a.skip_fused else fused):
        t = time.perf_counter()
        fenv = dict(env, DMX_PROFILE_IO="1")
        if tag.endswith("_seq_inflate"):
            fenv["DMX_SEQ_INFLATE"] = "1"
        zflag = ["-Z"] if "_Z" in tag else []
        p = subprocess.run([os.path.join(PKG, "bin", "dmx-demux-loop"), path, "-j",
                            str(a.threads), "--outdir", os.path.join(wd, tag)] + zflag, check=True,
                           env=fenv, stdout=subprocess.DEVNULL,
                           stderr=subprocess.PIPE, text=True)
        fs = time.perf_counter() - t
        res[f"{tag}_s"] = round(fs, 3)
        res[f"{tag}_reads_per_s"] = round(a.reads / fs, 1)
        res[f"{tag}_profile"] = p.stderr.strip().splitlines()[-1] if p.stderr.strip() else ""
    os.remove(plain)

    if not a.skip_calls:
        out = os.path.join(wd, "calls")
        os.makedirs(f"{out}/SP5", exist_ok=True)
        os.makedirs(f"{out}/SP27", exist_ok=True)
        cli = os.path.join(PKG, "bin", "cutadapt")
        j = str(a.threads)
        # the drop-in's default: calls served by the resident server (dmx/daemon.py); set
        # DMX_DAEMON=0 to time one process per call
        penv = dict(env, DMX_PROFILE_CLI="1")
        per_call = []

        def call(cmd):
            t1 = time.perf_counter()
            p = subprocess.run(cmd, check=True, env=penv, stdout=subprocess.DEVNULL,
                               stderr=subprocess.PIPE, text=True)
            prof = [ln for ln in p.stderr.splitlines() if ln.startswith("dmx cli phases")]
            per_call.append({"s": round(time.perf_counter() - t1, 3),
                             "phases": prof[-1][len("dmx cli phases: "):] if prof else ""})

        t = time.perf_counter()
        call([cli, "--action=trim", "-e", "0.1", "-j", j, "--rc",
              "-g", f"file:{panel.SP5_FASTA}", "-o", f"{out}/SP5/{{name}}_e2e.fastq.gz",
              gz1 if a.calls_input == "single" else gz,
              f"--json={out}/SP5/cutadapt_SP5_e2e.json"])
        res["calls_input"] = a.calls_input
        ids = sorted(os.path.basename(f)[:-len("_e2e.fastq.gz")]
                     for f in glob.glob(f"{out}/SP5/*_e2e.fastq.gz") if "unknown" not in f)
        for ident in ids:
            call([cli, "--action=trim", "-e", "0.1", "-j", j, "--rc",
                  "-a", f"file:{panel.SP27RC_FASTA}",
                  "-o", f"{out}/SP27/{{name}}_{ident}_e2e.fastq.gz",
                  f"{out}/SP5/{ident}_e2e.fastq.gz",
                  f"--json={out}/SP27/{ident}_e2e.json"])
        cs = time.perf_counter() - t
        res["calls_s"] = round(cs, 3)
        res["calls_reads_per_s"] = round(a.reads / cs, 1)
        res["calls_per_call"] = per_call
        res["calls_server"] = penv.get("DMX_DAEMON", "1") != "0"
        t1 = time.perf_counter()
        subprocess.run([sys.executable, "-c", "import numpy"], check=True)
        res["python_numpy_start_s"] = round(time.perf_counter() - t1, 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
