"""The drop-in CLI replaying scripts/02_cutadapt_loop.sh's command sequence on the GPU; every
output file is compared record-for-record with outputs rendered from the oracle."""
import glob
import json
import os
import subprocess

import numpy as np
import pytest

import oracle
from dmx import panel, synth
from helpers import (CLI, LOOP, amplicon_reads, instantiate, oracle_linked, oracle_round,
                     random_quals, read_fastq,
                     write_fastq)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("server", ["0", "1"])
def test_02_cutadapt_loop_dropin(tmp_path, server):
    """The unchanged script's 13 calls, each in its own process (server "0") or through the
    resident server bin/cutadapt starts (dmx/daemon.py, "1"): identical files either way."""
    d = synth.generate("c2", n=3000, seed=12)
    seqs = synth.to_strings(d)
    rng = np.random.default_rng(3)
    names = [f"read{i} runid=abc ch={i % 512}" for i in range(len(seqs))]
    quals = random_quals(rng, [len(s) for s in seqs])
    ds = "sample1"
    pych = tmp_path / "pychopped"
    pych.mkdir()
    infile = str(pych / f"pychopped_{ds}.fastq.gz")
    write_fastq(infile, names, seqs, quals)
    out = tmp_path / "demuxed"
    (out / "SP5").mkdir(parents=True)
    (out / "SP27").mkdir()
    env = dict(os.environ, DMX_DAEMON=server, DMX_DAEMON_IDLE="5",
               DMX_DAEMON_SOCK=str(tmp_path / "dmx.sock"))
    # round 1 (02_cutadapt_loop.sh:64-72)
    subprocess.run([CLI, "--action=trim", "-e", "0.1", "-j", "4", "--rc",
                    "-g", f"file:{panel.SP5_FASTA}", "-o", f"{out}/SP5/{{name}}_{ds}.fastq.gz",
                    infile, f"--json={out}/SP5/cutadapt_SP5_{ds}.json"], check=True, env=env,
                   stdout=subprocess.DEVNULL)
    suffix = f"_{ds}.fastq.gz"
    ids = sorted(os.path.basename(f)[:-len(suffix)] for f in glob.glob(f"{out}/SP5/*{suffix}")
                 if "unknown" not in f)
    # round 2 (02_cutadapt_loop.sh:91-103)
    for ident in ids:
        subprocess.run([CLI, "--action=trim", "-e", "0.1", "-j", "4", "--rc",
                        "-a", f"file:{panel.SP27RC_FASTA}",
                        "-o", f"{out}/SP27/{{name}}_{ident}_{ds}.fastq.gz",
                        f"{out}/SP5/{ident}_{ds}.fastq.gz", f"--json={out}/SP27/{ident}_{ds}.json"],
                       check=True, env=env, stdout=subprocess.DEVNULL)

    n5, s5 = panel.load_panel(panel.SP5_FASTA)
    n27, s27 = panel.load_panel(panel.SP27RC_FASTA)
    assert ids == n5    # every SP5 output exists (created even if empty)
    records = [("@" + n, s, q) for n, s, q in zip(names, seqs, quals)]
    exp1 = oracle_round(records, s5, oracle.FRONT, True)
    got_unknown = read_fastq(f"{out}/SP5/unknown{suffix}")
    assert got_unknown == [(("@" + n), s, q) for n, s, q in exp1.get(-1, [])]
    total2 = 0
    for a, ident in enumerate(n5):
        exp_bin = exp1.get(a, [])
        got_bin = read_fastq(f"{out}/SP5/{ident}{suffix}")
        assert got_bin == [("@" + n, s, q) for n, s, q in exp_bin], ident
        exp2 = oracle_round([("@" + n, s, q) for n, s, q in exp_bin], s27, oracle.BACK, True)
        for b, name27 in enumerate(n27):
            got = read_fastq(f"{out}/SP27/{name27}_{ident}{suffix}")
            assert got == [("@" + n, s, q) for n, s, q in exp2.get(b, [])], (ident, name27)
            total2 += len(got)
    assert total2 > 0.6 * len(seqs)
    rep = json.load(open(f"{out}/SP5/cutadapt_SP5_{ds}.json"))
    assert rep["read_counts"]["input"] == len(seqs)
    assert rep["read_counts"]["read1_with_adapter"] == sum(len(v) for k, v in exp1.items()
                                                          if k >= 0)
    assert [a["name"] for a in rep["adapters_read1"]] == n5

    # the fused driver (one pass, DMX_MODE_TWO_ROUND) writes the same files and reports
    fused = tmp_path / "fused"
    subprocess.run([LOOP, infile, "-j", "4", "--outdir", str(fused), "--no-cleanup"],
                   check=True, stdout=subprocess.DEVNULL)
    per_call = sorted(os.path.relpath(f, out) for f in glob.glob(f"{out}/*/*"))
    assert sorted(os.path.relpath(f, fused) for f in glob.glob(f"{fused}/*/*")) == per_call
    for rel in per_call:
        if rel.endswith(".json"):
            a, b = json.load(open(f"{out}/{rel}")), json.load(open(f"{fused}/{rel}"))
            for key in ("read_counts", "basepair_counts", "adapters_read1"):
                assert a[key] == b[key], (rel, key)
        else:
            assert read_fastq(f"{out}/{rel}") == read_fastq(f"{fused}/{rel}"), rel
    # default: the files 02_cutadapt_loop.sh keeps after its cleanup (:107-119)
    clean = tmp_path / "clean"
    subprocess.run([LOOP, infile, "--outdir", str(clean)], check=True, stdout=subprocess.DEVNULL)
    kept = sorted(os.path.relpath(f, clean) for f in glob.glob(f"{clean}/*/*"))
    assert kept == sorted(r for r in per_call if "unknown" not in r and
                          not any(f"SP27_0{k}" in r for k in ("09", "10", "11", "12")))


def test_cli_multi_gpu_sharding_keeps_order(tmp_path):
    """DMX_GPUS shards each batch over several contexts (here several contexts on one GPU);
    outputs and report equal the single-context run."""
    d = synth.generate("c2", n=4000, seed=21)
    seqs = synth.to_strings(d)
    rng = np.random.default_rng(4)
    names = [f"r{i}" for i in range(len(seqs))]
    write_fastq(str(tmp_path / "in.fastq"), names, seqs, random_quals(rng, map(len, seqs)))
    outs = {}
    for tag, gpus in (("one", "1"), ("three", "0,0,0")):
        od = tmp_path / tag
        od.mkdir()
        env = dict(os.environ, DMX_GPUS=gpus)
        subprocess.run([CLI, "-e", "0.1", "-j", "3", "--rc", "-g", f"file:{panel.SP5_FASTA}",
                        "-o", f"{od}/{{name}}.fastq.gz", str(tmp_path / "in.fastq"),
                        f"--json={od}/r.json", "--batch-mb", "1"], check=True, env=env,
                       stdout=subprocess.DEVNULL)
        outs[tag] = {os.path.basename(f): read_fastq(f) for f in glob.glob(f"{od}/*.fastq.gz")}
        outs[tag]["json"] = json.load(open(f"{od}/r.json"))["adapters_read1"]
    assert outs["one"] == outs["three"]
    assert sum(len(v) for k, v in outs["one"].items() if k != "json") == len(seqs)


def _read_fasta(path):
    recs = panel.read_fasta(path)
    return [(h, s, None) for h, s in recs]


def test_04_linked_primers_dropin(tmp_path):
    """scripts/04_cleaning_primers.sh:371-393: one call with every linked pair, FASTA in/out,
    --untrimmed-output; trimmed and untrimmed files equal the oracle's, record for record."""
    pairs = panel.primer_pairs(os.path.join(os.path.dirname(panel.SP5_FASTA), "COI_primers.fa"))
    rng = np.random.default_rng(8)
    seqs = amplicon_reads(rng, [(f, r) for _, f, r in pairs], 2500)
    infile = tmp_path / "consensus.fasta"
    names = [f"cluster{i};size={int(rng.integers(2, 90))}" for i in range(len(seqs))]
    infile.write_text("".join(f">{n}\n{s}\n" for n, s in zip(names, seqs)))
    out = tmp_path / "round1_amplicon.fasta"
    unt = tmp_path / "untrimmed_round1.fasta"
    cmd = [CLI, "-j", "4"]
    for _, f, r in pairs:
        cmd += ["-g", f"{f}...{r}"]
    cmd += [f"--untrimmed-output={unt}", "-o", str(out), str(infile)]
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL)
    trimmed, untrimmed = oracle_linked([(n, s, None) for n, s in zip(names, seqs)],
                                       [(f, r) for _, f, r in pairs])
    assert len(trimmed) > 0.6 * len(seqs) and len(untrimmed) > 0
    assert _read_fasta(str(out)) == trimmed
    assert _read_fasta(str(unt)) == untrimmed


def test_unverified_rule_cases_match_the_oracle(tmp_path):
    """The cases tools/parity_vs_cutadapt.sh runs against a real cutadapt 4.9 for every rule the
    oracle marks [UNVERIFIED] (tools/unverified_cases.py): the drop-in's outputs equal the
    restatement's (oracle/pyref.py, default readings) record for record."""
    import importlib.util
    import pyref
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location(
        "unverified_cases", os.path.join(root, "tools", "unverified_cases.py"))
    uc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(uc)
    cases = tmp_path / "cases"
    uc.write(str(cases))
    out = tmp_path / "out"
    out.mkdir()
    env = dict(os.environ, DMX_DAEMON="0")
    for c in uc.CASES:
        row = [r for r in open(cases / "cases.tsv").read().splitlines()
               if r.split("\t")[0] == c["name"]][0]
        _, inp, outs, opts = row.split("\t")
        subprocess.run([CLI] + opts.split() + outs.replace("@OUT@", str(out)).split() + [inp],
                       check=True, env=env, cwd=str(cases), stdout=subprocess.DEVNULL)
        name = c["name"]
        if c["where"] == "linked":
            f, r = c["adapters"][0][1].split("...")
            trimmed, untrimmed = [], []
            for i, s in enumerate(c["reads"]):
                a, _, _, tr = pyref.linked([f], [r], s, c["e"])
                (trimmed if a >= 0 else untrimmed).append((f"{name}{i}", tr, None))
            assert _read_fasta(str(out / f"{name}.fasta")) == trimmed, name
            assert _read_fasta(str(out / f"{name}_untrimmed.fasta")) == untrimmed, name
            continue
        seqs = [x for _, x in c["adapters"]]
        w = [pyref.BACK if c["where"] == "back" else pyref.FRONT] * len(seqs)
        per, ordered = {}, []
        for i, s in enumerate(c["reads"]):
            a, rc, _, tr = pyref.demux_round(seqs, w, s, c["rc"], c["e"], c["O"])
            rec = (f"@{name}{i}" + (" rc" if rc else ""), tr, "I" * len(tr))
            per.setdefault(a, []).append(rec)
            ordered.append(rec)
        if len(seqs) == 1:   # trimmed and untrimmed reads share the one output
            assert read_fastq(str(out / f"{name}.fastq")) == ordered, name
        else:
            for k, (an, _) in enumerate(c["adapters"]):
                assert read_fastq(str(out / f"{name}_{an}.fastq")) == per.get(k, []), (name, an)
            assert read_fastq(str(out / f"{name}_unknown.fastq")) == per.get(-1, []), name


def test_04_unlinked_round2_dropin(tmp_path):
    """scripts/04_cleaning_primers.sh:464-507 (--run-round2): one call on round 1's untrimmed
    consensuses with every round-1 pair as UNLINKED primers, `-g FWD -a REV` per pair in pair
    order (the reference's COI and rRNA primer files, literal IUPAC primers), default -e, no
    --rc, no --untrimmed-output and no {name}: every record, trimmed or not, goes to -o in
    input order (FASTA in, FASTA out).  Records equal the oracle's (one mixed FRONT / BACK
    panel: best_match over the adapters in command-line order; -g keeps seq[rstop:], -a keeps
    seq[:rstart])."""
    data = os.path.dirname(panel.SP5_FASTA)
    pairs = (panel.primer_pairs(os.path.join(data, "COI_primers.fa")) +
             panel.primer_pairs(os.path.join(data, "RNA_primers.fa")))
    assert len(pairs) == 4
    rng = np.random.default_rng(507)
    # round 1's untrimmed records: one primer of a pair, damaged copies, or none
    seqs = []
    for _ in range(3000):
        _, f, r = pairs[int(rng.integers(len(pairs)))]
        body = "".join(rng.choice(list("ACGT"), size=int(rng.integers(60, 900))))
        u = rng.random()
        if u < 0.4:
            s = instantiate(rng, f) + body
        elif u < 0.75:
            s = body + instantiate(rng, r)
        elif u < 0.85:
            s = instantiate(rng, f)[int(rng.integers(1, 8)):] + body   # partial at the start
        else:
            s = body
        flank = "".join(rng.choice(list("ACGT"), size=int(rng.integers(0, 30))))
        seqs.append(flank + s)
    names = [f"cluster{i};size={int(rng.integers(2, 90))}" for i in range(len(seqs))]
    infile = tmp_path / "untrimmed_round1.fasta"
    infile.write_text("".join(f">{n}\n{s}\n" for n, s in zip(names, seqs)))
    out = tmp_path / "round2_primerless.fasta"
    cmd = [CLI, "-j", "4"]
    adapters, wheres = [], []
    for _, f, r in pairs:
        cmd += ["-g", f, "-a", r]
        adapters += [f, r]
        wheres += [oracle.FRONT, oracle.BACK]
    cmd += ["-o", str(out), str(infile)]
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL)
    blob, offs, lens = oracle.pack_ascii(seqs)
    res = oracle.run_batch(oracle.Panel(adapters, wheres), None, blob, offs, lens, mode=0,
                           use_rc=False, threads=8)
    exp = []
    for n, s, r in zip(names, seqs, res):
        b = int(r["bin1"])
        if b < 0:
            exp.append((n, s, None))
        elif wheres[b] == oracle.FRONT:
            exp.append((n, s[int(r["m1_rstop"]):], None))
        else:
            exp.append((n, s[:int(r["m1_rstart"])], None))
    n_front = sum(1 for r in res if r["bin1"] >= 0 and wheres[int(r["bin1"])] == oracle.FRONT)
    n_back = sum(1 for r in res if r["bin1"] >= 0 and wheres[int(r["bin1"])] == oracle.BACK)
    assert n_front > 500 and n_back > 500 and sum(res["bin1"] < 0) > 100
    assert _read_fasta(str(out)) == exp


def test_loop_two_name_template(tmp_path):
    """dmx-demux-loop --template: the two-name layout of north_star ({name1}_{name2}), also with
    a directory per SP5 bin and plain text, writes the same records per (SP5, SP27) bin as the
    script's default names (02_cutadapt_loop.sh:100)."""
    d = synth.generate("c2", n=2500, seed=77)
    seqs = synth.to_strings(d)
    rng = np.random.default_rng(77)
    names = [f"r{i}" for i in range(len(seqs))]
    infile = tmp_path / "pychopped" / "pychopped_ds7.fastq"
    infile.parent.mkdir()
    write_fastq(str(infile), names, seqs, random_quals(rng, map(len, seqs)))
    n5, _ = panel.load_panel(panel.SP5_FASTA)
    n27, _ = panel.load_panel(panel.SP27RC_FASTA)
    runs = {}
    for tag, tmpl in (("default", None), ("n1n2", "{name1}_{name2}.fastq.gz"),
                      ("dirs", "{name1}/{name2}_{ds}.fastq")):
        od = tmp_path / tag
        cmd = [LOOP, str(infile), "-j", "4", "--outdir", str(od)]
        if tmpl:
            cmd += ["--template", tmpl]
        subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL)
        runs[tag] = od
    kept = [b for b in n27 if b not in ("SP27_009", "SP27_010", "SP27_011", "SP27_012")]
    total = 0
    for a in n5:
        for b in kept:
            ref = read_fastq(f"{runs['default']}/SP27/{b}_{a}_ds7.fastq.gz")
            assert read_fastq(f"{runs['n1n2']}/SP27/{a}_{b}.fastq.gz") == ref, (a, b)
            assert read_fastq(f"{runs['dirs']}/SP27/{a}/{b}_ds7.fastq") == ref, (a, b)
            total += len(ref)
    assert total > 0.5 * len(seqs)
    # same file set otherwise: no default-named round-2 file in the templated runs
    assert not glob.glob(f"{runs['n1n2']}/SP27/SP27_*_SP5_*")


def test_large_single_member_input_parallel_io_equals_sequential(tmp_path):
    """A ~60 MB single-member .gz round-1 input (02_cutadapt_loop.sh:64-72) through the parallel
    I/O paths (speculative inflate with rounds sized to the read-ahead block, parallel preads
    and block copies, record-aware level-5 members on 8 threads) gives the same records and
    report counts as the sequential paths (DMX_SEQ_INFLATE=1, -j 1, 4 MB batches)."""
    import zlib
    d = synth.generate("c2", n=25000, seed=21)
    seqs = synth.to_strings(d)
    rng = np.random.default_rng(5)
    names = [f"r{i} runid=abc ch={i % 512}" for i in range(len(seqs))]
    quals = random_quals(rng, [len(s) for s in seqs])
    text = "".join(f"@{n}\n{s}\n+\n{q}\n" for n, s, q in zip(names, seqs, quals)).encode()
    infile = str(tmp_path / "pychopped_big.fastq.gz")
    c = zlib.compressobj(1, zlib.DEFLATED, 31)
    with open(infile, "wb") as fh:
        fh.write(c.compress(text) + c.flush())
    outs = {}
    for tag, extra, env_add in (("par", ["-j", "8"], {}),
                                ("seq", ["-j", "1"], {"DMX_SEQ_INFLATE": "1",
                                                      "DMX_BATCH_MB": "4"})):
        od = tmp_path / tag
        od.mkdir()
        env = dict(os.environ, DMX_DAEMON="0", **env_add)
        subprocess.run([CLI, "--action=trim", "-e", "0.1", "--rc", *extra,
                        "-g", f"file:{panel.SP5_FASTA}", "-o", f"{od}/{{name}}_big.fastq.gz",
                        infile, f"--json={od}/report.json"], check=True, env=env,
                       stdout=subprocess.DEVNULL)
        files = sorted(os.path.basename(f) for f in glob.glob(f"{od}/*_big.fastq.gz"))
        outs[tag] = ({f: read_fastq(f"{od}/{f}") for f in files},
                     json.load(open(f"{od}/report.json"))["read_counts"])
    assert outs["par"][0] == outs["seq"][0]
    assert outs["par"][1] == outs["seq"][1]
    assert sum(len(v) for v in outs["par"][0].values()) == len(seqs)


def test_fused_reorient_under_a_memory_budget_equals_unbudgeted(tmp_path):
    """dmx-demux-loop --reorient (01 -> 02 fused) under DMX_MEM_BUDGET_MB=1400 (32 MB batches,
    256 KiB inflate chunks, small read-ahead blocks and buffer pools; nio.batch_bytes_for_budget,
    dmx_io_set_memory_budget) writes the same pychopper and demultiplexed records as without a
    budget, from an ordinary single-member .gz of raw (unoriented) reads."""
    import zlib
    d = synth.generate("c2", n=20000, seed=23)
    seqs = synth.to_strings(d)
    rng = np.random.default_rng(23)
    flip = rng.random(len(seqs)) < 0.5     # raw reads: either orientation
    comp = str.maketrans("ACGTN", "TGCAN")
    seqs = [s.translate(comp)[::-1] if f else s for s, f in zip(seqs, flip)]
    names = [f"r{i} runid=abc ch={i % 512}" for i in range(len(seqs))]
    quals = random_quals(rng, [len(s) for s in seqs])
    text = "".join(f"@{n}\n{s}\n+\n{q}\n" for n, s, q in zip(names, seqs, quals)).encode()
    raw = tmp_path / "raw.fastq.gz"
    c = zlib.compressobj(1, zlib.DEFLATED, 31)
    raw.write_bytes(c.compress(text) + c.flush())
    runs = {}
    for tag, env_add in (("free", {}), ("budget", {"DMX_MEM_BUDGET_MB": "1400"})):
        od = tmp_path / tag
        env = dict(os.environ, **env_add)
        env.pop("DMX_BATCH_MB", None)
        subprocess.run([LOOP, str(raw), "--reorient", "--pychopper-dir", str(od / "pych"),
                        "-j", "8", "--outdir", str(od / "demux")], check=True, env=env,
                       stdout=subprocess.DEVNULL)
        runs[tag] = od
    got = {}
    for tag, od in runs.items():
        files = sorted(p.relative_to(od) for p in od.rglob("*") if p.is_file()
                       and (p.name.endswith(".fastq") or p.name.endswith(".fastq.gz")))
        got[tag] = {str(f): read_fastq(str(od / f)) for f in files}
    assert got["free"].keys() == got["budget"].keys() and len(got["free"]) > 10
    for f in got["free"]:
        assert got["free"][f] == got["budget"][f], f
    assert sum(len(v) for k, v in got["free"].items() if "demux" in k) > 0.5 * len(seqs)
