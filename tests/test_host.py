"""Host-side logic without a GPU: the C-ABI library loads and exports every declared symbol,
the packer's layout, panel parsing, synthetic generator determinism."""
import re
import subprocess

import numpy as np
import pytest

from dmx import lib, panel, synth

ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__file__))


def test_library_exports_every_declared_symbol():
    hdr = open(f"{ROOT}/include/dmx.h").read()
    declared = set(re.findall(r"^\s*(?:int|void|const char\*|size_t)\s+(dmx_\w+)\(", hdr, re.M))
    assert declared == set(lib.EXPORTS)
    out = subprocess.run(["nm", "-D", "--defined-only", lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (dmx_\w+)", out))
    assert declared <= exported
    L = lib.load()
    assert L.dmx_abi_version() == 4


def _unpack(p: lib.Packed, i: int) -> str:
    off, n = int(p.offsets[i]), int(p.lengths[i])
    out = []
    for x in range(off, off + n):
        code = (int(p.seq2b[x // 16]) >> (2 * (x % 16))) & 3
        nb = (int(p.nmask[x // 32]) >> (x % 32)) & 1
        out.append("N" if nb else "ACGT"[code])
    return "".join(out)


def test_pack_layout_roundtrip():
    rng = np.random.default_rng(0)
    seqs = ["", "A", "acgtN", "".join(rng.choice(list("ACGTNRY"), 1000))] + \
           ["".join(rng.choice(list("ACGT"), int(rng.integers(0, 300)))) for _ in range(50)]
    blob = np.frombuffer("".join(seqs).encode(), dtype=np.uint8)
    lens = np.array([len(s) for s in seqs], dtype=np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.uint64)
    p = lib.pack(blob, offs, lens)
    assert p.offsets[0] == lib.PACK_PAD and all(o % 32 == 0 for o in p.offsets)
    for i, s in enumerate(seqs):
        exp = "".join(c if c in "ACGT" else "N" for c in s.upper())
        assert _unpack(p, i) == exp


def test_fasta_panels_match_survey_facts():
    n5, s5 = panel.load_panel(panel.SP5_FASTA)
    n27, s27 = panel.load_panel(panel.SP27RC_FASTA)
    assert len(s5) == 12 and {len(s) for s in s5} == {59}
    assert len(s27) == 12 and {len(s) for s in s27} == {57}
    assert n5[0] == "SP5_001" and n27[11] == "SP27_012"
    assert all(s.startswith("CATGTAATGCACGTACTTTCAGGGT") for s in s5)
    assert all(s.endswith("AGTCGTCGCAGCCTCACCTGATC") for s in s27)


def test_fasta_blank_lines_and_iupac():
    recs = panel.read_fasta(panel.RNA_FASTA)
    assert [h.split("|")[0] for h, _ in recs] == ["SSU_F04", "28S_3RC", "F63.2", "R3264.2"]
    assert recs[1][1] == "TTTTGGTAAGCAGAACTGGYG"


def test_adapter_specs():
    st = panel.AdapterSet()
    st.add_spec("file:" + panel.SP5_FASTA, "front")
    st.add_spec("ACGTu", "back")
    st.add_spec("TNTC...GGAA", "front")
    assert len(st.adapters) == 14
    assert st.adapters[12].name == "1" and st.adapters[12].seq == "ACGTT"
    assert isinstance(st.adapters[13], panel.LinkedAdapter) and st.adapters[13].name == "2"
    with pytest.raises(ValueError):
        panel.normalize("ACGZ")


def test_synth_deterministic_and_shardable():
    a = synth.generate("c2", n=300)
    b = synth.generate("c2", n=100, first=200)
    sa, sb = synth.to_strings(a), synth.to_strings(b)
    assert sa[200:] == sb
    assert np.array_equal(a["truth"][200:], b["truth"])


def test_synthetic_24_panel_distance():
    n1, s1, n2, s2 = synth.panels(24, 24)
    assert len(set(s1)) == 24 and len(set(s2)) == 24
    assert s1[:12] == panel.load_panel(panel.SP5_FASTA)[1]
    assert all(s.startswith(s1[0][:25]) and s.endswith(s1[0][42:]) for s in s1)


def test_primer_pairs_follow_04_header_convention(tmp_path):
    """scripts/04_cleaning_primers.sh:184-270: pair ids `_X` from Forward/Reverse headers; one
    reverse primer may serve several pairs; incomplete pairs are dropped."""
    import os
    coi = panel.primer_pairs(os.path.join(os.path.dirname(panel.SP5_FASTA), "COI_primers.fa"))
    assert [p[0] for p in coi] == ["A", "B"]
    assert coi[0][2] == coi[1][2] == "TGRTTYTTYGGNCAYCCNGNRGTNTA"
    f = tmp_path / "p.fa"
    f.write_text(">x|Forward_A\nACGT\nACGT\n\n>y|Forward_C\nGGGG\n>z|Reverse_A_C_D\nTTTT\n"
                 ">w|Forward_A\nCCCCAAAA\n")
    assert panel.primer_pairs(str(f)) == [("A", "CCCCAAAA", "TTTT"), ("C", "GGGG", "TTTT")]


def test_synth_config5_linked_shape():
    d = synth.generate("c5", n=2000)
    t = d["truth"]
    miss = (t[:, 0] < 0) | (t[:, 1] < 0)
    assert 0.05 < miss.mean() < 0.16                 # one primer missing in ~10%
    assert ((t[:, 0] == t[:, 1]) | miss).all()       # linked: the same pair at both ends
    assert set(np.unique(t[~miss, 0])) <= {0, 1}
    assert 300 < d["lengths"].mean() < 800
    e = synth.generate("c5", n=100, first=1900)
    assert (e["lengths"] == d["lengths"][1900:]).all()


def test_loop_dataset_name_and_device_spec(monkeypatch):
    """02_cutadapt_loop.sh:26-35 dataset naming; DMX_GPUS / DMX_DEVICE parsing (no GPU use)."""
    from dmx import cli, loop
    assert loop.dataset_name("/d/pychopped/pychopped_s1_pass.fastq.gz") == "s1"
    assert loop.dataset_name("x/run7.fq") == "run7"
    args = cli.build_parser().parse_args(["-g", "ACGT", "-o", "o.fq", "in.fq"])
    monkeypatch.setenv("DMX_GPUS", "0,2,5")
    assert cli._devices(args) == [0, 2, 5]
    monkeypatch.setenv("DMX_GPUS", "3")
    assert cli._devices(args) == [0, 1, 2]
    monkeypatch.delenv("DMX_GPUS")
    monkeypatch.setenv("DMX_DEVICE", "4")
    assert cli._devices(args) == [4]
    args.device = 1
    assert cli._devices(args) == [1]


def test_loop_composite_coordinates_match_two_calls():
    """plan_rounds: the fused coordinates equal applying round 1 then round 2 as two separate
    cutadapt calls would (orientation algebra checked on explicit strings)."""
    from dmx import fastx, loop
    rng = np.random.default_rng(9)
    n = 400
    seqs = ["".join(rng.choice(list("ACGT"), int(rng.integers(5, 60)))) for _ in range(n)]
    lens = np.array([len(s) for s in seqs], np.uint32)
    res = np.zeros(n, lib.RESULT_DTYPE)
    res["rc1"] = rng.integers(0, 2, n)
    res["rc2"] = rng.integers(0, 2, n)
    res["m1_rstop"] = [int(rng.integers(0, L + 1)) for L in lens]
    res["m2_rstart"] = [int(rng.integers(0, L - s + 1)) for L, s in zip(lens, res["m1_rstop"])]
    _, (s2, e2, o2, nrc) = loop.plan_rounds(res, lens)
    for i, s in enumerate(seqs):
        t1 = (fastx.revcomp(s.encode()) if res["rc1"][i] else s.encode())[res["m1_rstop"][i]:]
        t2 = (fastx.revcomp(t1) if res["rc2"][i] else t1)[:res["m2_rstart"][i]]
        full = fastx.revcomp(s.encode()) if o2[i] else s.encode()
        assert full[s2[i]:e2[i]] == t2
        assert nrc[i] == res["rc1"][i] + res["rc2"][i]


def test_mask_exceptions_match_dense_mask():
    """dmx_mask_exceptions lists exactly the nonzero no-match words, in order (the sparse upload
    of dmx_run_sparse); single- and multi-threaded ranges."""
    for n, nfrac in ((300, 0.01), (40000, 0.002)):
        d = synth.generate("c2", n=n, seed=7)
        blob = d["blob"].copy()
        rng = np.random.default_rng(n)
        hit = rng.random(len(blob)) < nfrac
        blob[hit] = ord("N")
        p = lib.pack(blob, d["offsets"], d["lengths"])
        idx, val = p.exceptions()
        nmw = min(p.n_words, (p.n_words + 1) // 2 + 2)
        nz = np.nonzero(p.nmask[:nmw])[0]
        assert idx.tolist() == nz.tolist()
        assert val.tolist() == p.nmask[nz].tolist()
        assert len(idx) > 0
