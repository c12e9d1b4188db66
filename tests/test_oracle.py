"""The oracle itself (CPU, no GPU): known-answer tests hand-derived from cutadapt's documented
alignment semantics, and agreement of its two independent formulations (one-column Ukkonen DP
in C vs full-matrix Python).  PARITY UNPINNED: the reference holds no fixtures for this path
(SURVEY.md §4/§8c); the KATs below are chosen so their answer is the same under every
plausible tie rule, except where a test name says `tie_rule`."""
import os
import random

import pytest

import oracle
import pyref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SP5_001 = "CATGTAATGCACGTACTTTCAGGGTGAGCGTCTAATCGTAATTGTAAAACGACGGCCAG"
SP27_001 = "GTCATAGCTGTTTCCTGTTAACCAGGCACGGAGGAGTCGTCGCAGCCTCACCTGATC"
F, B = oracle.FRONT, oracle.BACK


def test_exact_front_match():
    read = "ACGT" + SP5_001 + "TTTTGGGG"
    assert oracle.locate(SP5_001, read, 0.1, F) == (0, 59, 4, 63, 59, 0)


def test_exact_back_match():
    read = "ACGTACGTAA" + SP27_001 + "CC"
    assert oracle.locate(SP27_001, read, 0.1, B) == (0, 57, 10, 67, 57, 0)


def test_partial_front_at_read_start():
    # the read starts inside the adapter: adapter prefix skipped (FRONT only at read start)
    read = SP5_001[40:] + "GATTACAGATTACA"
    r = oracle.locate(SP5_001, read, 0.1, F)
    assert r[:4] == (40, 59, 0, 19) and r[5] == 0


def test_partial_back_at_read_end():
    read = "GATTACAGATTACAGATTACA" + SP27_001[:12]
    r = oracle.locate(SP27_001, read, 0.1, B)
    assert r[:4] == (0, 12, 21, 33) and r[5] == 0


def test_min_overlap():
    assert oracle.locate(SP27_001, "TTTTTTTTTTTTGT", 0.1, B) is None       # 2 < -O 3
    assert oracle.locate(SP27_001, "TTTTTTTTTTTTGTC", 0.1, B)[:4] == (0, 3, 12, 15)


def test_error_threshold_boundary():
    # k = int(0.1 * 59) = 5: five substitutions accepted, six rejected
    def subst(s, n):
        s = list(s)
        for p in range(n):
            i = 3 + 10 * p
            s[i] = "A" if s[i] != "A" else "C"
        return "".join(s)
    assert oracle.locate(SP5_001, "GG" + subst(SP5_001, 5) + "GG", 0.1, F)[5] == 5
    assert oracle.locate(SP5_001, "GG" + subst(SP5_001, 6) + "GG", 0.1, F) is None


def test_n_in_read_never_matches():
    read = SP5_001[:20] + "N" + SP5_001[21:]
    r = oracle.locate(SP5_001, read, 0.1, F)
    assert r[5] == 1 and r[4] == 57


def test_iupac_adapter_wildcards():
    adapter = "TNTCNACNAAYCAYAARGAYATTGG"     # jgLCO1490, COI_primers.fa:2
    inst = "TATCAACAAATCATAAAGATATTGG"
    r = oracle.locate(adapter, "GG" + inst + "CC", 0.1, F)
    assert r == (0, 25, 2, 27, 25, 0)


def test_rc_round_choice():
    p1 = oracle.Panel([SP5_001], F)
    read = pyref.revcomp("AC" + SP5_001 + "TTT")
    blob, offs, lens = oracle.pack_ascii([read])
    res = oracle.run_batch(p1, None, blob, offs, lens, mode=0)
    assert res["bin1"][0] == 0 and res["rc1"][0] == 1 and res["m1_rstop"][0] == 61


def test_tie_rule_forward_wins_equal_score():
    # palindromic-ish: the same adapter matches forward and RC with equal score -> forward
    a = "ACGTACGTTTAAACCC"
    read = a + "G" * 10 + pyref.revcomp(a)
    blob, offs, lens = oracle.pack_ascii([read])
    res = oracle.run_batch(oracle.Panel([a], F), None, blob, offs, lens, mode=0)
    assert res["rc1"][0] == 0


def test_tie_rule_earlier_adapter_wins():
    a1, a2 = "ACGTACGTAAGG", "ACGTACGTAAGG"
    blob, offs, lens = oracle.pack_ascii(["TT" + a1 + "TT"])
    res = oracle.run_batch(oracle.Panel([a1, a2], F), None, blob, offs, lens, mode=0)
    assert res["bin1"][0] == 0


def test_two_round_rc_rc():
    sp5, sp27 = [SP5_001], [SP27_001]
    fwd = "AA" + SP5_001 + "GATTACA" * 20 + SP27_001 + "TT"
    a, rc1, m1, b, rc2, m2, final = pyref.two_round(sp5, sp27, pyref.revcomp(fwd))
    assert (a, rc1, b, rc2) == (0, True, 0, False)
    assert final == "GATTACA" * 20


@pytest.mark.parametrize("seed", range(4))
def test_c_oracle_matches_full_matrix(seed):
    rng = random.Random(seed)
    for _ in range(300):
        ad = "".join(rng.choice("ACGT") for _ in range(rng.randint(3, 40)))
        if rng.random() < 0.3:
            ad = "".join(c if rng.random() > 0.2 else rng.choice("NRY") for c in ad)
        q = "".join(rng.choice("ACGTN") for _ in range(rng.randint(0, 90)))
        if rng.random() < 0.7:
            frag = "".join(c if rng.random() > 0.1 else rng.choice("ACGT")
                           for c in ad.replace("N", "A").replace("R", "G").replace("Y", "C"))
            p = rng.randint(0, len(q))
            q = q[:p] + frag + q[p:]
        for where in (F, B):
            e = rng.choice([0.1, 0.2, 0.3])
            assert oracle.locate(ad, q, e, where) == pyref.locate(ad, q, e, where)


def test_two_round_batch_equals_composition():
    """orc_two_round == round 1, then round 2 on the round-1 output (what 02 runs as 13 calls)."""
    from dmx import synth
    d = synth.generate("c1", n=200)
    p1, p2 = oracle.Panel(d["sp5"], F), oracle.Panel(d["sp27"], B)
    fused = oracle.run_batch(p1, p2, d["blob"], d["offsets"], d["lengths"], mode=1)
    seqs = synth.to_strings(d)
    for i, s in enumerate(seqs[:60]):
        a, rc1, m1, b, rc2, m2, _ = pyref.two_round(d["sp5"], d["sp27"], s)
        assert fused["bin1"][i] == a and fused["bin2"][i] == (b if a >= 0 else -1)
        if a >= 0:
            assert fused["m1_rstop"][i] == m1[3] and fused["m1_score"][i] == m1[4]
        if a >= 0 and b >= 0:
            assert fused["m2_rstart"][i] == m2[2] and fused["m2_errors"][i] == m2[5]


def test_linked_c_oracle_equals_full_matrix():
    """orc_linked (C) == pyref.linked (full-matrix restatement of LinkedAdapter.match_to)."""
    import os
    import numpy as np
    from dmx import panel
    from helpers import amplicon_reads
    pairs = [(f, r) for _, f, r in panel.primer_pairs(
        os.path.join(os.path.dirname(panel.SP5_FASTA), "COI_primers.fa"))]
    rng = np.random.default_rng(4)
    seqs = amplicon_reads(rng, pairs, 60, body=(20, 150), flank=(0, 12)) + ["", "ACG"]
    blob, offs, lens = oracle.pack_ascii(seqs)
    res = oracle.run_batch(oracle.Panel([p[0] for p in pairs], F),
                           oracle.Panel([p[1] for p in pairs], B), blob, offs, lens, mode=2,
                           use_rc=False)
    hits = 0
    for i, s in enumerate(seqs):
        a, mf, mb, _ = pyref.linked([p[0] for p in pairs], [p[1] for p in pairs], s)
        assert res["bin1"][i] == a and res["bin2"][i] == a
        if a >= 0:
            hits += 1
            assert (res["m1_rstart"][i], res["m1_rstop"][i], res["m1_score"][i],
                    res["m1_errors"][i]) == (mf[2], mf[3], mf[4], mf[5])
            assert (res["m2_rstart"][i], res["m2_rstop"][i], res["m2_score"][i],
                    res["m2_errors"][i]) == (mb[2], mb[3], mb[4], mb[5])
    assert hits > 30


def test_unverified_rule_cases_tell_the_readings_apart():
    """Every [UNVERIFIED] rule of the restatement has a case in tools/unverified_cases.py (run
    against a real cutadapt 4.9 by tools/parity_vs_cutadapt.sh) whose outputs differ between
    the restatement's reading and the alternative one (pyref.rules)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "unverified_cases", os.path.join(ROOT, "tools", "unverified_cases.py"))
    uc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(uc)
    assert {c["rule"] for c in uc.CASES} == set(pyref.DEFAULT_RULES)

    def outputs(c):
        res = []
        for s in c["reads"]:
            if c["where"] == "linked":
                f, r = c["adapters"][0][1].split("...")
                a, _, _, tr = pyref.linked([f], [r], s, c["e"])
                res.append((a, tr))
            else:
                seqs = [x for _, x in c["adapters"]]
                w = [pyref.BACK if c["where"] == "back" else pyref.FRONT] * len(seqs)
                a, rc, _, tr = pyref.demux_round(seqs, w, s, c["rc"], c["e"], c["O"])
                res.append((a, rc, tr))
        return res

    for c in uc.CASES:
        base = outputs(c)
        with pyref.rules(**{c["rule"]: c["alt"]}):
            alt = outputs(c)
        assert base != alt, c["name"]
        assert pyref.RULES == pyref.DEFAULT_RULES
