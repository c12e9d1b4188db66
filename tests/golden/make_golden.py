"""Generate the committed golden fixtures under tests/golden/ (run in the build container).

    python tests/golden/make_golden.py

WHAT THESE ARE.  cutadapt 4.9 (where the reference's arithmetic lives: scripts/02_cutadapt_loop.sh
:64-72,94-102, scripts/04_cleaning_primers.sh:377) is neither vendored in /root/reference nor
installable here, and the reference ships no test, golden vector or fixture for this path
(SURVEY.md §4, §8c).  So these vectors are produced by the repo's two independent CPU
restatements of cutadapt 4.9 — the C oracle (oracle/cutadapt_oracle.c, Ukkonen-banded single
column, literal) and the full-matrix Python restatement (oracle/pyref.py) — and every vector is
written only after the two agree on it.  They freeze the restated semantics (PARITY UNPINNED
against cutadapt itself) so that:
  * tests/test_golden.py (CPU) re-derives them with the oracle (a regression pin on the oracle);
  * tests/test_golden.py (GPU) runs libdmx.so on the same inputs and must reproduce every byte,
    without loading the oracle at all.

The adapter/primer panels are the reference's own data files (adapters_primers/*.fa, copied as
data into nanopore-barcoding-orc_amd/dmx/data/), the 24x24 panel is the synthetic extension of
SURVEY.md §8d, and reads come from dmx.synth (seeded) or from seeded random edge-case builders.

Files: one .npz per batch case (inputs: ASCII blob / offsets / lengths; panel sequences;
per-adapter FRONT/BACK; mode, --rc, -e; expected: n x 40 bytes of dmx_result), and
locate_kats.json (single Aligner.locate calls).  All loadable with allow_pickle=False.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "nanopore-barcoding-orc_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import oracle  # noqa: E402
import pyref  # noqa: E402
from dmx import panel, synth  # noqa: E402

MODE_SINGLE, MODE_TWO_ROUND, MODE_LINKED = 0, 1, 2


def _strings(blob, offs, lens):
    return [blob[int(o):int(o) + int(n)].tobytes().decode("ascii") for o, n in zip(offs, lens)]


def _crosscheck(case, seqs, res, k=None):
    """The full-matrix restatement must agree with the C oracle on (a prefix of) the case."""
    p1, p2, w1 = case["panel1"], case["panel2"], case["where1"]
    e, rc, mode = case["max_errors"], case["use_rc"], case["mode"]
    for i, s in enumerate(seqs[:k]):
        r = res[i]
        if mode == MODE_TWO_ROUND:
            a, rc1, m1, b, rc2, m2, _ = pyref.two_round(p1, p2, s, use_rc=rc, e=e)
            assert int(r["bin1"]) == a, (case["name"], i)
            if a >= 0:
                assert int(r["rc1"]) == int(rc1) and int(r["m1_rstop"]) == m1[3]
                assert int(r["m1_score"]) == m1[4] and int(r["m1_errors"]) == m1[5]
                assert int(r["bin2"]) == b, (case["name"], i)
                if b >= 0:
                    assert int(r["rc2"]) == int(rc2) and int(r["m2_rstart"]) == m2[2]
                    assert int(r["m2_score"]) == m2[4] and int(r["m2_errors"]) == m2[5]
        elif mode == MODE_LINKED:
            a, mf, mb, _ = pyref.linked(p1, p2, s, e=e)
            assert int(r["bin1"]) == a, (case["name"], i)
            if a >= 0:
                assert (int(r["m1_rstart"]), int(r["m1_rstop"]), int(r["m1_score"]),
                        int(r["m1_errors"])) == (mf[2], mf[3], mf[4], mf[5])
                assert (int(r["m2_rstart"]), int(r["m2_rstop"]), int(r["m2_score"]),
                        int(r["m2_errors"])) == (mb[2], mb[3], mb[4], mb[5])
        else:
            a, is_rc, m, _ = pyref.demux_round(p1, list(w1), s, use_rc=rc, e=e)
            assert int(r["bin1"]) == a, (case["name"], i)
            if a >= 0:
                assert int(r["rc1"]) == int(is_rc)
                assert (int(r["m1_rstart"]), int(r["m1_rstop"]), int(r["m1_astart"]),
                        int(r["m1_astop"]), int(r["m1_score"]), int(r["m1_errors"])) == (m[2], m[3], m[0], m[1], m[4], m[5])


def _save(case, blob, offs, lens, crosscheck_n):
    p1 = oracle.Panel(case["panel1"], case["where1"], max_errors=case["max_errors"])
    p2 = (oracle.Panel(case["panel2"], oracle.BACK, max_errors=case["max_errors"])
          if case["panel2"] else None)
    res = oracle.run_batch(p1, p2, blob, offs, lens, mode=case["mode"], use_rc=case["use_rc"],
                           threads=8)
    _crosscheck(case, _strings(blob, offs, lens), res, crosscheck_n)
    path = os.path.join(HERE, case["name"] + ".npz")
    np.savez_compressed(
        path, blob=np.asarray(blob, np.uint8), offsets=np.asarray(offs, np.uint64),
        lengths=np.asarray(lens, np.uint32),
        panel1=np.array(case["panel1"], dtype="U128"),
        panel2=np.array(case["panel2"] or [""], dtype="U128")[:len(case["panel2"] or [])],
        where1=np.array(case["where1"], np.int32), mode=np.int32(case["mode"]),
        use_rc=np.int32(case["use_rc"]), max_errors=np.float64(case["max_errors"]),
        expected=res.view(np.uint8).reshape(len(res), 40))
    hit = int((res["bin1"] >= 0).sum())
    print(f"{case['name']}: {len(lens)} reads, {hit} matched round 1 "
          f"({os.path.getsize(path) // 1024} KiB)")


def _synth_case(name, config, n, seed, e=0.1, crosscheck_n=60):
    d = synth.generate(config, n=n, seed=seed)
    linked = config == "c5"
    case = dict(name=name, panel1=list(d["sp5"]), panel2=list(d["sp27"]),
                where1=[oracle.FRONT] * len(d["sp5"]),
                mode=MODE_LINKED if linked else MODE_TWO_ROUND, use_rc=not linked,
                max_errors=e)
    _save(case, d["blob"], d["offsets"], d["lengths"], crosscheck_n)


def _mutated(rng, a, err):
    out = []
    for c in a:
        c = c if c in "ACGT" else "ACGT"[int(rng.integers(4))]
        r = rng.random()
        if r < err * 0.6:
            out.append("ACGT"[int(rng.integers(4))])
        elif r < err * 0.8:
            pass
        elif r < err:
            out += [c, "ACGT"[int(rng.integers(4))]]
        else:
            out.append(c)
    return "".join(out)


def _random_single_case(name, where, seed, n=300):
    """Random panel (lengths 3..64, IUPAC), reads with N, partial adapters at both ends, empty
    and one-character reads; one round with --rc."""
    rng = np.random.default_rng(seed)
    pan = []
    for _ in range(7):
        L = int(rng.integers(3, 65))
        s = "".join(rng.choice(list("ACGT"), size=L))
        pan.append("".join(c if rng.random() > 0.12 else str(rng.choice(list("NRYSWKMBDHV")))
                           for c in s))
    seqs = ["", "A", "ACG", pan[0][:5].replace("N", "A"), pan[1][-4:].replace("N", "C")]
    while len(seqs) < n:
        s = "".join(rng.choice(list("ACGTN"), size=int(rng.integers(0, 300)),
                               p=[0.249, 0.249, 0.249, 0.249, 0.004]))
        if rng.random() < 0.8:
            frag = _mutated(rng, pan[int(rng.integers(len(pan)))], 0.06)
            if rng.random() < 0.25:
                cut = int(rng.integers(1, max(2, len(frag))))
                frag = frag[cut:] if rng.random() < 0.5 else frag[:cut]
            p = int(rng.integers(0, len(s) + 1))
            s = s[:p] + frag + s[p:]
        if rng.random() < 0.3:
            s = pyref.revcomp(s)
        seqs.append(s)
    blob, offs, lens = oracle.pack_ascii(seqs)
    w = oracle.FRONT if where == "front" else oracle.BACK
    case = dict(name=name, panel1=pan, panel2=None, where1=[w] * len(pan), mode=MODE_SINGLE,
                use_rc=True, max_errors=0.15)
    _save(case, blob, offs, lens, crosscheck_n=n)


def _rna_linked_case(name, seed, n=400):
    from helpers import amplicon_reads
    pairs = [(f, r) for _, f, r in panel.primer_pairs(
        os.path.join(os.path.dirname(panel.SP5_FASTA), "RNA_primers.fa"))]
    rng = np.random.default_rng(seed)
    seqs = amplicon_reads(rng, pairs, n - 4, body=(40, 400), flank=(0, 20)) + [
        "", "ACGT", pairs[0][0].replace("N", "A"), (pairs[0][0] + pairs[0][1]).replace("N", "G")]
    blob, offs, lens = oracle.pack_ascii(seqs)
    case = dict(name=name, panel1=[p[0] for p in pairs], panel2=[p[1] for p in pairs],
                where1=[oracle.FRONT] * len(pairs), mode=MODE_LINKED, use_rc=False,
                max_errors=0.1)
    _save(case, blob, offs, lens, crosscheck_n=n)


def _locate_kats(path, seed=2024, n=400):
    """Single Aligner.locate calls: (adapter, read, FRONT/BACK, rate) -> 6-tuple or null; the C
    oracle and the full-matrix restatement must agree on each."""
    rng = np.random.default_rng(seed)
    _, sp5 = panel.load_panel(panel.SP5_FASTA)
    _, sp27 = panel.load_panel(panel.SP27RC_FASTA)
    cases = []
    # real panel adapters at both ends, partial, internal, absent
    for i in range(24):
        ad = sp5[i % 12] if i < 12 else sp27[i % 12]
        ins = "".join(rng.choice(list("ACGT"), size=int(rng.integers(20, 120))))
        frag = _mutated(rng, ad, 0.05)
        cut = int(rng.integers(3, len(ad)))
        for q in (frag + ins, ins + frag, ins[:10] + frag + ins, frag[cut:] + ins,
                  ins + frag[:cut], ins):
            for where in (oracle.FRONT, oracle.BACK):
                cases.append((ad, q, where, 0.1))
    target = len(cases) + n
    while len(cases) < target:
        L = int(rng.integers(3, 45))
        ad = "".join(rng.choice(list("ACGT"), size=L))
        if rng.random() < 0.3:
            ad = "".join(c if rng.random() > 0.2 else str(rng.choice(list("NRY"))) for c in ad)
        q = "".join(rng.choice(list("ACGTN"), size=int(rng.integers(0, 90))))
        if rng.random() < 0.7:
            frag = _mutated(rng, ad, 0.1)
            p = int(rng.integers(0, len(q) + 1))
            q = q[:p] + frag + q[p:]
        cases.append((ad, q, int(rng.choice([oracle.FRONT, oracle.BACK])),
                      float(rng.choice([0.1, 0.2, 0.3]))))
    out = []
    for ad, q, where, e in cases:
        got = oracle.locate(ad, q, e, where)
        ref = pyref.locate(ad, q, e, where)
        assert got == ref, (ad, q, where, e, got, ref)
        out.append({"adapter": ad, "read": q, "where": "front" if where == oracle.FRONT else
                    "back", "max_error_rate": e, "min_overlap": 3,
                    "expected": list(got) if got is not None else None})
    with open(path, "w") as fh:
        json.dump({"fields": ["ref_start", "ref_stop", "query_start", "query_stop", "score",
                              "errors"], "cases": out}, fh, indent=0)
    print(f"locate_kats.json: {len(out)} cases, "
          f"{sum(c['expected'] is not None for c in out)} matches")


CASES = {
    "locate_kats": lambda: _locate_kats(os.path.join(HERE, "locate_kats.json")),
    "c1_two_round": lambda: _synth_case("c1_two_round", "c1", 400, 1, crosscheck_n=40),
    "c2_two_round": lambda: _synth_case("c2_two_round", "c2", 300, 2, crosscheck_n=20),
    "c2x24_two_round": lambda: _synth_case("c2x24_two_round", "c2x24", 300, 22, crosscheck_n=10),
    "c4_two_round": lambda: _synth_case("c4_two_round", "c4", 200, 4, crosscheck_n=20),
    "c4_two_round_e2": lambda: _synth_case("c4_two_round_e2", "c4", 150, 44, e=2,
                                           crosscheck_n=20),
    "c5_linked": lambda: _synth_case("c5_linked", "c5", 600, 5, crosscheck_n=200),
    "rna_linked": lambda: _rna_linked_case("rna_linked", 7),
    "random_front_iupac": lambda: _random_single_case("random_front_iupac", "front", 101),
    "random_back_iupac": lambda: _random_single_case("random_back_iupac", "back", 102),
}


def main(names):
    """Regenerate the named cases (all by default).  The full-matrix cross-check is pure Python
    (minutes for the long-read cases), so only a prefix of each long-read case is re-derived by
    it; the C oracle produces every vector."""
    oracle.build()
    for name in names or list(CASES):
        CASES[name]()


if __name__ == "__main__":
    main(sys.argv[1:])
