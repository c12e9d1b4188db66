"""One small case per rule the oracle marks [UNVERIFIED] (oracle/cutadapt_oracle.c,
oracle/pyref.py), built so that the two plausible readings of the rule give
different outputs.  tools/parity_vs_cutadapt.sh runs every case through a real cutadapt 4.9
(where one is installed) and through the drop-in, and diffs the outputs: a DIFF names the rule
to correct.  tests/test_oracle.py checks, with oracle/pyref.py switched to each alternative
reading (pyref.rules), that every case really tells the readings apart.

The reads were found by a seeded search over random adapters and reads (pyref under both
readings); the reference's own settings (-e 0.1 -O 3) never reach most of these rules.

Usage: python tools/unverified_cases.py DIR   (writes DIR/<case>.fastq|.fasta, DIR/ads_<case>.fa
and DIR/cases.tsv: case, input file, output options with @OUT@ for the output directory,
cutadapt options)
"""
from __future__ import annotations

import os
import sys

# name: rule, alternative reading, adapters (name, seq), where, -e, -O, --rc, reads, linked
CASES = [
    {"name": "negscore", "rule": "best_init", "alt": "zero", "where": "back",
     "adapters": [("a1", "AAAC")], "e": 3, "O": 1, "rc": False,
     "reads": ["CCG", "TTTTTTTG", "GGGGGGGA"],
     "why": "absolute -e 3 on a 4-nt 3' adapter with -O 1: the only acceptable cells of CCG "
            "score < 0; a best match seeded with score 0 refuses them"},
    {"name": "scoretie", "rule": "tie", "alt": "first", "where": "back",
     "adapters": [("a1", "AATAACCT")], "e": 0.2, "O": 3, "rc": False,
     "reads": ["AAATCAACCTATTGGAATAAC", "GGGGAATAACCTGGGGAATAAC"],
     "why": "an internal 1-error full match and a later exact 3' partial of equal score: "
            "lower cost wins vs the first cell found"},
    {"name": "col0", "rule": "col0", "alt": "zero", "where": "back",
     "adapters": [("a1", "TCTACTCC")], "e": 0.3, "O": 3, "rc": False,
     "reads": ["TACTCCCCTA", "CTACTCCGGGGGG"],
     "why": "the adapter's first bases are missing at the read start: BACK column-0 cells "
            "score -2 i (insertion score) vs 0"},
    {"name": "besttie", "rule": "besttie", "alt": "first", "where": "front",
     "adapters": [("a1", "AGCTGGACGC"), ("a2", "AGCTGGACGCT"), ("a3", "AGCTGGACG")],
     "e": 0.2, "O": 3, "rc": False,
     "reads": ["ACGTAGCAGGACGTTGAAAA"],
     "why": "two adapters reach the same score: fewer errors wins vs file order"},
    {"name": "rctie", "rule": "rc", "alt": "geq", "where": "front",
     "adapters": [("a1", "CAGATCATAC")], "e": 0.1, "O": 3, "rc": True,
     "reads": ["TTGCAGATCATACGCTGGTATGATCTGCGA"],
     "why": "forward and reverse complement score the same: the reverse complement only on a "
            "strictly greater score vs on >="},
    {"name": "linked", "rule": "linked", "alt": "front", "where": "linked",
     "adapters": [("p1", "ACGTTGCA...GGATCCAA")], "e": 0.1, "O": 3, "rc": False,
     "reads": ["ACGTTGCATTTTTTTTTTTTTTGGATCCAA", "ACGTTGCATTTTTTTTTTTTTTTTTTT",
               "TTTTTTTTTTTTTTTTGGATCCAA"],
     "why": "-g F...R with only the front primer present: both parts required (untrimmed) vs "
            "the front part alone trims"},
]


def cutadapt_options(c) -> list[str]:
    """The cutadapt options of a case (output options are added by the caller)."""
    opt = ["-e", str(c["e"]), "-O", str(c["O"])] + (["--rc"] if c["rc"] else [])
    if c["where"] == "linked":
        for _, s in c["adapters"]:
            opt += ["-g", s]
    elif len(c["adapters"]) == 1:
        opt += ["-a" if c["where"] == "back" else "-g", c["adapters"][0][1]]
    else:
        opt += ["-a" if c["where"] == "back" else "-g", f"file:ads_{c['name']}.fa"]
    return opt


def write(d: str):
    os.makedirs(d, exist_ok=True)
    rows = []
    for c in CASES:
        if c["where"] == "linked":
            inp = f"{c['name']}.fasta"
            with open(os.path.join(d, inp), "w") as fh:
                for i, s in enumerate(c["reads"]):
                    fh.write(f">{c['name']}{i}\n{s}\n")
            out = (f"-o @OUT@/{c['name']}.fasta "
                   f"--untrimmed-output=@OUT@/{c['name']}_untrimmed.fasta")
        else:
            inp = f"{c['name']}.fastq"
            with open(os.path.join(d, inp), "w") as fh:
                for i, s in enumerate(c["reads"]):
                    fh.write(f"@{c['name']}{i}\n{s}\n+\n{'I' * len(s)}\n")
            out = (f"-o @OUT@/{c['name']}_{{name}}.fastq" if len(c["adapters"]) > 1
                   else f"-o @OUT@/{c['name']}.fastq")
        if len(c["adapters"]) > 1 and c["where"] != "linked":
            with open(os.path.join(d, f"ads_{c['name']}.fa"), "w") as fh:
                for nm, s in c["adapters"]:
                    fh.write(f">{nm}\n{s}\n")
        rows.append("\t".join([c["name"], inp, out, " ".join(cutadapt_options(c))]))
    with open(os.path.join(d, "cases.tsv"), "w") as fh:
        fh.write("\n".join(rows) + "\n")


if __name__ == "__main__":
    write(sys.argv[1])
