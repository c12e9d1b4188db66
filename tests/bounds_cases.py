"""Cases shared by tests/test_bounds.py: caller-packed batches at the edges of dmx_run's layout
contract, and the panels whose kernels reach farthest around a view.

Imported by the GPU tests (release library, in-process) and run as a script by
`test_bounds_build_suite` under DMX_DEBUG_BOUNDS=1 (dmx/libdmx_bounds.so, in a child process),
where every gather and slot access is checked and a violation fails the call naming the kernel.
The oracle (oracle/, the CPU restatement of cutadapt 4.9) is only the checker here.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "nanopore-barcoding-orc_amd"), os.path.join(ROOT, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import oracle  # noqa: E402  (checker)
from dmx import lib, synth  # noqa: E402


def rand_dna(rng, n):
    return "".join(rng.choice(list("ACGT"), size=n))


def seed46_panel(rng, m_fixed=None):
    """The shape of the round-4 seed-46 fault: a 3' panel of 15 adapters sharing a 12-nt prefix
    and a 21-nt suffix (index screen on), to run at -e 0.3, whose screen warm-up starts up to
    m + k columns before a view."""
    pre, suf = rand_dna(rng, 12), rand_dna(rng, 21)
    if m_fixed:
        return [pre + rand_dna(rng, m_fixed - 33) + suf for _ in range(15)]
    return [pre + rand_dna(rng, int(rng.integers(6, 28))) + suf for _ in range(15)]


def edge_reads(rng, panel, n=400):
    """Short and empty reads first and last, partial adapters at both read ends."""
    seqs = ["", "A", "ACG", rand_dna(rng, 5)]
    for _ in range(n):
        s = rand_dna(rng, int(rng.integers(0, 160)))
        a = panel[int(rng.integers(len(panel)))]
        u = rng.random()
        if u < 0.35:
            s = s + a[:int(rng.integers(1, len(a) + 1))]
        elif u < 0.7:
            s = a[int(rng.integers(0, len(a))):] + s
        seqs.append(s)
    seqs += ["", "T", rand_dna(rng, 7)]
    return seqs


def tight_pack(seqs, first_offset=16, gap=0):
    """A caller-packed batch at the edge of dmx_run's contract: read 0 at nt offset 16 (the
    smallest accepted), the reads back to back `gap` nt apart (no 32-nt grid, no pads), and
    n_words as small as the contract allows (the last read ends exactly 64 nt before the end)."""
    lens = np.array([len(s) for s in seqs], dtype=np.uint32)
    offs = np.zeros(len(seqs), dtype=np.uint64)
    g = first_offset
    for i, s in enumerate(seqs):
        offs[i] = g
        g += len(s) + gap
    end = int(max((offs + lens).max(), first_offset)) + 64
    end = (end + 15) // 16 * 16          # n_words * 16 >= every read's end + 64, minimal
    n_words = end // 16
    codes = np.zeros(end, dtype=np.uint8)
    nmb = np.zeros(2 * end, dtype=np.uint8)  # the mask buffer has as many words (1 bit per nt)
    tab = np.full(256, 4, dtype=np.uint8)
    for ch, v in zip(b"ACGT", range(4)):
        tab[ch] = v
    for i, s in enumerate(seqs):
        if not s:
            continue
        c = tab[np.frombuffer(s.encode(), dtype=np.uint8)]
        o = int(offs[i])
        codes[o:o + len(s)] = np.where(c < 4, c, 0)
        nmb[o:o + len(s)] = c >= 4
    bits = np.zeros(2 * end, dtype=np.uint8)
    bits[0::2] = codes & 1
    bits[1::2] = codes >> 1
    seq2b = np.packbits(bits, bitorder="little").view(np.uint32)[:n_words].copy()
    nmask = np.packbits(nmb, bitorder="little").view(np.uint32)[:n_words].copy()
    return lib.Packed(seq2b, nmask, offs, lens)


def same(got, exp) -> int:
    g = got.view(np.uint8).reshape(len(got), -1)
    e = exp.view(np.uint8).reshape(len(exp), -1)
    return int((g != e).any(axis=1).sum())


def case_results(ctx, name):
    """Run one named case on ctx; returns (mismatching reads vs the oracle, reads)."""
    rng = np.random.default_rng(sum(map(ord, name)))
    if name.startswith("seed46"):
        m_fixed = 64 if "m64" in name else None
        panel = seed46_panel(rng, m_fixed)
        seqs = edge_reads(rng, panel)
        blob, offs, lens = oracle.pack_ascii(seqs)
        bad = 0
        for use_rc in (True, False):
            exp = oracle.run_batch(oracle.Panel(panel, oracle.BACK, max_errors=0.3,
                                                min_overlap=3),
                                   None, blob, offs, lens, mode=0, use_rc=use_rc, threads=8)
            ctx.set_panel(0, panel, lib.DMX_BACK | (lib.DMX_RC if use_rc else 0), 0.3, 3)
            ctx.set_mode(lib.MODE_SINGLE)
            packed = tight_pack(seqs) if "tight" in name else lib.pack(blob, offs, lens)
            bad += same(ctx.run(packed), exp)
        return bad, 2 * len(seqs)
    if name.startswith("c2x24"):   # the benchmark's panels, FRONT then BACK, edge bands
        d = synth.generate("c2x24", n=3000, seed=sum(map(ord, name)))
        seqs = [bytes(d["blob"][int(o):int(o) + int(n)]).decode()
                for o, n in zip(d["offsets"], d["lengths"])]
        seqs = ["", "ACGT"] + seqs[:1500] + [s[:40] for s in seqs[1500:1600]] + ["G"]
        blob, offs, lens = oracle.pack_ascii(seqs)
        exp = oracle.run_batch(oracle.Panel(d["sp5"], oracle.FRONT),
                               oracle.Panel(d["sp27"], oracle.BACK), blob, offs, lens, mode=1,
                               threads=8)
        ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC)
        ctx.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC)
        ctx.set_mode(lib.MODE_TWO_ROUND)
        packed = tight_pack(seqs) if "tight" in name else lib.pack(blob, offs, lens)
        return same(ctx.run(packed), exp), len(seqs)
    raise ValueError(name)


CASES = ["seed46", "seed46_m64", "seed46_tight", "seed46_m64_tight", "c2x24", "c2x24_tight"]


def main():
    """Child process of test_bounds_build_suite (DMX_DEBUG_BOUNDS=1): the self test, then every
    case; one JSON line."""
    assert lib.BOUNDS and lib.LIB_PATH.endswith("libdmx_bounds.so"), lib.LIB_PATH
    out = {"lib": os.path.basename(lib.LIB_PATH), "cases": {}}
    with lib.Context(0) as ctx:
        # the self test needs a loaded batch and pipeline buffers
        bad, n = case_results(ctx, "c2x24")
        out["cases"]["c2x24"] = [bad, n, ""]
        rc, msg, vals = ctx.bounds_selftest()
        out["selftest"] = {"rc": rc, "msg": msg, "out": [int(v) for v in vals]}
        for name in CASES:
            try:
                bad, n = case_results(ctx, name)
                out["cases"][name] = [bad, n, ""]
            except lib.DmxError as e:
                out["cases"][name] = [-1, 0, str(e)]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
