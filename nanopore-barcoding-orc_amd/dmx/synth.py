"""Seeded synthetic workloads via libdmx_synth.so (host C++).

Benchmark / test input only.  Every read is a pure function of (seed, read index), so a shard
[first, first+n) equals the same slice of one big generation.
"""
from __future__ import annotations

import ctypes
import os
import random

import numpy as np

from . import panel as _panel

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.environ.get("DMX_LIBDIR") or HERE, "libdmx_synth.so")


class SynthParams(ctypes.Structure):
    _fields_ = [("length_model", ctypes.c_int32), ("len_mean", ctypes.c_double),
                ("len_sigma_log", ctypes.c_double), ("len_min", ctypes.c_int32),
                ("len_max", ctypes.c_int32), ("adapter_error", ctypes.c_double),
                ("rc_fraction", ctypes.c_double), ("adapterless_fraction", ctypes.c_double),
                ("n_fraction", ctypes.c_double), ("n1_used", ctypes.c_int32),
                ("n2_used", ctypes.c_int32), ("flank_max", ctypes.c_int32),
                ("linked", ctypes.c_int32), ("missing_fraction", ctypes.c_double)]


# name -> (params, n_sp5, n_sp27, panel kind)
CONFIGS = {
    # config 1: 1k x 800 nt, 4 SP5 x 4 SP27, 3% adapter error, 10% RC, 5% adapterless
    "c1": dict(length_model=0, len_mean=800, len_sigma_log=0, len_min=800, len_max=800,
               adapter_error=0.03, rc_fraction=0.10, adapterless_fraction=0.05, n_fraction=0.0,
               panel=(4, 4), flank_max=8, default_n=1000, seed=1),
    # config 2: 10M reads, lognormal mean 1200 (sigma_log 0.35, [300, 6000]), 5% error, 10% RC,
    # 2% adapterless, full 12x12 panel (SP27 j from all 12 so invalid wells are exercised)
    "c2": dict(length_model=1, len_mean=1200, len_sigma_log=0.35, len_min=300, len_max=6000,
               adapter_error=0.05, rc_fraction=0.10, adapterless_fraction=0.02,
               n_fraction=0.001, panel=(12, 12), flank_max=8, default_n=10_000_000, seed=2),
    # config 2 with the synthetic 24x24 panel (seed 22)
    "c2x24": dict(length_model=1, len_mean=1200, len_sigma_log=0.35, len_min=300, len_max=6000,
                  adapter_error=0.05, rc_fraction=0.10, adapterless_fraction=0.02,
                  n_fraction=0.001, panel=(24, 24), flank_max=8, default_n=10_000_000, seed=2),
    # config 4: 70% COI (insert 300-900) + 30% rRNA (insert ~3 kb), 15% adapter error
    "c4": dict(length_model=2, len_mean=0, len_sigma_log=0, len_min=300, len_max=6000,
               adapter_error=0.15, rc_fraction=0.10, adapterless_fraction=0.02, n_fraction=0.001,
               panel=(12, 12), flank_max=8, default_n=50_000_000, seed=4),
    # config 5: amplicon_sorter consensuses (FASTA) framed by the linked COI primer pairs of
    # COI_primers.fa (IUPAC positions instantiated at random), 5% primer error, 10% with one
    # primer missing (these must stay untrimmed), no RC (04_cleaning_primers.sh:377)
    "c5": dict(length_model=3, len_mean=0, len_sigma_log=0, len_min=100, len_max=2000,
               adapter_error=0.05, rc_fraction=0.0, adapterless_fraction=0.0, n_fraction=0.0,
               panel=(2, 2), flank_max=4, default_n=10_000_000, seed=5, linked=1,
               missing_fraction=0.10),
}


def linked_panels():
    """(pair ids, forward primers, reverse primers) of the config-5 linked pairs."""
    from . import panel
    pairs = panel.primer_pairs(os.path.join(os.path.dirname(panel.SP5_FASTA), "COI_primers.fa"))
    return [p[0] for p in pairs], [p[1] for p in pairs], [p[2] for p in pairs]

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built (make -C nanopore-barcoding-orc_amd)")
        L = ctypes.CDLL(LIB_PATH)
        L.synth_lengths.argtypes = [ctypes.POINTER(SynthParams), ctypes.c_uint64,
                                    ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p]
        L.synth_fill.argtypes = [ctypes.POINTER(SynthParams), ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                 ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        _lib = L
    return _lib


def _mutate_variable(rng: random.Random, s: str) -> str:
    return "".join(rng.choice("ACGT") for _ in s)


def _edit_distance(a: str, b: str) -> int:
    prev = list(range(len(b) + 1))
    for i, ca in enumerate(a, 1):
        cur = [i]
        for j, cb in enumerate(b, 1):
            cur.append(min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (ca != cb)))
        prev = cur
    return prev[-1]


def panels(n1: int, n2: int, seed: int = 22) -> tuple[list[str], list[str], list[str], list[str]]:
    """(names1, sp5, names2, sp27rc).  Beyond the 12 real adapters per side, extra adapters keep
    the constant flanks and get rejection-sampled 17-nt variable regions with edit distance >= 7
    to every other adapter of the panel (the synthetic 24x24 panel of SURVEY.md §8d)."""
    n5, s5 = _panel.load_panel(_panel.SP5_FASTA)
    n27, s27 = _panel.load_panel(_panel.SP27RC_FASTA)
    rng = random.Random(seed)

    def extend(names, seqs, n, pre, var_len, suf_off, prefix):
        names, seqs = list(names), list(seqs)
        while len(seqs) < n:
            cand = seqs[0][:pre] + _mutate_variable(rng, "N" * var_len) + seqs[0][suf_off:]
            if all(_edit_distance(cand, s) >= 7 for s in seqs):
                seqs.append(cand)
                names.append(f"{prefix}_{len(seqs):03d}")
        return names[:n], seqs[:n]

    n5, s5 = extend(n5, s5, n1, 25, 17, 42, "SP5")
    n27, s27 = extend(n27, s27, n2, 17, 17, 34, "SP27")
    return n5, s5, n27, s27


def generate(config: str, n: int | None = None, seed: int | None = None, first: int = 0,
             threads: int = 8):
    """Return dict(blob, offsets, lengths, truth, sp5, sp27, names1, names2)."""
    cfg = dict(CONFIGS[config])
    n = cfg.pop("default_n") if n is None else n
    cfg.pop("default_n", None)
    seed = cfg.pop("seed") if seed is None else seed
    cfg.pop("seed", None)
    n1, n2 = cfg.pop("panel")
    if cfg.get("linked"):
        names1, sp5, sp27 = linked_panels()
        names2 = list(names1)
    else:
        names1, sp5, names2, sp27 = panels(n1, n2)
    p = SynthParams(n1_used=n1, n2_used=n2, **cfg)
    L = lib()
    caps = np.empty(n, dtype=np.uint32)
    L.synth_lengths(ctypes.byref(p), seed, first, n, caps.ctypes.data)
    offs = np.zeros(n, dtype=np.uint64)
    if n > 1:
        offs[1:] = np.cumsum(caps[:-1], dtype=np.uint64)
    total = int(offs[-1] + caps[-1]) if n else 0
    blob = np.empty(total, dtype=np.uint8)
    lens = np.empty(n, dtype=np.uint32)
    truth = np.empty((n, 3), dtype=np.int32)
    a1 = (ctypes.c_char_p * n1)(*[s.encode() for s in sp5])
    l1 = (ctypes.c_int * n1)(*[len(s) for s in sp5])
    a2 = (ctypes.c_char_p * n2)(*[s.encode() for s in sp27])
    l2 = (ctypes.c_int * n2)(*[len(s) for s in sp27])
    L.synth_fill(ctypes.byref(p), a1, l1, a2, l2, seed, first, n, offs.ctypes.data,
                 blob.ctypes.data, lens.ctypes.data, truth.ctypes.data, threads)
    return dict(blob=blob, offsets=offs, lengths=lens, truth=truth, sp5=sp5, sp27=sp27,
                names1=names1, names2=names2)


def shard_bounds(config: str, n_total: int, world: int, seed: int | None = None) -> list[int]:
    """Contiguous read ranges [b[r], b[r+1]) of one seeded generation of n_total reads, balanced
    on the sum of the drawn read lengths (the rule dmx_run_multi applies to a
    batch's real lengths): every rank computes the same bounds without generating the reads."""
    cfg = dict(CONFIGS[config])
    seed = cfg["seed"] if seed is None else seed
    n1, n2 = cfg["panel"]
    for k in ("default_n", "seed", "panel"):
        cfg.pop(k)
    p = SynthParams(n1_used=n1, n2_used=n2, **cfg)
    caps = np.empty(n_total, dtype=np.uint32)
    lib().synth_lengths(ctypes.byref(p), seed, 0, n_total, caps.ctypes.data)
    drawn = caps.astype(np.uint64) - np.uint64(2 * cfg["flank_max"] + 64)
    acc = np.cumsum(drawn, dtype=np.uint64)
    total = int(acc[-1]) if n_total else 0
    bounds = [0]
    for r in range(1, world):
        # first read index whose prefix sum reaches r/world of the total (dmx_run_multi's cut)
        bounds.append(int(np.searchsorted(acc, -(-total * r // world), side="left")) + 1
                      if n_total else 0)
    bounds.append(n_total)
    for r in range(1, world + 1):
        bounds[r] = max(bounds[r], bounds[r - 1])
    return bounds


def to_strings(d) -> list[str]:
    b = d["blob"]
    return [b[o:o + l].tobytes().decode("ascii") for o, l in zip(d["offsets"], d["lengths"])]
