"""Bounds of the device buffers (VERDICT r4 'next' item 1).

Round 4's two GPU faults were one class of bug: a gather position or a list index outside its
buffer (an unsigned wrap of a position before the first read; an item list sized by another
list's capacity).  This module covers the three answers:
  * the DMX_DEBUG_BOUNDS build (dmx/libdmx_bounds.so): every gather and slot / item / result /
    count access checked against its buffer, a violation failing the call naming the kernel;
  * the host check of every panel's reach around a view against the device guard
    (dmx_panel_reach, refused by dmx_set_panel when it does not fit);
  * caller-packed batches at the edge of dmx_run's layout contract (offset 16, no pads, tight
    n_words), run without a fault and with the oracle's results.
"""
import json
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

import bounds_cases as bc
from dmx import lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nanopore-barcoding-orc_amd")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC) and not shutil.which("hipcc"),
                    reason="hipcc not installed")
def test_bounds_build_compiles():
    """The checked build of the kernels compiles for gfx950 (hipcc, no GPU)."""
    r = subprocess.run([HIPCC, "-std=c++17", "--offload-arch=gfx950", "-fsyntax-only",
                        "-Wno-unused-result", "-DDMX_DEBUG_BOUNDS=1",
                        os.path.join(PKG, "csrc", "dmx_kernels.hip")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]


def test_bounds_library_exports_the_abi():
    """dmx/libdmx_bounds.so (built by `make all` / build()) exports every dmx.h entry point, so
    DMX_DEBUG_BOUNDS=1 can stand in for libdmx.so in any run (no GPU calls here)."""
    import ctypes
    path = os.path.join(PKG, "dmx", "libdmx_bounds.so")
    assert os.path.exists(path), "run make -C nanopore-barcoding-orc_amd all"
    L = ctypes.CDLL(path)
    for sym in lib.EXPORTS:
        assert hasattr(L, sym), sym
    L.dmx_abi_version.restype = ctypes.c_int
    assert L.dmx_abi_version() == lib.ABI_VERSION


def test_panel_reach_seed46_shape():
    """The seed-46 fault's panel shape (3' adapters of 64 nt with a 12-nt shared prefix and a
    21-nt shared suffix, -e 0.3): the index screen's warm-up asks for positions more than
    m + k before a view, past the clamp; after the clamp every gather stays inside the guard
    for the smallest offset (16) and tail (64) dmx_run accepts, so the panel is accepted."""
    rng = np.random.default_rng(46)
    for m_fixed in (64, None):
        panel = bc.seed46_panel(rng, m_fixed)
        for flags in (lib.DMX_BACK | lib.DMX_RC, lib.DMX_BACK):
            rc, r = lib.panel_reach(panel, flags, 0.3, 3)
            assert rc == 0, (rc, r)
            if m_fixed == 64:
                # m - pre_len + kf + 31 = 64 - 12 + 19 + 31 nt before the view: beyond the clamp
                assert r["pre_raw"] == 102
            assert r["pre_raw"] > 64 + 16 >= r["pre"]
            assert r["need_pre"] <= r["guard"] and r["need_post"] <= r["guard"]
            assert r["guard"] == 1024


def test_panel_reach_reference_and_random_panels():
    """Every shipped panel, and random panels (IUPAC, 3..64 nt, FRONT / BACK / mixed, -e up to
    0.3 and absolute counts), keep the kernels' reach inside the guard; the clamp bounds the
    pre-view reach at 80 nt whatever the panel."""
    from dmx import panel as dpanel
    data = os.path.join(PKG, "dmx", "data")
    checked = 0
    for f in sorted(os.listdir(data)):
        if not f.endswith(".fa"):
            continue
        seqs = [s for _, s in dpanel.read_fasta(os.path.join(data, f))]
        seqs = [s.upper().replace("U", "T") for s in seqs if 0 < len(s) <= 64]
        if not seqs:
            continue
        for flags in (lib.DMX_FRONT | lib.DMX_RC, lib.DMX_BACK | lib.DMX_RC):
            for e in (0.1, 0.2, 0.3, 3.0):
                rc, r = lib.panel_reach(seqs, flags, e, 3)
                if rc == -4:        # resolve window too small for this rate: refused anyway
                    continue
                assert rc == 0, (f, flags, e, rc)
                assert r["pre"] <= 80 and r["need_pre"] <= r["guard"]
                assert r["need_post"] <= r["guard"]
                checked += 1
    rng = np.random.default_rng(5)
    for _ in range(300):
        n = int(rng.integers(1, 33))
        m = int(rng.integers(3, 65))
        shared = int(rng.integers(0, m // 2 + 1))
        suf = bc.rand_dna(rng, shared)
        seqs = [bc.rand_dna(rng, m - shared) + suf for _ in range(n)]
        if rng.random() < 0.3:
            seqs = [s[:3] + "N" + s[4:] for s in seqs]
        wheres = None
        flags = int(rng.choice([lib.DMX_FRONT, lib.DMX_BACK])) | lib.DMX_RC
        if rng.random() < 0.2:
            wheres = [int(rng.choice([lib.DMX_FRONT, lib.DMX_BACK])) for _ in seqs]
        e = float(rng.choice([0.0, 0.1, 0.2, 0.3, 1.0, 4.0]))
        rc, r = lib.panel_reach(seqs, flags, e, int(rng.integers(1, 8)), wheres=wheres)
        assert rc in (0, -4), rc
        if rc == 0:
            assert r["pre"] <= 80 and r["need_pre"] <= r["guard"]
            assert r["need_post"] <= r["guard"]
            checked += 1
    assert checked > 250


def test_tight_pack_layout_is_accepted_shape():
    """The tight caller layout used by the GPU cases meets the contract exactly: first read at
    offset 16, last read ending 64 nt before the end of the words (CPU, no GPU)."""
    rng = np.random.default_rng(1)
    seqs = bc.edge_reads(rng, bc.seed46_panel(rng), n=50)
    p = bc.tight_pack(seqs)
    assert int(p.offsets[0]) == 16
    assert int((p.offsets + p.lengths).max()) + 64 <= p.n_words * 16 < \
        int((p.offsets + p.lengths).max()) + 64 + 16


@pytest.mark.gpu
@pytest.mark.parametrize("name", bc.CASES)
def test_edge_layouts_and_far_reaching_panels(ctx, name):
    """Release library: caller-packed batches at the contract's edge (offset 16, no pads, tight
    n_words) and the seed-46 panel shape (index screen warming up before short views at
    -e 0.3), FRONT + BACK two-round on the benchmark panels: no fault, every result byte equal
    to the oracle's."""
    bad, n = bc.case_results(ctx, name)
    assert bad == 0, f"{bad} of {n} reads differ"


@pytest.mark.gpu
def test_bounds_build_suite():
    """DMX_DEBUG_BOUNDS=1 (dmx/libdmx_bounds.so) in a child process: the self test's planted
    violations are caught and named (the gather below the guard is skipped and reads 0), and
    every edge case runs with no violation and the oracle's results."""
    path = os.path.join(PKG, "dmx", "libdmx_bounds.so")
    assert os.path.exists(path)
    env = dict(os.environ, DMX_DEBUG_BOUNDS="1")
    env.pop("DMX_LIBDMX", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "bounds_cases.py")],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["lib"] == "libdmx_bounds.so"
    st = out["selftest"]
    assert st["rc"] == -5, st
    assert "bounds_selftest_kernel" in st["msg"] and "seq index" in st["msg"], st
    assert st["out"][0] == 0 and st["out"][1] == 0, st
    for name, (bad, n, err) in out["cases"].items():
        assert err == "" and bad == 0, (name, bad, n, err)
