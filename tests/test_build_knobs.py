"""Compile-time invariants of the A/B build knobs (CPU: hipcc -fsyntax-only for gfx950, no GPU).

The filter groups every view's last segment into four step buckets (csrc/dmx_kernels.hip,
kStepsPerBucket).  In round 3 a DMX_SEG_SPAN=384 A/B build sized the buckets as span / 256 = 1
step, so 6-step last segments landed in buckets 5-6, indexed past the four-bucket tables and
faulted (illegal memory access).  The bucket width is now derived from the span and the invariant
is a static_assert, so every span the knob accepts builds with in-range buckets and every other
span is refused at compile time."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "nanopore-barcoding-orc_amd", "csrc", "dmx_kernels.hip")
HIPCC = "/opt/rocm/bin/hipcc"

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC) and not shutil.which("hipcc"),
                                reason="hipcc not installed")


def _syntax(defs):
    return subprocess.run([HIPCC, "-std=c++17", "--offload-arch=gfx950", "-fsyntax-only",
                           "-Wno-unused-result"] + defs + [SRC],
                          capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("span", [256, 384, 512, 640, 768, 1024])
def test_segment_spans_build(span):
    r = _syntax([f"-DDMX_SEG_SPAN={span}"])
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.parametrize("span,why", [(100, "whole 64-position steps"),
                                      (2048, "128..1024 positions")])
def test_bad_segment_spans_are_refused(span, why):
    r = _syntax([f"-DDMX_SEG_SPAN={span}"])
    assert r.returncode != 0
    assert why in r.stderr
