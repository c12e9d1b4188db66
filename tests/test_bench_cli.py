"""bench.py's multi-GPU surface on CPU (no GPU calls): `--gpus` must agree with the launcher,
and `--reads-total` (BASELINE configs[2]: 10M reads sharded across 8 GPUs) splits one seeded
generation into contiguous ranges balanced on the sum of read lengths, the rule dmx_run_multi
applies to a batch (csrc/dmx_api.cpp dmx_run_multi)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from dmx import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("gpus,world", [(1, "2"), (8, "2"), (2, "1")])
def test_gpus_must_match_world_size(gpus, world):
    r = _bench(["--gpus", str(gpus), "--no-cpu-baseline"], {"WORLD_SIZE": world, "RANK": "0"})
    assert r.returncode != 0
    assert f"--gpus {gpus} but WORLD_SIZE={world}" in r.stderr
    assert r.stdout == ""


def test_gpus_zero_is_refused():
    r = _bench(["--gpus", "0"], {})
    assert r.returncode != 0


def _multi_cut(lens, n):
    """dmx_run_multi's split (csrc/dmx_api.cpp), restated."""
    total = int(lens.sum())
    cut = [len(lens)] * (n + 1)
    cut[0] = 0
    acc, k = 0, 1
    for r, L in enumerate(lens):
        if k >= n:
            break
        acc += int(L)
        while k < n and acc * n >= total * k:
            cut[k] = r + 1
            k += 1
    for j in range(1, n + 1):
        cut[j] = max(cut[j], cut[j - 1])
    return cut


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_reads_total_shards_by_length(world):
    n = 20000
    b = synth.shard_bounds("c2x24", n, world)
    assert b[0] == 0 and b[-1] == n and all(x <= y for x, y in zip(b, b[1:]))
    d = synth.generate("c2x24", n=n, threads=4)
    # the bounds follow the drawn lengths; the real ones differ only by adapter edits
    caps = np.array(d["lengths"], dtype=np.int64)
    sums = [caps[b[r]:b[r + 1]].sum() for r in range(world)]
    assert max(sums) - min(sums) <= 0.01 * caps.sum() + 2 * caps.max()
    # the same rule as dmx_run_multi, applied to the drawn lengths
    from dmx.synth import CONFIGS, SynthParams, lib as slib
    import ctypes
    cfg = dict(CONFIGS["c2x24"])
    n1, n2 = cfg.pop("panel")
    seed = cfg.pop("seed")
    cfg.pop("default_n")
    p = SynthParams(n1_used=n1, n2_used=n2, **cfg)
    drawn = np.empty(n, dtype=np.uint32)
    slib().synth_lengths(ctypes.byref(p), seed, 0, n, drawn.ctypes.data)
    drawn = drawn.astype(np.int64) - (2 * cfg["flank_max"] + 64)
    assert b == _multi_cut(drawn, world)
    # every rank's shard is the same slice of the one generation
    r = world - 1
    part = synth.generate("c2x24", n=b[r + 1] - b[r], first=b[r], threads=4)
    assert part["lengths"].tolist() == d["lengths"][b[r]:b[r + 1]].tolist()


def test_reads_total_edge_cases():
    assert synth.shard_bounds("c2x24", 0, 4) == [0, 0, 0, 0, 0]
    b = synth.shard_bounds("c2x24", 3, 8)
    assert b[0] == 0 and b[-1] == 3 and all(x <= y for x, y in zip(b, b[1:]))


def test_roofline_bytes_follow_survey_8d():
    """roofline.achieved uses SURVEY.md §8(d)'s B(read) = ceil(L/4) + 8 + ceil(L/64) + 24."""
    sys.path.insert(0, ROOT)
    import bench
    # §8(d)'s worked figure: L = 1200 -> 300 + 8 + 19 + 24 = 351 B
    assert bench.survey_bytes_per_read(np.array([1200])).tolist() == [351.0]
    L = np.array([0, 1, 4, 5, 63, 64, 65, 1208], dtype=np.uint32)
    want = [32, 34, 34, 35, 16 + 32 + 1, 16 + 32 + 1, 17 + 32 + 2, 302 + 32 + 19]
    assert bench.survey_bytes_per_read(L).tolist() == want
    assert bench.survey_bytes(L) == sum(want)
    # c2x24's reads average ~1.2 kb: ~350 B per read, as VERDICT r3 recomputed (353.7 B)
    d = synth.generate("c2x24", n=20000, threads=4)
    per = bench.survey_bytes(d["lengths"]) / len(d["lengths"])
    assert 340 < per < 365
    # the layout figure (1-bit mask, 40-B windows) is a different, larger number
    assert bench.filter_layout_bytes(d["lengths"], 0) > bench.survey_bytes(d["lengths"])
