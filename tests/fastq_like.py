"""Nanopore-style FASTQ text for the gzip writer's size and speed checks (tests/test_nio.py,
tools/gzip_levels.py): MinKNOW-like header lines (read id, run id, channel, start time, flow
cell, model, the read id again as parent_read_id, the "start:stop|id strand=" prefix the
pychopper step adds), log-normal read lengths around 1.1 kb, uniform random bases, and
autocorrelated Phred scores around a per-read mean (AR(1), clipped to 2..50).  No real data
ships with the reference; this is the shape the writer is tuned for, stated, not measured."""
from __future__ import annotations

import uuid

import numpy as np


def nanopore_fastq(n_bytes: int, seed: int = 1) -> bytes:
    rng = np.random.default_rng(seed)
    run = "".join(rng.choice(list("0123456789abcdef"), 40))
    out, tot, i = [], 0, 0
    acgt = np.frombuffer(b"ACGT", np.uint8)
    while tot < n_bytes:
        n = int(np.clip(rng.lognormal(7.0, 0.4), 200, 8000))
        seq = acgt[rng.integers(0, 4, n)].tobytes()
        e = rng.normal(0, 4, n)
        z = np.empty(n)
        acc = 0.0
        for k in range(n):             # AR(1), a = 0.6
            acc = 0.6 * acc + e[k]
            z[k] = acc
        q = np.clip(np.round(rng.normal(16, 3) + z), 2, 50).astype(np.uint8) + 33
        u = uuid.UUID(bytes=rng.bytes(16))
        a = int(rng.integers(0, 60))
        head = (f"@{a}:{a + n}|{u} strand=+ runid={run} read={int(rng.integers(1, 99999))} "
                f"ch={int(rng.integers(1, 3000))} start_time=2024-03-"
                f"{int(rng.integers(1, 28)):02d}T{int(rng.integers(0, 24)):02d}:"
                f"{int(rng.integers(0, 60)):02d}:{int(rng.integers(0, 60)):02d}."
                f"{int(rng.integers(0, 999999)):06d}+00:00 flow_cell_id=PAS12345 "
                f"protocol_group_id=barcoding_run1 sample_id=pool1 parent_read_id={u} "
                f"basecall_model_version_id=dna_r10.4.1_e8.2_400bps_sup@v4.3.0")
        rec = head.encode() + b"\n" + seq + b"\n+\n" + q.tobytes() + b"\n"
        out.append(rec)
        tot += len(rec)
        i += 1
    return b"".join(out)
