"""Multi-GPU sharding of the demultiplexing path.

Reads are independent, so a batch is split into contiguous read ranges balanced by total
length (long rRNA reads must not skew one rank), each rank runs the whole two-round pipeline
on its range on its own GPU, and the only exchange is one all-reduce of the per-bin counts
(RCCL over xGMI with the `nccl` backend on MI355X; `gloo` in the CPU tests).  Per-read outputs
stay on their rank; concatenating shard outputs in rank order preserves input order.
"""
from __future__ import annotations

import numpy as np


def balanced_ranges(lengths: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous [lo, hi) read ranges, one per rank, with near-equal total length."""
    n = len(lengths)
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    csum = np.cumsum(lengths.astype(np.float64))
    total = csum[-1]
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(csum, total * r / world, side="left")) + 1)
    cuts.append(n)
    cuts = np.minimum(np.maximum.accumulate(np.array(cuts)), n)
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def allreduce_counts(counts: np.ndarray, device=None) -> np.ndarray:
    """Sum per-bin counts over all ranks of the default process group (no-op if none)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return counts
    t = torch.from_numpy(counts.astype(np.int64))
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t)
    return t.cpu().numpy()
