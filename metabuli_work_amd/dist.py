"""Multi-GPU read sharding: one process per GPU, reads split across ranks, the DB
replicated in every GPU's HBM, and one collective at the end — an all-gather of the fixed-size
per-read result records (RCCL over xGMI with the "nccl" backend; gloo on CPU for tests).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch
import torch.distributed as dist


def shard_bounds(off: np.ndarray, world: int) -> List[Tuple[int, int]]:
    """Split reads [0, n) into `world` contiguous shards of ~equal base count (long reads vary
    500x in length, so equal read counts would not balance the work)."""
    n = len(off) - 1
    if n == 0:
        return [(0, 0)] * world
    total = float(off[-1] - off[0])
    cuts = [0]
    for r in range(1, world):
        target = off[0] + total * r / world
        cuts.append(int(np.searchsorted(off[:-1], target, side="left")))
    cuts.append(n)
    for i in range(1, len(cuts)):
        cuts[i] = max(cuts[i], cuts[i - 1])
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def shard_reads(seq: np.ndarray, off: np.ndarray, lo: int, hi: int) -> Tuple[np.ndarray, np.ndarray]:
    a, b = int(off[lo]), int(off[hi])
    return seq[a:b], (off[lo:hi + 1] - off[lo]).astype(np.uint64)


def gather_records(local: torch.Tensor, counts: List[int], group=None) -> torch.Tensor:
    """All-gather variable-length rows (records of `local.shape[1]` bytes) in rank order."""
    world = dist.get_world_size(group)
    width = local.shape[1]
    cap = max(counts)
    pad = torch.zeros((cap, width), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    out = torch.empty((world * cap, width), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out.view(-1), pad.view(-1), group=group)
    parts = [out[r * cap:r * cap + counts[r]] for r in range(world)]
    return torch.cat(parts, 0)
