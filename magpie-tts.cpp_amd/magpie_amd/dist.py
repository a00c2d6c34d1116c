"""Multi-GPU coordination for the replica path.

Utterances are independent, so N GPUs hold full weight replicas and split the
utterances; there is no collective on the data path. torch.distributed (gloo,
host-side) only carries the bench barrier and the max-over-ranks timing.
"""
from __future__ import annotations

from typing import List


def shard_utterances(n_total: int, rank: int, world: int) -> List[int]:
    """Contiguous blocks: utterance b goes to GPU floor(b * world / n_total)."""
    return [b for b in range(n_total) if (b * world) // n_total == rank]


def max_over_ranks(value: float) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
