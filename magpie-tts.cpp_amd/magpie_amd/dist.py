"""Multi-GPU coordination for the replica path.

Utterances are independent, so N GPUs hold full weight replicas and split the
utterances; there is no collective on the data path. torch.distributed (gloo,
host-side) only carries the bench barrier, the max-over-ranks timing and, for
natural-EOS work, a shared claim counter.

Two ways to split:
  * shard_utterances: a static contiguous split (the fixed-length bench, where every
    utterance costs the same);
  * WorkQueue / synthesize_queue: a dynamic work-queue. With EOS live the
    utterances' lengths differ (magpie.cpp:4340-4352 stops each one at its own EOS),
    so a static split leaves GPUs idle behind the rank that drew the long ones. Each
    rank instead claims the next `batch` utterances from an atomic counter in the
    process group's store whenever its device batch is free, longest text first (the
    longest-processing-time rule: a text's length is the host's best predictor of its
    frame count), so the ranks finish within about one batch of each other.
"""
from __future__ import annotations

import itertools
from typing import Callable, Dict, List, Optional, Sequence


def shard_utterances(n_total: int, rank: int, world: int) -> List[int]:
    """Contiguous blocks: utterance b goes to GPU floor(b * world / n_total)."""
    return [b for b in range(n_total) if (b * world) // n_total == rank]


def _dist():
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover - torch is in the image
        return None
    return dist if dist.is_available() and dist.is_initialized() else None


def max_over_ranks(value: float) -> float:
    import torch
    dist = _dist()
    if dist is None:
        return value
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float) -> float:
    import torch
    dist = _dist()
    if dist is None:
        return value
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


_queue_ids = itertools.count()


class WorkQueue:
    """Items 0..n_items-1 handed out in order to whichever rank asks next.

    claim(k) atomically takes the next k positions from a counter in the default
    process group's store (c10d Store.add: one round trip to the rendezvous host, no
    device work), so every position goes to exactly one rank. Without an initialised
    process group the counter is local (world size 1). Every rank must construct its
    queues in the same order: the store key is derived from a per-process sequence
    number."""

    def __init__(self, n_items: int, store=None, key: Optional[str] = None):
        if n_items < 0:
            raise ValueError("n_items must be >= 0")
        self.n = n_items
        seq = next(_queue_ids)
        self.key = key or f"magpie_amd/work_queue/{seq}"
        if store is None and _dist() is not None:
            from torch.distributed import distributed_c10d
            store = distributed_c10d._get_default_store()
        self.store = store
        self._local = 0

    def claim(self, k: int = 1) -> List[int]:
        """The next up to k positions (empty once the queue is drained)."""
        if k < 1:
            raise ValueError("k must be >= 1")
        if self.store is not None:
            end = int(self.store.add(self.key, k))
            start = end - k
        else:
            start = self._local
            self._local += k
        return list(range(start, min(start + k, self.n)))


def longest_first(tokens: Sequence[Sequence[int]]) -> List[int]:
    """Utterance order of the queue: text length descending, ties by index."""
    return sorted(range(len(tokens)), key=lambda i: (-len(tokens[i]), i))


def synthesize_queue(synth: Callable[[List[Sequence[int]], List[int]], List], tokens: Sequence[Sequence[int]],
                     speakers: Optional[Sequence[int]] = None, batch: int = 8,
                     queue: Optional[WorkQueue] = None) -> Dict[int, object]:
    """Run this rank's share of `tokens` through synth(tokens_batch, speakers_batch) ->
    one result per utterance (e.g. a Device.synthesize(...).codes wrapper), claiming
    `batch` utterances at a time from the shared queue until it is drained.
    Returns {utterance index: result} for the utterances this rank decoded."""
    n = len(tokens)
    spk = [0] * n if speakers is None else list(speakers)
    if len(spk) != n:
        raise ValueError("speakers must match tokens")
    order = longest_first(tokens)
    q = queue if queue is not None else WorkQueue(n)
    mine: Dict[int, object] = {}
    while True:
        pos = q.claim(batch)
        if not pos:
            break
        utt = [order[p] for p in pos]
        out = synth([tokens[u] for u in utt], [spk[u] for u in utt])
        if len(out) != len(utt):
            raise RuntimeError(f"synth returned {len(out)} results for {len(utt)} utterances")
        for u, r in zip(utt, out):
            mine[u] = r
    return mine


def gather_results(mine: Dict[int, object], n_total: int) -> List[object]:
    """Every rank's {index: result} merged into one list in utterance order (gloo
    all_gather_object on the host; world size 1: the dict itself)."""
    dist = _dist()
    parts = [mine]
    if dist is not None:
        parts = [None] * dist.get_world_size()
        dist.all_gather_object(parts, mine)
    out: List[object] = [None] * n_total
    seen = 0
    for part in parts:
        for u, r in part.items():
            if out[u] is not None:
                raise RuntimeError(f"utterance {u} decoded twice")
            out[u] = r
            seen += 1
    if seen != n_total:
        raise RuntimeError(f"{n_total - seen} utterances were never decoded")
    return out


def device_synth(dev, max_dec_steps: int = 500, **kw) -> Callable[[List[Sequence[int]], List[int]], List]:
    """synth callable over a magpie_amd.Device: one device batch per claim (at most
    dev.max_batch() utterances), EOS live unless kw says otherwise; returns the codes."""
    def run(toks, spks):
        return dev.synthesize(toks, speakers=spks, max_dec_steps=max_dec_steps, **kw).codes
    return run
