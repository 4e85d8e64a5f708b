"""Utterance sharding across GPUs: one process per GPU, independent utterances,
no data-path collective. Only bookkeeping crosses ranks: the total audio-seconds (SUM), the wall
time (MAX) and per-utterance summaries (all_gather_object). Works with the "nccl" (RCCL) backend on
the GPU box and "gloo" on CPU (tests)."""
from __future__ import annotations

import heapq
from typing import Dict, List, Sequence


def assign_lpt(lengths: Sequence[int], world: int) -> List[List[int]]:
    """Longest-processing-time-first assignment of utterance indices to ranks: sort by length
    (descending, index ascending on ties), give each to the least-loaded rank (lowest rank on ties).
    Equal lengths reduce to round-robin (i::world, like extract.py:101-117)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    order = sorted(range(len(lengths)), key=lambda i: (-int(lengths[i]), i))
    heap = [(0, r) for r in range(world)]
    out: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + int(lengths[i]), r))
    return [sorted(x) for x in out]


def reduce_throughput(dist, audio_sec: float, elapsed: float, device=None) -> Dict[str, float]:
    """Whole-job numbers: SUM of audio seconds over ranks and MAX of wall time over ranks."""
    import torch

    if dist is None or not dist.is_initialized():
        return {"audio_sec": audio_sec, "elapsed": elapsed, "value": audio_sec / elapsed if elapsed > 0 else 0.0}
    if dist.get_backend() == "gloo":
        device = "cpu"  # gloo reduces host tensors
    t = torch.tensor([audio_sec, elapsed], dtype=torch.float64, device=device)
    s = t.clone()
    dist.all_reduce(s[0:1], op=dist.ReduceOp.SUM)
    dist.all_reduce(s[1:2], op=dist.ReduceOp.MAX)
    a, e = float(s[0].item()), float(s[1].item())
    return {"audio_sec": a, "elapsed": e, "value": a / e if e > 0 else 0.0}


def gather_records(dist, records: list) -> list:
    """All ranks' per-utterance records, flattened in rank order."""
    if dist is None or not dist.is_initialized():
        return list(records)
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, records)
    return [r for part in out for r in part]
