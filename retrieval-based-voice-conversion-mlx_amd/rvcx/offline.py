"""Batched offline conversion across the GPUs of one node (config C4: 512 x 30 s utterances on 8 GPUs).

The reference shards a file list over devices with one process per device and no communication
(``files[i :: len(devices)]``, rvc/train/extract/extract.py:101-117, :150-170). Here:

* ``plan``: every rank builds the SAME job list and takes its shard by longest-processing-time-first
  assignment (``sharding.assign_lpt``; equal lengths reduce to the reference's ``i :: world``). Within a
  shard, utterances of equal length are grouped into batches of up to B: one batch = one
  ``rvcx_pipeline_batch`` pass (batched RMVPE, HuBERT and Synthesizer.infer).
* ``run``: converts the shard batch by batch through a caller-supplied ``convert(batch, step)`` that
  returns one record row per utterance (id, n_out, peak, rms) as a [b, 4] tensor -- kept where it was made
  (the GPU bench leaves them in HBM, so the loop never waits for the device) -- the GPU bench passes the
  device pipeline, the gloo test a CPU stand-in. No data-path collective.
* ``finish``: the bookkeeping collectives: SUM of audio-seconds and MAX of wall time
  (``sharding.reduce_throughput``) and an ``all_gather`` of the per-utterance records into one
  [world * max_shard, 4] tensor (RCCL over xGMI with the "nccl" backend, host tensors with "gloo"); rank 0
  then checks that every utterance of the job was converted exactly once.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence

from .sharding import assign_lpt, reduce_throughput

REC_FIELDS = ("utt", "n_out", "peak", "rms")


@dataclass(frozen=True)
class Utterance:
    idx: int        # position in the job list
    n: int          # samples @16 kHz
    seed: int       # synthetic content seed


def c4_job(n_utt: int = 512, n_samples: int = 480000, seed0: int = 1000) -> List[Utterance]:
    """BASELINE configs[3]: 512 utterances of 30 s (480000 samples @16 kHz), seeds 1000 + i."""
    return [Utterance(i, n_samples, seed0 + i) for i in range(n_utt)]


@dataclass
class Plan:
    rank: int
    world: int
    batch: int
    shard: List[int]                 # job indices of this rank (ascending)
    batches: List[List[int]]         # job indices per batched pass, equal length within a batch


def plan(job: Sequence[Utterance], world: int, rank: int, batch: int) -> Plan:
    if batch < 1:
        raise ValueError("batch must be >= 1")
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    shard = assign_lpt([u.n for u in job], world)[rank]
    by_len: Dict[int, List[int]] = {}
    for i in shard:
        by_len.setdefault(job[i].n, []).append(i)
    batches = []
    for n in sorted(by_len, reverse=True):
        ids = by_len[n]
        batches += [ids[k:k + batch] for k in range(0, len(ids), batch)]
    return Plan(rank, world, batch, shard, batches)


def run(p: Plan, convert: Callable[[List[int], int], "object"], sync: Callable[[], None] = lambda: None,
        dist=None, steps: Optional[int] = None):
    """Convert the shard (or its first ``steps`` batches) between two barriers; returns (records, elapsed s)."""
    todo = p.batches if steps is None else p.batches[:steps]
    sync()
    if dist is not None and dist.is_initialized():
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    recs = []
    for step, b in enumerate(todo):
        recs.append(convert(b, step))
    sync()
    if dist is not None and dist.is_initialized():
        dist.barrier()
    return recs, time.perf_counter() - t0


def stack_records(recs) -> "object":
    """The per-batch record blocks of ``run`` as one host [n, 4] float64 tensor."""
    import torch

    if not recs:
        return torch.empty((0, len(REC_FIELDS)), dtype=torch.float64)
    return torch.cat([torch.as_tensor(r, dtype=torch.float64).reshape(-1, len(REC_FIELDS)).cpu() for r in recs])


def gather_records(dist, recs, max_shard: int, device=None):
    """all_gather of fixed-size record tensors ([max_shard, 4] float64 per rank, utt = -1 for padding);
    returns the valid rows of all ranks (every rank gets them)."""
    import torch

    mine = stack_records(recs)
    t = torch.full((max_shard, len(REC_FIELDS)), -1.0, dtype=torch.float64)
    t[: mine.shape[0]] = mine
    if dist is None or not dist.is_initialized():
        parts = [t]
    else:
        dev = "cpu" if dist.get_backend() == "gloo" else device
        t = t.to(dev)
        parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, t)
    allr = torch.cat([x.cpu() for x in parts])
    return allr[allr[:, 0] >= 0]


def finish(p: Plan, job: Sequence[Utterance], recs, elapsed: float, dist=None, device=None, sr: int = 16000):
    """Whole-job numbers (audio-seconds SUM, wall MAX over ranks) and the gathered per-utterance records.
    Raises if the gathered records do not cover the converted utterances exactly once."""
    done_ids = [int(u) for u in stack_records(recs)[:, 0].tolist()]
    audio_sec = sum(job[i].n for i in done_ids) / sr
    tot = reduce_throughput(dist, audio_sec, elapsed, device=device)
    world_max = max(len(plan(job, p.world, r, p.batch).shard) for r in range(p.world))
    allr = gather_records(dist, recs, world_max, device=device)
    ids = sorted(int(u) for u in allr[:, 0].tolist())
    if len(ids) != len(set(ids)):
        raise RuntimeError("offline job: an utterance was converted twice")
    expected = round(tot["audio_sec"] * sr)
    got = sum(job[i].n for i in ids)
    if got != expected:
        raise RuntimeError(f"offline job: gathered records cover {got} samples, ranks report {expected}")
    tot["records"] = allr
    tot["utterances"] = len(ids)
    return tot
