"""N > 1 path on CPU: two gloo ranks shard utterances and reduce throughput like bench.py does over
RCCL (the rendezvous uses 127.0.0.1)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, lengths, q):
    import torch.distributed as dist

    from rvcx.sharding import assign_lpt, gather_records, reduce_throughput

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = assign_lpt(lengths, world)[rank]
        audio = sum(lengths[i] for i in mine) / 16000.0
        elapsed = 1.0 + rank  # rank 1 is the slow one: MAX must pick it
        res = reduce_throughput(dist, audio, elapsed)
        recs = gather_records(dist, [(i, rank) for i in mine])
        q.put((rank, mine, res, recs))
    finally:
        dist.destroy_process_group()


def test_assign_lpt_balanced_and_complete():
    from rvcx.sharding import assign_lpt

    lengths = [480000] * 512
    parts = assign_lpt(lengths, 8)
    assert [len(p) for p in parts] == [64] * 8
    assert parts[0][:3] == [0, 8, 16]  # equal lengths -> round-robin i::8
    rag = [5, 1, 9, 3, 7, 7, 2]
    p2 = assign_lpt(rag, 3)
    assert sorted(i for p in p2 for i in p) == list(range(len(rag)))
    loads = [sum(rag[i] for i in p) for p in p2]
    assert max(loads) - min(loads) <= max(rag)


def test_two_rank_gloo_sharding():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    lengths = [16000 * (3 + (i % 5)) for i in range(10)]
    procs = [ctx.Process(target=_worker, args=(r, 2, port, lengths, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    shards = [o[1] for o in out]
    assert sorted(shards[0] + shards[1]) == list(range(10))
    total = sum(lengths) / 16000.0
    for _, _, res, recs in out:
        assert res["audio_sec"] == pytest.approx(total)
        assert res["elapsed"] == 2.0
        assert res["value"] == pytest.approx(total / 2.0)
        assert sorted(r[0] for r in recs) == list(range(10))


def _c4_worker(rank, world, port, n_utt, batch, q):
    """The C4 driver of bench.py (rvcx.offline: plan -> run -> finish) with a CPU stand-in for the device
    pipeline; the collectives are the same calls bench.py makes over RCCL."""
    import torch
    import torch.distributed as dist

    from rvcx import offline

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        job = offline.c4_job(n_utt, n_samples=4800)
        p = offline.plan(job, world, rank, batch)
        seen = []

        def convert(ids, step):
            assert len(ids) <= batch and len({job[i].n for i in ids}) == 1
            seen.extend(ids)
            out = torch.stack([torch.full((job[i].n * 3,), 0.01 * (i + 1)) for i in ids])
            rec = torch.empty((len(ids), 4), dtype=torch.float64)
            rec[:, 0] = torch.tensor(ids, dtype=torch.float64)
            rec[:, 1] = out.shape[1]
            rec[:, 2] = out.abs().amax(1).double()
            rec[:, 3] = out.double().pow(2).mean(1).sqrt()
            return rec

        recs, el = offline.run(p, convert, dist=dist)
        tot = offline.finish(p, job, recs, el + rank, dist=dist)
        q.put((rank, p.shard, [len(b) for b in p.batches], sorted(seen), tot["utterances"], tot["audio_sec"],
               tot["elapsed"], tot["records"][:, 0].tolist(), tot["records"][:, 2].tolist()))
    finally:
        dist.destroy_process_group()


def test_c4_driver_two_rank_gloo():
    """bench.py --config c4's driver at world 2: the shards partition the job (i::2), batches of <= B equal-length
    utterances, every utterance converted once, the all_gather'd records complete on every rank, audio-seconds
    SUMmed and wall time MAXed over ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n_utt, batch = 37, 8
    procs = [ctx.Process(target=_c4_worker, args=(r, 2, port, n_utt, batch, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0][1] == list(range(0, n_utt, 2)) and out[1][1] == list(range(1, n_utt, 2))
    for rank, shard, sizes, seen, nutt, audio_sec, elapsed, ids, peaks in out:
        assert seen == shard and max(sizes) <= batch and sum(sizes) == len(shard)
        assert nutt == n_utt and sorted(int(i) for i in ids) == list(range(n_utt))
        assert audio_sec == pytest.approx(n_utt * 4800 / 16000.0)
        assert elapsed >= 1.0  # rank 1 reported el + 1: the MAX over ranks
        for i, pk in zip(ids, peaks):
            assert pk == pytest.approx(0.01 * (int(i) + 1))
