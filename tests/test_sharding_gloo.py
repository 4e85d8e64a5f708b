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
