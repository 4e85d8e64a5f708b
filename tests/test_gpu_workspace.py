"""Device workspace ownership (SURVEY.md 8(b) "Ownership": workspace sized by rvcx_workspace_bytes, or allocated by
the caller via torch and passed in): the size query, a caller-owned torch arena carrying a whole pipeline call with a
bit-identical result, a too-small arena failing with RVCX_E_OOM at the API edge, and the return to internal
allocation."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

RVCX_E_OOM = -4


def _audio(n, seed=3):
    rng = np.random.Generator(np.random.PCG64(seed))
    t = np.arange(n) / 16000.0
    return 0.3 * np.sin(2 * np.pi * 220.0 * t) + 0.05 * rng.standard_normal(n)


def test_workspace_query_and_caller_arena(engine):
    from rvcx._lib import RvcxError

    engine.set_pipeline_highpass()
    n = 3 * 16000
    audio = _audio(n)
    need = engine.workspace_bytes(n)
    assert need > 0
    ref = engine.pipeline(audio, seed=7).cpu()
    held, arena_bytes, _ = engine.workspace_info()
    assert 0 < held <= need and arena_bytes == 0
    arena = torch.empty(need, dtype=torch.uint8, device=engine.device)
    try:
        engine.set_workspace(arena)
        out = engine.pipeline(audio, seed=7).cpu()
        held, arena_bytes, used = engine.workspace_info()
        assert arena_bytes == need and 0 < used <= need and held <= used
        assert torch.equal(out, ref)
        # the same call again reuses the carved regions
        assert torch.equal(engine.pipeline(audio, seed=7).cpu(), ref)
        assert engine.workspace_info()[2] == used
        # half the size: the call fails at the API edge instead of allocating
        engine.set_workspace(arena[: need // 2])
        with pytest.raises(RvcxError) as ei:
            engine.pipeline(audio, seed=7)
        assert ei.value.code == RVCX_E_OOM
    finally:
        engine.set_workspace(None)
    assert engine.workspace_info()[1] == 0
    assert torch.equal(engine.pipeline(audio, seed=7).cpu(), ref)


def test_workspace_bytes_grows_with_the_call(engine):
    engine.set_pipeline_highpass()
    # (the reflect pad needs n > t_pad = 1 s)
    short = engine.workspace_bytes(2 * 16000)
    long = engine.workspace_bytes(6 * 16000)
    batch = engine.workspace_bytes(2 * 16000, B=4)
    assert 0 < short < long and short < batch


def _split_opts(engine):
    # a multi-chunk plan at test sizes: t_max 3 s, t_center 2 s, t_query 0.5 s (pipeline.py:440-452 with x_max 3,
    # x_center 2, x_query 0.5)
    return engine.pipeline_opts(t_pad=16000, t_pad_tgt=48000, t_max=48000, t_center=32000, t_query=8000)


def _speech_with_gaps(n, gaps, seed=5):
    a = _audio(n, seed)
    for g in gaps:
        a[g:g + 800] *= 1e-4
    return a


def test_workspace_query_holds_long_inputs_with_off_centre_splits(engine):
    """for inputs above t_max the chunk plan depends on the audio. Quiet stretches at the low end of the
    first split window and the high end of the second give the longest middle chunk real audio can give; an arena
    of the queried size (sized on the worst-case plan) holds the call, bit-identical to internal allocation."""
    engine.set_pipeline_highpass()
    o = _split_opts(engine)
    n = 8 * 16000
    audio = _speech_with_gaps(n, [32000 - 8000 + 10, 64000 + 8000 - 900])
    ref = engine.pipeline_ex(audio, o, seed=3).cpu()
    need = engine.workspace_bytes(n, opts=o)
    arena = torch.empty(need, dtype=torch.uint8, device=engine.device)
    try:
        engine.set_workspace(arena)
        out = engine.pipeline_ex(audio, o, seed=3).cpu()
        used = engine.workspace_info()[2]
        assert 0 < used <= need
        assert torch.equal(out, ref)
    finally:
        engine.set_workspace(None)


def test_workspace_arena_short_then_long_call(engine):
    """an arena sized for the long call carries a short call and then the long one (each call carves its
    regions from offset 0: the short call's regions are not kept beside the long call's), and writes by the caller
    into the arena between calls do not leak into results (the memoised zeros / scalars go with the regions)."""
    engine.set_pipeline_highpass()
    o = _split_opts(engine)
    long_n, short_n = 8 * 16000, int(2.5 * 16000)
    a_long, a_short = _speech_with_gaps(long_n, [30000, 70000]), _audio(short_n, 9)
    ref_long = engine.pipeline_ex(a_long, o, seed=1).cpu()
    ref_short = engine.pipeline_ex(a_short, o, seed=2).cpu()
    need = engine.workspace_bytes(long_n, opts=o)
    assert need >= engine.workspace_bytes(short_n, opts=o)
    arena = torch.empty(need, dtype=torch.uint8, device=engine.device)
    try:
        engine.set_workspace(arena)
        assert torch.equal(engine.pipeline_ex(a_short, o, seed=2).cpu(), ref_short)
        assert torch.equal(engine.pipeline_ex(a_long, o, seed=1).cpu(), ref_long)
        arena.fill_(0x5A)
        assert torch.equal(engine.pipeline_ex(a_short, o, seed=2).cpu(), ref_short)
        arena.fill_(0xA5)
        assert torch.equal(engine.pipeline_ex(a_long, o, seed=1).cpu(), ref_long)
    finally:
        engine.set_workspace(None)


@pytest.mark.parametrize("with_arena", [True, False])
def test_calls_on_two_streams_do_not_share_live_regions(engine, with_arena):
    """a call enqueued on stream B right after a call on stream A (no host synchronisation between them)
    must not overwrite the regions A's call still uses -- in arena mode every call carves from offset 0, and in pool
    mode both calls take the same named buffers. begin_call orders the second call after the first one's streams, so
    both results equal their serial runs."""
    engine.set_pipeline_highpass()
    n_long, n_short = 6 * 16000, int(2.5 * 16000)
    a_long, a_short = _audio(n_long, 4), _audio(n_short, 5)
    ref_long = engine.pipeline(a_long, seed=3).cpu()
    ref_short = engine.pipeline(a_short, seed=4).cpu()
    arena = torch.empty(engine.workspace_bytes(n_long), dtype=torch.uint8, device=engine.device) if with_arena else None
    sa, sb = torch.cuda.Stream(engine.device), torch.cuda.Stream(engine.device)
    try:
        engine.set_workspace(arena)
        torch.cuda.synchronize(engine.device)
        for _ in range(2):
            with torch.cuda.stream(sa):
                out_a = engine.pipeline(a_long, seed=3)
            with torch.cuda.stream(sb):
                out_b = engine.pipeline(a_short, seed=4)
            torch.cuda.synchronize(engine.device)
            assert torch.equal(out_a.cpu(), ref_long)
            assert torch.equal(out_b.cpu(), ref_short)
    finally:
        engine.set_workspace(None)
