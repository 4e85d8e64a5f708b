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
