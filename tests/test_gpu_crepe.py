"""CREPE f0 ("crepe" / "crepe-tiny", rvc_mlx/lib/mlx/crepe.py) on device vs the oracle restatement
(oracle/crepe.py; parity against the MLX reference itself is unpinned: mlx and torchcrepe are absent), and the
"fcpe" method of the MLX port (its RMVPE fallback, rvc_mlx/lib/mlx/fcpe.py:129-132)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def cents(a, b):
    return 1200.0 * np.abs(np.log2(np.maximum(a, 1e-3) / np.maximum(b, 1e-3)))


@pytest.fixture(scope="module")
def crepe_case():
    from oracle import crepe as oc
    from rvcx import synthetic

    audio = synthetic.speech_like(24000, seed=7).astype(np.float32)
    out = {}
    for kind in ("tiny", "full"):
        w = synthetic.crepe_state(kind, seed=11)
        out[kind] = (w,) + tuple(oc.get_f0(w, audio, return_periodicity=True))
    return audio, out


@pytest.mark.parametrize("kind", ["tiny", "full"])
def test_crepe_vs_oracle(engine, crepe_case, kind):
    """probabilities within 1e-4 of the peak (fp32 convs in another order); where the argmax agrees the decoded
    f0 is the same to fp32 rounding; >= 99 % of frames within 50 cents, voicing decisions agree on >= 99.5 %."""
    audio, cases = crepe_case
    w, f0_o, per_o, probs_o = cases[kind]
    engine.load_crepe(w)
    f0, per, probs = engine.crepe(audio, 50.0, 1100.0, 0.1, want_periodicity=True, want_probs=True)
    f0, per, probs = f0.cpu().numpy(), per.cpu().numpy(), probs.cpu().numpy()
    assert f0.shape == f0_o.shape == (1 + len(audio) // 160,)
    err = np.abs(probs - probs_o).max() / np.abs(probs_o).max()
    assert err < 1e-4, err
    same_peak = np.argmax(probs, 1) == np.argmax(probs_o, 1)
    assert same_peak.mean() > 0.98
    voiced = (f0 > 0) & (f0_o > 0)
    assert np.mean((f0 > 0) == (f0_o > 0)) >= 0.995
    assert np.mean(cents(f0[voiced], f0_o[voiced]) < 50) >= 0.99
    np.testing.assert_allclose(per, per_o, rtol=0, atol=1e-4)


def test_crepe_decode_range_and_threshold(engine, crepe_case):
    """f0_min / f0_max mask the bins outside the range (crepe.py:407-414) and threshold zeroes the frames whose
    filtered periodicity falls below it (crepe.py:319-320), as in the oracle."""
    from oracle import crepe as oc

    audio, cases = crepe_case
    w, _, _, probs_o = cases["tiny"]
    engine.load_crepe(w)
    for lo, hi, thr in ((100.0, 400.0, 0.1), (50.0, 1100.0, 0.6)):
        f0, per, probs = engine.crepe(audio, lo, hi, thr, want_periodicity=True, want_probs=True)
        f0d, perd = oc.decode(probs.cpu().numpy(), lo, hi)  # the oracle's decode on the device's own probs
        from scipy.ndimage import median_filter, uniform_filter1d

        perd = median_filter(perd, size=3)
        f0d = uniform_filter1d(f0d, size=3)
        f0d[perd < thr] = 0
        np.testing.assert_allclose(f0.cpu().numpy(), f0d, rtol=2e-6, atol=0)
        np.testing.assert_array_equal(per.cpu().numpy(), perd)


def test_pipeline_crepe_and_fcpe(engine, crepe_case):
    """PipelineMLX with f0_method crepe-tiny (state passed in) and fcpe (MLX semantics: RMVPE at 0.006 x 5):
    get_f0 equals the engine-level calls, and the whole pipeline runs with those f0 tracks."""
    from rvcx.infer import Config, HubertModel, PipelineMLX, RMVPE0Predictor, Synthesizer

    audio, cases = crepe_case
    w = cases["tiny"][0]
    pl = PipelineMLX(48000, Config(), HubertModel(engine), RMVPE0Predictor(engine), semantics="mlx",
                     crepe_weights={"tiny": w})
    x = audio.astype(np.float64)
    coarse, f0 = pl.get_f0(x, len(x) // 160, f0_method="crepe-tiny")
    ref = engine.crepe(audio, 50.0, 1100.0, 0.1).double()
    c_ref, _, f_ref = engine.f0_post(ref, 0.0)
    np.testing.assert_array_equal(coarse, c_ref.cpu().numpy())
    np.testing.assert_array_equal(f0, f_ref.cpu().numpy())
    coarse2, f02 = pl.get_f0(x, len(x) // 160, f0_method="fcpe")
    np.testing.assert_array_equal(f02, engine.f0_post(engine.rmvpe(audio, 0.03), 0.0)[2].cpu().numpy())
    net_g = Synthesizer(engine)
    y = pl.pipeline(None, net_g, 0, x, f0_method="crepe-tiny", seed=3)
    assert y.ndim == 1 and np.isfinite(y).all() and np.abs(y).max() > 0
    # the pipeline's f0 is CREPE on the high-passed, 1600-padded input (pipeline_mlx.py:284-318), then f0_post
    _, p32 = engine.highpass_pad(x, 1600)
    want = engine.f0_post(engine.crepe(p32, 50.0, 1100.0, 0.1).double(), 0.0)[2]
    np.testing.assert_array_equal(pl.last_f0.cpu().numpy(), want.cpu().numpy())
    with pytest.raises(ValueError):
        PipelineMLX(48000, Config(), HubertModel(engine), RMVPE0Predictor(engine)).get_f0(x, 0, f0_method="fcpe")


# ---------------------------------------------------------------- rvc/ semantics (torchcrepe.predict + viterbi)
def test_crepe_rvc_semantics_vs_oracle(engine, crepe_case):
    """rvc/'s CREPE.get_f0 (rvcx_crepe_ex semantics 1): the torchcrepe framing gives the oracle's probabilities
    (oracle.crepe.frame_audio_torch + forward) to 1e-4, and the viterbi decode + filters with the same dither values
    give the oracle's f0 / periodicity on the device's own probabilities."""
    from oracle import crepe as oc

    audio, cases = crepe_case
    w = cases["tiny"][0]
    engine.load_crepe(w)
    F = 1 + len(audio) // 160
    dither = np.random.default_rng(5).triangular(-20.0, 0.0, 20.0, size=F).astype(np.float32)
    f0, per, probs = engine.crepe(audio, 50.0, 1100.0, 0.1, want_periodicity=True, want_probs=True, semantics="rvc",
                                  dither=dither)
    probs = probs.cpu().numpy()
    probs_o = oc.forward(w, oc.frame_audio_torch(audio))
    assert np.abs(probs - probs_o).max() / np.abs(probs_o).max() < 1e-4
    f0_o, per_o, _ = oc.get_f0_rvc(w, audio, dither=dither, probs=probs)
    np.testing.assert_allclose(f0.cpu().numpy(), f0_o, rtol=2e-6, atol=0)
    np.testing.assert_array_equal(per.cpu().numpy(), per_o)


def _structured_probs(F, seed):
    """sigmoid-like outputs with a moving pitch track (a vibrato, an octave jump, a gap of unvoiced frames)."""
    rng = np.random.default_rng(seed)
    t = np.arange(F)
    track = 150 + 40 * np.sin(2 * np.pi * t / 90.0)
    track[F // 2:] += 60
    probs = rng.uniform(0.0, 0.35, size=(F, 360))
    bump = 0.95 * np.exp(-0.5 * ((np.arange(360)[None, :] - track[:, None]) / 1.5) ** 2)
    probs = np.maximum(probs, bump)
    probs[F // 3:F // 3 + 12] = rng.uniform(0.0, 0.06, size=(12, 360))
    return probs.astype(np.float32)


@pytest.mark.parametrize("lo,hi,thr", [(50.0, 1100.0, 0.1), (100.0, 400.0, 0.5)])
def test_crepe_viterbi_decode_vs_oracle(engine, lo, hi, thr):
    """The viterbi decode alone (rvcx_crepe_decode) on structured probabilities: the oracle's restatement of
    torchcrepe.decode.viterbi / librosa.sequence.viterbi and rvc/'s filters, f0 to fp32 rounding, the periodicity
    exactly; the path follows the track (a bin-exact decode, not a constant)."""
    from oracle import crepe as oc

    probs = _structured_probs(400, 9)
    f0, per = engine.crepe_decode(probs, lo, hi, thr, semantics="rvc")
    f0_o, per_o, _ = oc.get_f0_rvc(None, None, lo, hi, thr, probs=probs)
    np.testing.assert_allclose(f0.cpu().numpy(), f0_o, rtol=2e-6, atol=0)
    np.testing.assert_array_equal(per.cpu().numpy(), per_o)
    voiced = f0_o > 0
    assert 0.5 < voiced.mean() < 1.0 and len(np.unique(np.round(f0_o[voiced]))) > 20


def test_crepe_viterbi_decode_per_512_frame_batch(engine):
    """torchcrepe.predict (batch_size 512, rvc/lib/predictors/f0.py:38-49) decodes every 512-frame batch as
    its own viterbi sequence. F = 1300 (three batches, the last ragged) with the pitch track crossing both boundaries:
    the device decode equals the oracle's per-batch decode, and a whole-sequence decode differs from it (so the
    segmentation is observable on this input)."""
    from oracle import crepe as oc

    F = 1300
    rng = np.random.default_rng(21)
    t = np.arange(F)
    track = 180 + 35 * np.sin(2 * np.pi * t / 700.0)
    probs = rng.uniform(0.0, 0.3, size=(F, 360))
    probs = np.maximum(probs, 0.9 * np.exp(-0.5 * ((np.arange(360)[None, :] - track[:, None]) / 1.5) ** 2))
    # an ambiguous stretch at each boundary: a second, equally strong track 30 bins up, which the viterbi of a fresh
    # batch (uniform prior) and of a continued sequence (the previous state's band) resolve differently
    for b in (512, 1024):
        probs[b - 6:b + 6] = np.maximum(probs[b - 6:b + 6],
                                        0.95 * np.exp(-0.5 * ((np.arange(360)[None, :] - track[b - 6:b + 6, None] - 30)
                                                              / 1.5) ** 2))
    probs = probs.astype(np.float32)
    f0, per = engine.crepe_decode(probs, 50.0, 1100.0, 0.1, semantics="rvc")
    f0_o, per_o, _ = oc.get_f0_rvc(None, None, 50.0, 1100.0, 0.1, probs=probs)
    np.testing.assert_allclose(f0.cpu().numpy(), f0_o, rtol=2e-6, atol=0)
    np.testing.assert_array_equal(per.cpu().numpy(), per_o)
    whole = oc.viterbi_bins(probs, 50.0, 1100.0, batch=F)
    assert not np.array_equal(whole, oc.viterbi_bins(probs, 50.0, 1100.0))


def test_pipeline_crepe_rvc_semantics(engine, crepe_case):
    """PipelineRVCX(semantics="rvc") with f0_method crepe-tiny: get_f0 is rvcx_crepe_ex semantics 1 + f0_post, and the
    device pipeline (rvcx_pipeline_opts.f0_method 2) decodes CREPE on the high-passed, t_pad-padded input."""
    from rvcx.infer import Config, HubertModel, PipelineMLX, RMVPE0Predictor, Synthesizer

    audio, cases = crepe_case
    w = cases["tiny"][0]
    pl = PipelineMLX(48000, Config(), HubertModel(engine), RMVPE0Predictor(engine), semantics="rvc",
                     crepe_weights={"tiny": w})
    x = audio.astype(np.float64)
    coarse, f0 = pl.get_f0(x, len(x) // 160, f0_method="crepe-tiny")
    ref = engine.crepe(audio, 50.0, 1100.0, 0.1, semantics="rvc").double()
    c_ref, _, f_ref = engine.f0_post(ref, 0.0)
    np.testing.assert_array_equal(coarse, c_ref.cpu().numpy())
    np.testing.assert_array_equal(f0, f_ref.cpu().numpy())
    y = pl.pipeline(None, Synthesizer(engine), 0, x, f0_method="crepe-tiny", seed=3)
    assert y.ndim == 1 and np.isfinite(y).all() and np.abs(y).max() > 0
    _, p32 = engine.highpass_pad(x, pl.t_pad)
    want = engine.f0_post(engine.crepe(p32, 50.0, 1100.0, 0.1, semantics="rvc").double(), 0.0)[2]
    np.testing.assert_array_equal(pl.last_f0.cpu().numpy(), want.cpu().numpy())


@pytest.mark.parametrize("method", [1, 2])
def test_pipeline_batch_crepe_rows_match_single(engine, crepe_case, method):
    """rvcx_pipeline_batch with f0_method 1 (MLX CREPE) / 2 (rvc/'s CREPE, viterbi): each row's adjusted f0 equals
    rvcx_pipeline_ex's on that utterance alone (CREPE runs per row in both), and the outputs are finite."""
    audio, cases = crepe_case
    engine.load_crepe(cases["tiny"][0])
    engine.set_pipeline_highpass()
    x = np.stack([audio.astype(np.float64), 0.7 * np.roll(audio, 4000).astype(np.float64)])
    opts = engine.pipeline_opts(f0_method=method, protect=0.33)
    y, f0 = engine.pipeline_batch(x, opts, sids=0, seed=3, want_f0=True)
    assert torch.isfinite(y).all()
    for b in range(2):
        _, f0b = engine.pipeline_ex(x[b], opts, seed=3, want_f0=True)
        np.testing.assert_array_equal(f0[b].cpu().numpy(), f0b.cpu().numpy())
