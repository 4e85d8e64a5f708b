"""Decoders beside the default HiFi-GAN (NSF) on the device, against the reference's own modules
(tests/golden/make_golden_vocoders.py) and the CPU oracle:
  * MRF HiFi-GAN (synthesizers.py:86-98, generators/hifigan_mrf.py): 9-harmonic per-sample source
    (source_harm.hip, exact double-accumulated phase scans), MRF blocks on the conv kernels, conv_post bias.
Bars: latents rel <= 1e-4, waveform rel <= 2e-3 and spectrogram corr >= 0.999 (the NSF synth test's bar)."""
import dataclasses

import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))


@pytest.fixture(scope="module")
def mrf_engine(hubert_w, rmvpe_w):
    from rvcx import synthetic
    from rvcx.config import SYNTH_48K_V2
    from rvcx.engine import Engine
    from rvcx.weights import normalize_state

    g = golden("synth_mrf_b2.npz")
    cfg = dataclasses.replace(SYNTH_48K_V2, vocoder="MRF HiFi-GAN")
    w = normalize_state(synthetic.synth_state(int(g["seed_w"]), cfg))
    e = Engine(0)
    e.load_synth(w, cfg)
    e.load_hubert(hubert_w)
    e.load_rmvpe(rmvpe_w)
    yield e, w, cfg
    e.close()


def test_mrf_synth_vs_reference(mrf_engine):
    from oracle.metrics import spectrogram_correlation

    eng, _, _ = mrf_engine
    g = golden("synth_mrf_b2.npz")
    out, zp, z = eng.synth_infer(g["phone"], g["lengths"], g["pitch"], g["f0"], g["sid"], eps_z=g["eps_z"],
                                 eps_src=g["eps_src"], want_latents=True)
    torch.cuda.synchronize()
    assert rel_err(z.cpu().numpy().transpose(0, 2, 1), g["z"]) < 1e-4
    o = out.cpu().numpy()
    ref = g["o"].reshape(o.shape)
    assert rel_err(o, ref) < 2e-3, rel_err(o, ref)
    for b in range(o.shape[0]):
        assert spectrogram_correlation(o[b], ref[b]) > 0.999


def test_mrf_generated_noise_is_seeded(mrf_engine):
    """Without injected noise the source draws from Philox(seed): same seed -> same output, new seed -> new."""
    eng, _, _ = mrf_engine
    g = golden("synth_mrf_b2.npz")
    a = eng.synth_infer(g["phone"], g["lengths"], g["pitch"], g["f0"], g["sid"], seed=5).cpu().numpy()
    b = eng.synth_infer(g["phone"], g["lengths"], g["pitch"], g["f0"], g["sid"], seed=5).cpu().numpy()
    c = eng.synth_infer(g["phone"], g["lengths"], g["pitch"], g["f0"], g["sid"], seed=6).cpu().numpy()
    assert np.array_equal(a, b) and not np.array_equal(a, c) and np.isfinite(a).all()


def test_mrf_pipeline_vs_oracle(mrf_engine, hubert_w, rmvpe_w):
    from oracle.metrics import spectrogram_correlation
    from oracle.pipeline import OraclePipeline
    from rvcx.config import HUBERT_BASE, RMVPE_CFG

    eng, w, cfg = mrf_engine
    g = golden("pipeline_2p5s.npz")
    m = g["audio"].shape[0] + 2 * 16000
    T = min(m // 160, 2 * HUBERT_BASE.frames(m))
    rng = np.random.Generator(np.random.PCG64(91))
    eps_z = rng.standard_normal((1, cfg.inter_channels, T)).astype(np.float32)
    eps_src = np.concatenate([rng.standard_normal(T * cfg.upp * 9), rng.random(9)]).astype(np.float32)
    eng.set_pipeline_highpass()
    out = eng.pipeline(g["audio"], sid=0, semitones=0, protect=0.33, t_pad=16000, t_pad_tgt=48000, eps_z=eps_z,
                       eps_src=eps_src).cpu().numpy()
    noise = {"z": torch.from_numpy(eps_z), "src": torch.from_numpy(eps_src)}
    orc = OraclePipeline(48000, synth_w=w, synth_cfg=cfg, hubert_w=hubert_w, hubert_cfg=HUBERT_BASE, rmvpe_w=rmvpe_w,
                         rmvpe_cfg=RMVPE_CFG, noise_fn=lambda shape, which: noise[which].reshape(shape))
    ref = orc.pipeline(0, g["audio"].astype(np.float64).copy(), protect=0.33)
    assert out.shape == ref.shape
    # the pitch track comes from RMVPE on both sides (near-tie bins may differ): spectrogram-level bar
    assert spectrogram_correlation(out, ref) >= 0.995, spectrogram_correlation(out, ref)


@pytest.fixture(scope="module")
def refinegan_engine(hubert_w, rmvpe_w):
    from rvcx import synthetic
    from rvcx.config import SYNTH_48K_V2
    from rvcx.engine import Engine
    from rvcx.weights import normalize_state

    g = golden("synth_refinegan_b1.npz")
    cfg = dataclasses.replace(SYNTH_48K_V2, vocoder="RefineGAN")
    w = normalize_state(synthetic.synth_state(int(g["seed_w"]), cfg))
    e = Engine(0)
    e.load_synth(w, cfg)
    e.load_hubert(hubert_w)
    e.load_rmvpe(rmvpe_w)
    yield e, w, cfg
    e.close()


def test_refinegan_synth_vs_reference(refinegan_engine):
    """RefineGAN: linear-f0 source, kaiser-sinc downsampling branch, AdaIN-noised ParallelResBlocks
    (refinegan.hip, runtime_refinegan.cpp) vs the reference RefineGANGenerator (torchaudio's resample restated)."""
    from conftest import refinegan_noise
    from oracle.metrics import spectrogram_correlation

    eng, _, cfg = refinegan_engine
    g = golden("synth_refinegan_b1.npz")
    eps_z, eps_src = refinegan_noise(g)
    T = g["phone"].shape[1]
    out, zp, z = eng.synth_infer(g["phone"], g["lengths"], g["pitch"], g["f0"], g["sid"],
                                 eps_z=eps_z.reshape(1, cfg.inter_channels, T), eps_src=eps_src, want_latents=True)
    torch.cuda.synchronize()
    eng.check_device_status()
    assert rel_err(z.cpu().numpy().transpose(0, 2, 1), g["z"]) < 1e-4
    o = out.cpu().numpy()
    ref = g["o"].reshape(o.shape)
    assert rel_err(o, ref) < 2e-3, rel_err(o, ref)
    assert spectrogram_correlation(o[0], ref[0]) > 0.999


def test_refinegan_vs_oracle_longer(refinegan_engine):
    """A longer ragged-free batch (B=2, T=40) against the oracle with the same injected draws."""
    from oracle import synth as osynth
    from oracle.metrics import spectrogram_correlation
    from rvcx import synthetic

    eng, w, cfg = refinegan_engine
    B, T = 2, 40
    rng = np.random.Generator(np.random.PCG64(5))
    phone = rng.standard_normal((B, T, 768)).astype(np.float32)
    f0 = synthetic.f0_walk(B, T, seed=6)
    pitch = rng.integers(1, 256, size=(B, T)).astype(np.int64)
    lengths = np.array([T, T], np.int64)
    sid = np.array([0, 3], np.int64)
    eps_z = rng.standard_normal((B, cfg.inter_channels, T)).astype(np.float32)
    n_src = len(osynth.refinegan_noise_sizes(cfg, B, T))
    sizes = osynth.refinegan_noise_sizes(cfg, B, T)
    eps_src = np.concatenate([rng.standard_normal(sizes[0]), rng.random(sizes[1])] +
                             [rng.standard_normal(s) for s in sizes[2:]]).astype(np.float32)
    assert n_src == 26
    out = eng.synth_infer(phone, lengths, pitch, f0, sid, eps_z=eps_z, eps_src=eps_src).cpu().numpy()
    t = torch.from_numpy
    ref = osynth.synth_infer(w, cfg, t(phone), t(lengths), t(pitch), t(f0), t(sid), t(eps_z), t(eps_src))[0].numpy()
    ref = ref.reshape(out.shape)
    assert rel_err(out, ref) < 2e-3, rel_err(out, ref)
    for b in range(B):
        assert spectrogram_correlation(out[b], ref[b]) > 0.999
