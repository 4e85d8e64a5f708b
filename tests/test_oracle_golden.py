"""Pin the CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py) and the reference's own KAT data (ios_test_data)."""
import numpy as np
import pytest
import torch

from conftest import golden
from rvcx.config import HUBERT_BASE, RMVPE_CFG, SYNTH_48K_V2


def _t(x):
    return torch.from_numpy(np.asarray(x))


def rel_err(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))


def test_synth_t64_matches_reference(synth_w):
    from oracle import synth as osynth

    g = golden("synth_t64.npz")
    o, mask, (z, z_p, m_p, logs_p) = osynth.synth_infer(
        synth_w, SYNTH_48K_V2, _t(g["phone"]), _t(g["lengths"]), _t(g["pitch"]), _t(g["f0"]), _t(g["sid"]),
        _t(g["eps_z"]), _t(g["eps_src"]))
    assert rel_err(m_p, g["m_p"]) < 1e-5
    assert rel_err(logs_p, g["logs_p"]) < 1e-5
    assert rel_err(z, g["z"]) < 1e-5
    assert rel_err(o, g["o"]) < 1e-4


def test_synth_ragged_batch_matches_reference(synth_w):
    from oracle import synth as osynth

    g = golden("synth_b2_ragged.npz")
    o, mask, (z, z_p, m_p, logs_p) = osynth.synth_infer(
        synth_w, SYNTH_48K_V2, _t(g["phone"]), _t(g["lengths"]), _t(g["pitch"]), _t(g["f0"]), _t(g["sid"]),
        _t(g["eps_z"]), _t(g["eps_src"]))
    assert rel_err(m_p, g["m_p"]) < 1e-5
    assert rel_err(o, g["o"]) < 1e-4


def test_dec_matches_reference(synth_w):
    from oracle import synth as osynth

    g = golden("dec_b2_t24.npz")
    o = osynth.dec_only(synth_w, SYNTH_48K_V2, _t(g["z"]), _t(g["f0"]), _t(g["sid"]), _t(g["eps_src"]))
    assert rel_err(o, g["o"]) < 1e-4


def test_hubert_matches_reference(hubert_w):
    from oracle import hubert as ohub

    g = golden("hubert_1s.npz")
    f = ohub.hubert_forward(hubert_w, HUBERT_BASE, _t(g["audio"])[None])
    assert f.shape == g["feats"].shape
    assert rel_err(f, g["feats"]) < 1e-4


def test_rmvpe_matches_reference(rmvpe_w):
    from oracle import rmvpe as ormvpe

    g = golden("rmvpe_1s.npz")
    mel = ormvpe.mel_spectrogram(_t(g["audio"])[None])
    assert rel_err(mel, g["mel"]) < 1e-5
    f0, hidden = ormvpe.infer_from_audio(rmvpe_w, RMVPE_CFG, g["audio"])
    assert rel_err(hidden, g["hidden"]) < 1e-4
    np.testing.assert_array_equal(f0 > 0, g["f0"] > 0)
    assert np.max(np.abs(f0 - g["f0"])) < 1e-2


def test_rmvpe_decode_kat():
    """Known-answer test from the reference's ios_test_data: decode(hidden) == f0."""
    from oracle import rmvpe as ormvpe

    g = golden("ios_kat.npz")
    f0 = ormvpe.decode(g["rmvpe_hidden"][0], thred=0.03)
    assert f0.shape == g["rmvpe_f0"].shape
    assert np.max(np.abs(f0 - g["rmvpe_f0"])) < 1e-9
    assert int((f0 > 0).sum()) == int((g["rmvpe_f0"] > 0).sum())


def test_pipeline_matches_reference(synth_w, hubert_w, rmvpe_w):
    from oracle.metrics import spectrogram_correlation
    from oracle.pipeline import OraclePipeline

    g = golden("pipeline_2p5s.npz")
    draws = {"z": _t(g["eps_z"]), "src": _t(g["eps_src"])}
    pipe = OraclePipeline(48000, synth_w=synth_w, synth_cfg=SYNTH_48K_V2, hubert_w=hubert_w,
                          hubert_cfg=HUBERT_BASE, rmvpe_w=rmvpe_w, rmvpe_cfg=RMVPE_CFG,
                          noise_fn=lambda shape, which: draws[which].reshape(shape))
    out = pipe.pipeline(0, g["audio"].copy(), pitch=0, protect=0.33)
    assert out.shape == g["out"].shape
    assert rel_err(out, g["out"]) < 1e-3
    assert spectrogram_correlation(out, g["out"]) > 0.9999


def test_synth_nof0_matches_reference():
    """Models without pitch guidance (use_f0=False): TextEncoder without emb_pitch + HiFiGANGenerator, against
    the reference Synthesizer(use_f0=False).infer (tests/golden/make_golden_vocoders.py nof0)."""
    import dataclasses

    from oracle import synth as osynth
    from rvcx import synthetic
    from rvcx.weights import normalize_state

    g = golden("synth_nof0_b2.npz")
    cfg = dataclasses.replace(SYNTH_48K_V2, use_f0=False)
    w = normalize_state(synthetic.synth_state(int(g["seed_w"]), cfg))
    assert "enc_p.emb_pitch.weight" not in w and "dec.m_source.l_linear.weight" not in w
    o, mask, (z, z_p, m_p, logs_p) = osynth.synth_infer(w, cfg, _t(g["phone"]), _t(g["lengths"]), None, None,
                                                        _t(g["sid"]), _t(g["eps_z"]), None)
    assert rel_err(z_p, g["z_p"]) < 1e-5
    assert rel_err(z, g["z"]) < 1e-5
    assert rel_err(o, g["o"]) < 1e-4


def test_synth_mrf_matches_reference():
    """MRF HiFi-GAN decoder (9-harmonic source with per-sample phase accumulation, MRF blocks, conv_post bias)
    against the reference Synthesizer(vocoder="MRF HiFi-GAN").infer (make_golden_vocoders.py mrf)."""
    import dataclasses

    from oracle import synth as osynth
    from rvcx import synthetic
    from rvcx.weights import normalize_state

    g = golden("synth_mrf_b2.npz")
    cfg = dataclasses.replace(SYNTH_48K_V2, vocoder="MRF HiFi-GAN")
    w = normalize_state(synthetic.synth_state(int(g["seed_w"]), cfg))
    o, mask, (z, z_p, m_p, logs_p) = osynth.synth_infer(w, cfg, _t(g["phone"]), _t(g["lengths"]), _t(g["pitch"]),
                                                        _t(g["f0"]), _t(g["sid"]), _t(g["eps_z"]), _t(g["eps_src"]))
    assert rel_err(z, g["z"]) < 1e-5
    assert rel_err(o, g["o"]) < 1e-4, rel_err(o, g["o"])


def test_synth_refinegan_matches_reference():
    """RefineGAN decoder against the reference Synthesizer(vocoder="RefineGAN").infer (make_golden_vocoders.py;
    torchaudio's resample restated there and here: that piece is pinned to the restatement only)."""
    import dataclasses

    from oracle import synth as osynth
    from rvcx import synthetic
    from rvcx.weights import normalize_state

    g = golden("synth_refinegan_b1.npz")
    cfg = dataclasses.replace(SYNTH_48K_V2, vocoder="RefineGAN")
    w = normalize_state(synthetic.synth_state(int(g["seed_w"]), cfg))
    from conftest import refinegan_noise

    eps_z, eps_src = refinegan_noise(g)
    T = g["phone"].shape[1]
    o, mask, (z, z_p, m_p, logs_p) = osynth.synth_infer(w, cfg, _t(g["phone"]), _t(g["lengths"]), _t(g["pitch"]),
                                                        _t(g["f0"]), _t(g["sid"]),
                                                        _t(eps_z.reshape(1, cfg.inter_channels, T)), _t(eps_src))
    assert rel_err(z, g["z"]) < 1e-5
    assert rel_err(o, g["o"]) < 1e-4, rel_err(o, g["o"])
