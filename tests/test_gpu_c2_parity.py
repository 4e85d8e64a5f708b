"""Parity at the headline config C2 (13.5 s, 216100 samples, x_pad = 1) against the REFERENCE itself:
tests/golden/pipeline_c2_{ios,synth}.npz hold rvc/infer/pipeline.py Pipeline.pipeline's output on the
reference's own real-speech clip (ios_test_data/input_audio.npy) and on the bench's C2 clip, with the
seeded synthetic weights, recorded noise and the RMVPE salience the reference decoded
(tests/golden/make_golden_sizes.py c2).

Tolerances (fp32 throughout, as the reference):
  * RMVPE: device salience vs the reference's (rel <= 1e-3 of the peak over the whole [1551, 360] matrix); an
    argmax that differs from the reference's only on frames whose reference top-1/top-2 margin is within twice
    the measured salience error; every other frame's f0 within the cents bound that error implies
    (tests/rmvpe_parity.py) -- a summation-order change can only fail this through a real salience error;
  * the pipeline's own f0 equals the standalone RMVPE call's on the same padded input (bitwise), and its output
    equals voice_conversion fed that f0, trimmed and normalised (rel <= 1e-6: the same kernels);
  * whole pipeline vs the reference: spectrogram correlation >= 0.999 (a sample-level bar here would measure the
    NSF phase drift of fp32-noise f0 differences, not the kernels);
  * voice_conversion fed the reference's pitch track (the strict sample-level gate): rel <= 1e-4;
  * HuBERT rel <= 1e-3 (fixture in fp16); the coarse pitch of the reference's own f0 bit-exact.
"""
import numpy as np
import pytest

from conftest import c2_audio, fixture_noise, golden
from rmvpe_parity import check_rmvpe, rel_err, trim_normalize

pytestmark = pytest.mark.gpu

CLIPS = ["ios", "synth"]


@pytest.mark.parametrize("clip", CLIPS)
def test_c2_pipeline_vs_reference(engine, clip):
    from oracle.metrics import spectrogram_correlation

    g = golden(f"pipeline_c2_{clip}.npz")
    ez, es = fixture_noise(g)
    engine.set_pipeline_highpass()
    audio = c2_audio(clip)
    out, f0p = engine.pipeline(audio, sid=0, semitones=0, protect=0.33, t_pad=16000, t_pad_tgt=48000, eps_z=ez,
                               eps_src=es, want_f0=True)
    _, p32 = engine.highpass_pad(audio, 16000)
    f0d, hid = engine.rmvpe(p32, want_hidden=True)
    engine.check_device_status()
    out, f0p, f0d, hid = (v.cpu().numpy() for v in (out, f0p, f0d, hid))
    np.testing.assert_array_equal(f0p, f0d)
    r = check_rmvpe(f0d, hid, g, g["f0_raw"])
    assert out.shape == g["out"].shape == (648000,)
    c = spectrogram_correlation(out, g["out"])
    assert c >= 0.999
    p_len = p32.shape[0] // 160
    coarse, pitchf, _ = engine.f0_post(f0d, 0.0)
    vc = engine.voice_conversion(p32, coarse[:p_len], pitchf[:p_len], 0, 0.33, eps_z=ez, eps_src=es).cpu().numpy()
    cons = rel_err(out, trim_normalize(vc))
    assert cons <= 1e-6, cons
    # sample-level bar where f0 cannot have drifted yet: the output up to 20 frames (the generator's
    # receptive field) before the first frame whose f0 may legitimately differ, at the round-2 bar rel <= 2e-3
    end = out.shape[0] if r["first_flip"] is None else max(0, (r["first_flip"] - 20) * 480 - 48000)
    if end >= 48000:
        pre = float(np.abs(out[:end] - g["out"][:end]).max() / (np.abs(g["out"]).max() + 1e-12))
        assert pre <= 2e-3, (pre, end)
    print(f"\nC2 {clip}: salience err {r['err']:.2e} (bound {3 * float(g['sal_fp32_noise']):.2e}), {r['n_near']} "
          f"near-tied frames, flips {list(r['flips'])}, spec corr {c:.6f}, rel to reference {rel_err(out, g['out']):.2e}, "
          f"pipeline vs staged {cons:.1e}")


@pytest.mark.parametrize("clip", CLIPS)
def test_c2_stages_vs_reference(engine, clip):
    g = golden(f"pipeline_c2_{clip}.npz")
    engine.set_pipeline_highpass()
    _, x = engine.highpass_pad(c2_audio(clip), 16000)
    coarse, pitchf, _ = engine.f0_post(g["f0_raw"], 0.0)
    assert np.array_equal(coarse.cpu().numpy(), g["pitch"])
    assert np.array_equal(pitchf.cpu().numpy(), g["f0_raw"].astype(np.float32))
    h = engine.hubert(x).cpu().numpy()
    assert h.shape == g["feats16"].shape == (775, 768)
    assert rel_err(h, g["feats16"].astype(np.float32)) <= 1e-3


@pytest.mark.parametrize("clip", CLIPS)
def test_c2_voice_conversion_on_reference_pitch(engine, clip):
    """HuBERT -> x2 upsample -> protect -> Synthesizer.infer on the full padded clip, fed the reference's own
    pitch / pitchf and noise, then the reference's trim and peak-normalise (pipeline.py:494, :550-552)."""
    from oracle.metrics import spectrogram_correlation

    g = golden(f"pipeline_c2_{clip}.npz")
    ez, es = fixture_noise(g)
    engine.set_pipeline_highpass()
    _, x = engine.highpass_pad(c2_audio(clip), 16000)
    p_len = x.shape[0] // 160
    vc = engine.voice_conversion(x, g["pitch"][:p_len], g["f0_raw"][:p_len].astype(np.float32), 0, 0.33, eps_z=ez,
                                 eps_src=es).cpu().numpy()
    vc = trim_normalize(vc)
    ref = g["out"]
    assert vc.shape == ref.shape
    assert spectrogram_correlation(vc, ref) >= 0.9999
    assert rel_err(vc, ref) <= 1e-4, rel_err(vc, ref)
