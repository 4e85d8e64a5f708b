"""Models without pitch guidance (cpt["f0"] == 0) on the device: Synthesizer.infer against the reference's own
Synthesizer(use_f0=False) (tests/golden/synth_nof0_b2.npz, make_golden_vocoders.py), and the whole pipeline with
pitch_guidance=False (no RMVPE, no protect, rvc/infer/pipeline.py:324-365, :461-512) against the CPU oracle.
The reference's own no-f0 pipeline branch cannot run (pipeline.py:370 calls pitchf.float() on None), so the
pipeline-level check is against the oracle's evident restatement; the model itself is pinned by the fixture."""
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
def nof0_engine(hubert_w, rmvpe_w):
    from rvcx import synthetic
    from rvcx.config import SYNTH_48K_V2
    from rvcx.engine import Engine
    from rvcx.weights import normalize_state

    g = golden("synth_nof0_b2.npz")
    cfg = dataclasses.replace(SYNTH_48K_V2, use_f0=False)
    w = normalize_state(synthetic.synth_state(int(g["seed_w"]), cfg))
    e = Engine(0)
    e.load_synth(w, cfg)
    e.load_hubert(hubert_w)
    e.load_rmvpe(rmvpe_w)
    yield e, w, cfg
    e.close()


def test_nof0_synth_vs_reference(nof0_engine):
    from oracle.metrics import spectrogram_correlation

    eng, _, _ = nof0_engine
    g = golden("synth_nof0_b2.npz")
    out, zp, z = eng.synth_infer(g["phone"], g["lengths"], None, None, g["sid"], eps_z=g["eps_z"],
                                 want_latents=True)
    torch.cuda.synchronize()
    assert rel_err(zp.cpu().numpy().transpose(0, 2, 1), g["z_p"]) < 1e-4
    assert rel_err(z.cpu().numpy().transpose(0, 2, 1), g["z"]) < 1e-4
    o = out.cpu().numpy()
    ref = g["o"].reshape(o.shape)
    assert rel_err(o, ref) < 2e-3, rel_err(o, ref)
    for b in range(o.shape[0]):
        assert spectrogram_correlation(o[b], ref[b]) > 0.999


def test_nof0_pipeline_vs_oracle(nof0_engine, hubert_w, rmvpe_w):
    from oracle.metrics import spectrogram_correlation
    from oracle.pipeline import OraclePipeline
    from rvcx import synthetic
    from rvcx.config import HUBERT_BASE, RMVPE_CFG
    from rvcx.infer.models import HubertModel, Synthesizer
    from rvcx.infer.pipeline import Config, PipelineMLX

    eng, w, cfg = nof0_engine
    audio = synthetic.speech_like(40000, seed=77)
    m = 40000 + 2 * 16000
    T = min(m // 160, 2 * HUBERT_BASE.frames(m))  # p_len = min(len // 160, 2 L) frames (pipeline.py:346)
    rng = np.random.Generator(np.random.PCG64(78))
    eps_z = rng.standard_normal((1, cfg.inter_channels, T)).astype(np.float32)
    pipe = PipelineMLX(48000, Config(), HubertModel(eng), None)
    with pytest.raises(ValueError):  # pitch_guidance must match the model
        pipe.pipeline(HubertModel(eng), Synthesizer(eng), 0, audio, pitch_guidance=True)
    out = pipe.pipeline(HubertModel(eng), Synthesizer(eng), 0, audio, pitch_guidance=False, protect=0.33,
                        eps_z=eps_z)
    eng.check_device_status()

    class NoRmvpe(OraclePipeline):
        def get_f0(self, *a, **k):
            raise AssertionError("no f0 without pitch guidance")

        def pipeline(self, sid, audio, **kw):  # pipeline.py:390-558 with pitch_guidance False, one chunk
            from scipy import signal

            from oracle.pipeline import AH, BH

            x = signal.filtfilt(BH, AH, audio)
            x = np.pad(x, (self.t_pad, self.t_pad), mode="reflect")
            y = self.voice_conversion(torch.tensor([sid]).long(), x, None, None, 0.33)[self.t_pad_tgt:-self.t_pad_tgt]
            m = np.abs(y).max() / 0.99
            return y / m if m > 1 else y

        def voice_conversion(self, sid, audio0, pitch, pitchf, protect, version="v2", index=None, index_rate=0.0):
            import torch.nn.functional as F

            from oracle import hubert as ohubert
            from oracle import synth as osynth

            with torch.no_grad():
                feats = ohubert.hubert_forward(self.hw, self.hc, torch.from_numpy(audio0).float().view(1, -1), version)
                feats = F.interpolate(feats.permute(0, 2, 1), scale_factor=2).permute(0, 2, 1)
                p_len = min(audio0.shape[0] // self.window, feats.shape[1])
                Tn = feats.shape[1]
                o = osynth.synth_infer(self.sw, self.sc, feats.float(), torch.tensor([p_len]).long(), None, None, sid,
                                       self.noise_fn((1, self.sc.inter_channels, Tn), "z"), None)[0]
                return o[0, 0].float().numpy()

    orc = NoRmvpe(48000, synth_w=w, synth_cfg=cfg, hubert_w=hubert_w, hubert_cfg=HUBERT_BASE, rmvpe_w=rmvpe_w,
                  rmvpe_cfg=RMVPE_CFG, noise_fn=lambda shape, which: torch.from_numpy(eps_z).reshape(shape))
    ref = orc.pipeline(0, audio.astype(np.float64).copy())
    assert out.shape == ref.shape, (out.shape, ref.shape)
    assert spectrogram_correlation(out, ref) >= 0.999
    assert rel_err(out, ref) <= 2e-3, rel_err(out, ref)
