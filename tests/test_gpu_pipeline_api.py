"""Drop-in API (rvcx.infer: PipelineMLX / RVC_MLX names) and the full Pipeline.pipeline options on
device vs the CPU oracle (oracle/pipeline.py, itself pinned to the reference's pipeline fixture),
with the same injected noise: long-input splitting, autotune, proposed pitch, volume envelope."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


class NoiseRecorder:
    """noise_fn for OraclePipeline: seeded draws, kept in call order for the device run."""

    def __init__(self, seed):
        self.rng = np.random.default_rng(seed)
        self.z, self.src = [], []

    def __call__(self, shape, which):
        a = self.rng.standard_normal(shape).astype(np.float32)
        (self.z if which == "z" else self.src).append(a.reshape(-1))
        return torch.from_numpy(a)

    def cat(self):
        return np.concatenate(self.z), np.concatenate(self.src)


def oracle_pipeline(synth_w, hubert_w, rmvpe_w, noise, **cfg):
    from oracle.pipeline import OraclePipeline
    from rvcx.config import HUBERT_BASE, RMVPE_CFG, SYNTH_48K_V2

    return OraclePipeline(48000, synth_w=synth_w, synth_cfg=SYNTH_48K_V2, hubert_w=hubert_w, hubert_cfg=HUBERT_BASE,
                          rmvpe_w=rmvpe_w, rmvpe_cfg=RMVPE_CFG, noise_fn=noise, **cfg)


@pytest.fixture(scope="module")
def api(engine):
    from rvcx.infer import Config, HubertModel, PipelineMLX, RMVPE0Predictor, Synthesizer

    hub, rm, net_g = HubertModel(engine), RMVPE0Predictor(engine), Synthesizer(engine)
    return hub, rm, net_g, PipelineMLX, Config


def test_pipeline_api_matches_reference_fixture(api):
    """PipelineMLX.pipeline (reference signature) reproduces the reference's pipeline output."""
    from oracle.metrics import spectrogram_correlation

    hub, rm, net_g, PipelineMLX, Config = api
    g = golden("pipeline_2p5s.npz")
    pipe = PipelineMLX(48000, Config(), hub, rm)
    out = pipe.pipeline(hub, net_g, 0, g["audio"], 0, "rmvpe", None, 0.0, True, 1.0, "v2", 0.33, False, 1.0,
                        False, 155.0, eps_z=g["eps_z"], eps_src=g["eps_src"])
    assert isinstance(out, np.ndarray) and out.dtype == np.float32
    assert out.shape == g["out"].shape
    assert spectrogram_correlation(out, g["out"]) > 0.995


def test_get_f0_and_voice_conversion_api(api, synth_w, hubert_w, rmvpe_w):
    from oracle.metrics import cents_agreement, spectrogram_correlation

    hub, rm, net_g, PipelineMLX, Config = api
    g = golden("pipeline_2p5s.npz")
    from scipy import signal

    from oracle.pipeline import AH, BH

    x = np.pad(signal.filtfilt(BH, AH, g["audio"]), (16000, 16000), mode="reflect")
    pipe = PipelineMLX(48000, Config(), hub, rm)
    p_len = x.shape[0] // 160
    coarse, f0 = pipe.get_f0(x, p_len, "rmvpe", 3)
    noise = NoiseRecorder(21)
    orc = oracle_pipeline(synth_w, hubert_w, rmvpe_w, noise)
    oc, of0 = orc.get_f0(x, p_len, 3)
    assert coarse.dtype == np.int64 and coarse.shape == oc.shape
    acc, vuv = cents_agreement(f0, of0, 50.0)
    assert acc >= 0.99 and vuv >= 0.995, (acc, vuv)
    assert np.mean(coarse == oc) > 0.98
    # one chunk through voice_conversion with the oracle's own pitch track and noise
    pc = torch.tensor(oc[:p_len]).unsqueeze(0).long()
    pf = torch.tensor(of0[:p_len]).unsqueeze(0).float()
    ref = orc.voice_conversion(torch.tensor([0]).long(), x, pc, pf, 0.33)
    ez, es = noise.cat()
    out = pipe.voice_conversion(hub, net_g, np.array([0]), x, oc[:p_len], of0[:p_len].astype(np.float32), None,
                                None, 0.0, "v2", 0.33, eps_z=ez, eps_src=es)
    assert out.shape == ref.shape
    assert spectrogram_correlation(out, ref) > 0.995


def test_pipeline_long_input_splits_like_reference(engine, synth_w, hubert_w, rmvpe_w):
    """opt_ts splitting (pipeline.py:440-512) with shrunk x_query/x_center/x_max so an 8 s clip is cut
    twice; same noise per chunk. Equal output length means the same split points were chosen."""
    from oracle.metrics import spectrogram_correlation
    from rvcx import synthetic

    audio = synthetic.speech_like(8 * 16000, seed=33)
    noise = NoiseRecorder(5)
    orc = oracle_pipeline(synth_w, hubert_w, rmvpe_w, noise, x_pad=1, x_query=1, x_center=3, x_max=4)
    ref = orc.pipeline(0, audio.copy(), protect=0.33)
    ez, es = noise.cat()
    assert len(noise.z) == 3  # two split points -> three chunks
    opts = engine.pipeline_opts(sid=0, protect=0.33, t_pad=16000, t_pad_tgt=48000, t_query=16000, t_center=48000,
                                t_max=64000)
    out = engine.pipeline_ex(audio, opts, eps_z=ez, eps_src=es).cpu().numpy()
    assert out.shape == ref.shape
    assert spectrogram_correlation(out, ref) > 0.99


@pytest.mark.parametrize("case", ["autotune", "proposed_pitch", "volume_envelope"])
def test_pipeline_options_vs_oracle(engine, synth_w, hubert_w, rmvpe_w, case):
    from oracle.metrics import cents_agreement, spectrogram_correlation

    g = golden("pipeline_2p5s.npz")
    kw = {"autotune": dict(f0_autotune=True, f0_autotune_strength=0.8),
          "proposed_pitch": dict(proposed_pitch=True, proposed_pitch_threshold=220.0),
          "volume_envelope": dict(volume_envelope=0.5)}[case]
    noise = NoiseRecorder(9)
    orc = oracle_pipeline(synth_w, hubert_w, rmvpe_w, noise)
    ref = orc.pipeline(0, g["audio"].copy(), pitch=2, protect=0.33, **kw)
    ez, es = noise.cat()
    ckw = dict(kw)
    for k in ("f0_autotune", "proposed_pitch"):
        if k in ckw:
            ckw[k] = int(ckw[k])
    opts = engine.pipeline_opts(sid=0, pitch=2.0, protect=0.33, **ckw)
    out, f0 = engine.pipeline_ex(g["audio"], opts, eps_z=ez, eps_src=es, want_f0=True)
    out = out.cpu().numpy()
    f0 = f0.cpu().numpy()[: len(orc.last["pitchf"])]
    acc, vuv = cents_agreement(f0, orc.last["pitchf"], 50.0)
    assert acc >= 0.99 and vuv >= 0.995, (acc, vuv)
    assert out.shape == ref.shape
    assert spectrogram_correlation(out, ref) > 0.99


def test_pipeline_mlx_semantics_runs(api):
    hub, rm, net_g, PipelineMLX, Config = api
    g = golden("pipeline_2p5s.npz")
    pipe = PipelineMLX(48000, Config(), hub, rm, semantics="mlx")
    out = pipe.pipeline(hub, net_g, 0, g["audio"], 0, "rmvpe", None, 0.0, True, 1.0, "v2", 0.33, True, 1.0,
                        False, 155.0)
    from rvcx.config import HUBERT_BASE

    m = g["audio"].shape[0] + 3200  # t_pad forced to 1600 (pipeline_mlx.py:318)
    T = min(m // 160, 2 * HUBERT_BASE.frames(m))
    assert out.shape[0] == T * net_g.dec.upp - 2 * 4800
    assert np.isfinite(out).all() and np.abs(out).max() <= 0.99 + 1e-6


def test_unsupported_options_raise(api):
    hub, rm, net_g, PipelineMLX, Config = api
    for m in ("harvest", "dio", "pm"):  # pyworld CPU methods: outside this path
        with pytest.raises(ValueError):
            PipelineMLX(48000, Config(), hub, rm, f0_method=m)
    with pytest.raises(ValueError):  # torchfcpe on the rvc/ path (the MLX port's fcpe is its RMVPE fallback)
        PipelineMLX(48000, Config(), hub, rm, f0_method="fcpe")
    pipe = PipelineMLX(48000, Config(), hub, rm)
    with pytest.raises(ValueError):  # pitch_guidance=False with a pitch-guided model (the reference crashes there)
        pipe.pipeline(hub, net_g, 0, np.zeros(32000), 0, "rmvpe", None, 0.0, False, 1.0, "v2", 0.33, False, 1.0,
                      False, 155.0)


def test_pipeline_batch_matches_single(engine):
    """rvcx_pipeline_batch (C4: B equal-length utterances in one batched pass) == rvcx_pipeline_ex per
    utterance with the same noise (up to split-K summation order), per-utterance sid and pitch shift."""
    from oracle.metrics import spectrogram_correlation
    from rvcx import synthetic

    engine.set_pipeline_highpass()
    B, n = 3, 40000
    audio = np.stack([synthetic.speech_like(n, seed=90 + b) for b in range(B)])
    opts = engine.pipeline_opts(pitch=2.0, protect=0.33)
    upp = engine.upp
    sids = [0, 3, 7]
    n_out = engine.pipeline_batch(audio, opts, sids=sids).shape[1]
    T = (n_out + 2 * 48000) // upp  # p_len = min(len // 160, 2L): the synthesizer's frame count
    assert T <= (n + 2 * 16000) // 160 and T * upp == n_out + 2 * 48000
    rng = np.random.default_rng(3)
    ez = rng.standard_normal((B, 192, T)).astype(np.float32)
    es = rng.standard_normal((B, T * upp)).astype(np.float32)
    yb = engine.pipeline_batch(audio, opts, sids=sids, eps_z=ez, eps_src=es).cpu().numpy()
    for b in range(B):
        o1 = engine.pipeline_opts(pitch=2.0, protect=0.33, sid=sids[b])
        y1 = engine.pipeline_ex(audio[b], o1, eps_z=ez[b], eps_src=es[b]).cpu().numpy()
        assert y1.shape == yb[b].shape
        assert spectrogram_correlation(yb[b], y1) > 0.999
        assert float(np.abs(yb[b] - y1).max()) < 5e-3 * max(float(np.abs(y1).max()), 1e-6)


def test_pipeline_batch_vs_reference_and_oracle(engine, synth_w, hubert_w, rmvpe_w):
    """C4's batched pass (rvcx_pipeline_batch) against references, not only against itself: row 0 is the
    reference fixture clip (tests/golden/pipeline_2p5s.npz: rvc Pipeline.pipeline output), rows 1-2 are other
    clips of the same length against the CPU oracle pipeline, each with its own noise and sid 0."""
    from oracle.metrics import spectrogram_correlation
    from rvcx import synthetic

    def rel(a, b):
        return float(np.abs(np.asarray(a, np.float64) - b).max() / (np.abs(b).max() + 1e-12))

    engine.set_pipeline_highpass()
    g = golden("pipeline_2p5s.npz")
    n = g["audio"].shape[0]
    clips = [g["audio"], synthetic.speech_like(n, seed=91), synthetic.speech_like(n, seed=92)]
    refs, ez, es = [g["out"]], [g["eps_z"].reshape(-1)], [g["eps_src"].reshape(-1)]
    for b in (1, 2):
        noise = NoiseRecorder(40 + b)
        orc = oracle_pipeline(synth_w, hubert_w, rmvpe_w, noise)
        refs.append(orc.pipeline(0, clips[b].copy(), protect=0.33))
        z, s = noise.cat()
        ez.append(z)
        es.append(s)
    opts = engine.pipeline_opts(protect=0.33)
    yb = engine.pipeline_batch(np.stack(clips), opts, sids=0, eps_z=np.stack(ez), eps_src=np.stack(es))
    engine.check_device_status()
    yb = yb.cpu().numpy()
    for b in range(3):
        assert yb[b].shape == refs[b].shape
        assert spectrogram_correlation(yb[b], refs[b]) >= 0.999
        assert rel(yb[b], refs[b]) <= 2e-3, (b, rel(yb[b], refs[b]))
