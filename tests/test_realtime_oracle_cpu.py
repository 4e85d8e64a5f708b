"""Streaming oracle (oracle/realtime.py) on CPU: torchaudio-restated resampler, Realtime.realloc geometry
and two hops of VoiceChanger.on_request (the device path is checked against it in test_gpu_stream.py)."""
import math

import numpy as np
import torch


def test_resample_kernel_and_lengths():
    from oracle.realtime import resample, sinc_resample_kernel

    k, width, orig, new = sinc_resample_kernel(48000, 16000)
    assert (orig, new, width) == (3, 1, 19) and tuple(k.shape) == (1, 1, 41)
    assert abs(float(k.sum()) - 1.0) < 1e-3  # unity DC gain
    for n in (12288, 12289, 1000):
        x = torch.randn(n)
        assert resample(x, 48000, 16000).shape[0] == math.ceil(n / 3)
    t = torch.arange(48000, dtype=torch.float32) / 48000
    y = resample(torch.sin(2 * math.pi * 1000 * t), 48000, 16000)
    ref = torch.sin(2 * math.pi * 1000 * torch.arange(16000, dtype=torch.float32) / 16000)
    assert float((y[100:-100] - ref[100:-100]).abs().max()) < 1e-2
    x = torch.randn(777)
    assert torch.equal(resample(x, 48000, 48000), x)
    k2, _, o2, n2 = sinc_resample_kernel(40000, 48000)
    assert (o2, n2) == (5, 6) and k2.shape[0] == 6


def test_oracle_stream_two_hops(synth_w, hubert_w, rmvpe_w):
    from oracle.realtime import OracleVoiceChanger
    from rvcx import synthetic
    from rvcx.config import HUBERT_BASE, RMVPE_CFG, SYNTH_48K_V2

    vc = OracleVoiceChanger(synth_w, SYNTH_48K_V2, hubert_w, HUBERT_BASE, rmvpe_w, RMVPE_CFG, read_chunk_size=96,
                            silent_threshold=-90)
    assert (vc.convert_feature_size_16k, vc.skip_head, vc.return_length) == (87, 50, 37)
    assert vc.convert_buffer.shape[0] == 13920 and vc.audio_buffer.shape[0] == 4096 + 1600
    x = synthetic.speech_like(12288 * 2, seed=3, sr=48000).astype(np.float32)
    torch.manual_seed(0)
    for h in range(2):
        out, vol = vc.on_request(x[h * 12288:(h + 1) * 12288])
        assert out.shape == (12288,) and np.isfinite(out).all() and vol > 0
        assert 0 <= vc.last["sola_offset"] <= 480


def test_oracle_stream_vs_reference_fixture(synth_w, hubert_w, rmvpe_w):
    """Pins oracle/realtime.py to the reference's own rvc/realtime run (tests/golden/stream_c5_16.npz, made by
    make_golden_stream.py): 4 of its 16 streams (incl. the gated one), all 6 hops, same inputs and noise."""
    import hashlib

    from conftest import golden
    from oracle.metrics import spectrogram_correlation
    from oracle.realtime import OracleVoiceChanger
    from rvcx import synthetic
    from rvcx.config import HUBERT_BASE, RMVPE_CFG, SYNTH_48K_V2

    g = golden("stream_c5_16.npz")
    S, H, blk = int(g["n_streams"]), int(g["hops"]), int(g["block"])
    x = np.stack([synthetic.speech_like(blk * H, seed=int(g["input_seed0"]) + s, sr=48000).astype(np.float32)
                  for s in range(S)])
    x[int(g["silent_stream"]), 2 * blk:4 * blk] = 0.0
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(g["input_sha256"])
    same = n = 0
    for s in (0, 5, 11, int(g["silent_stream"])):
        rng = np.random.Generator(np.random.PCG64(int(g["noise_seed0"]) + s))
        vc = OracleVoiceChanger(synth_w, SYNTH_48K_V2, hubert_w, HUBERT_BASE, rmvpe_w, RMVPE_CFG, read_chunk_size=96,
                                silent_threshold=-90, sid=int(g["sids"][s]),
                                noise_fn=lambda shape, which, rng=rng: torch.from_numpy(
                                    rng.standard_normal((1, *shape[1:]) if which == "z" else (1, shape[1], 1))
                                    .astype(np.float32).reshape(shape)))
        for h in range(H):
            out, vol = vc.on_request(x[s, h * blk:(h + 1) * blk].copy(), f0_up_key=int(g["f0_up_key"]),
                                     index_rate=0.0, protect=float(g["protect"]))
            ref = g["out16"][s, h].astype(np.float32)
            assert abs(vol - float(g["vol"][s, h])) <= 1e-6 * max(float(g["vol"][s, h]), 1e-12)
            n += 1
            same += int(vc.last["sola_offset"] == int(g["sola_offset"][s, h]))
            assert spectrogram_correlation(out, ref) >= 0.999, (s, h)
            if vc.last["sola_offset"] == int(g["sola_offset"][s, h]):
                assert float(np.abs(out - ref).max()) <= 2e-3 * max(1e-3, float(np.abs(ref).max())), (s, h)
    assert same >= 0.95 * n, (same, n)
