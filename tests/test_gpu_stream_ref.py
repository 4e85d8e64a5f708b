"""Streaming (C5) against the REFERENCE's own realtime code: tests/golden/stream_c5_16.npz holds
rvc/realtime VoiceChanger.on_request outputs for 16 independent streams x 6 hops at the C5 geometry
(256 ms hops, read_chunk_size 96), run in the survey container by tests/golden/make_golden_stream.py with
the seeded weights and recorded noise (torchaudio's Resample being the one restated piece).

The device converts all 16 streams per hop in ONE rvcx_rt_process call (StreamGroup, batched RMVPE /
HuBERT / Synthesizer.infer / SOLA). Bar: vol rel <= 1e-5; SOLA offsets equal on >= 95 %
of the voiced hops; per-hop output spectrogram correlation >= 0.999 and max |diff| <= 2e-3 of the hop's peak
(the fixture is stored in fp16: 5e-4 relative); gated (silent) hops: offset 0 and the crossfade tail.
"""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def _inputs(g):
    import hashlib

    from rvcx import synthetic

    S, H, blk = int(g["n_streams"]), int(g["hops"]), int(g["block"])
    x = np.stack([synthetic.speech_like(blk * H, seed=int(g["input_seed0"]) + s, sr=48000).astype(np.float32)
                  for s in range(S)])
    x[int(g["silent_stream"]), 2 * blk:4 * blk] = 0.0
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(g["input_sha256"]), "regenerated inputs differ"
    return x


def test_stream_group_16_matches_reference(engine):
    from oracle.metrics import spectrogram_correlation
    from rvcx.config import SYNTH_48K_V2
    from rvcx.realtime import StreamGroup

    g = golden("stream_c5_16.npz")
    S, H, blk = int(g["n_streams"]), int(g["hops"]), int(g["block"])
    x = _inputs(g)
    grp = StreamGroup(engine, S, read_chunk_size=96, cross_fade_overlap_size=0.1, extra_convert_size=0.5,
                      silent_threshold=-90.0, sid=[int(v) for v in g["sids"]])
    geo = grp.geometry
    assert (geo["block48"], geo["convert16"], geo["frames"], geo["skip_head"], geo["return_length"]) == \
        (blk, 13920, 87, 50, 37)
    T, I, upp = geo["frames"], SYNTH_48K_V2.inter_channels, SYNTH_48K_V2.upp
    rngs = [np.random.Generator(np.random.PCG64(int(g["noise_seed0"]) + s)) for s in range(S)]
    opts = grp.opts(f0_up_key=float(g["f0_up_key"]), protect=float(g["protect"]), index_rate=0.0)
    same, voiced = 0, 0
    for h in range(H):
        ez = np.empty((S, I, T), np.float32)
        es = np.empty((S, T * upp), np.float32)
        for s in range(S):
            ez[s] = rngs[s].standard_normal((1, I, T)).astype(np.float32)[0]
            es[s] = rngs[s].standard_normal((1, T * upp, 1)).astype(np.float32).reshape(-1)
        out, vol = grp.process(x[:, h * blk:(h + 1) * blk], opts, eps_z=ez, eps_src=es)
        torch.cuda.synchronize()
        out, vol, offs = out.cpu().numpy(), vol.cpu().numpy(), grp.offs.cpu().numpy()
        for s in range(S):
            ref = g["out16"][s, h].astype(np.float32)
            rv = float(g["vol"][s, h])
            assert abs(float(vol[s]) - rv) <= 1e-5 * max(rv, 1e-12), (h, s, vol[s], rv)
            if rv == 0.0:  # gated hop: zeros through SOLA -> offset 0, output = the crossfade tail
                assert offs[s] == 0 == int(g["sola_offset"][s, h])
                np.testing.assert_allclose(out[s], ref, atol=2e-3 * max(1e-3, float(np.abs(ref).max())))
                continue
            if h == 0:  # first hop: the SOLA buffer is zeros, every offset ties at 0
                assert offs[s] == int(g["sola_offset"][s, h]) == 0
            voiced += 1
            same += int(offs[s] == int(g["sola_offset"][s, h]))
            if offs[s] == int(g["sola_offset"][s, h]):
                peak = float(np.abs(ref).max())
                assert float(np.abs(out[s] - ref).max()) <= 2e-3 * peak, (h, s, float(np.abs(out[s] - ref).max()), peak)
            assert spectrogram_correlation(out[s], ref) >= 0.999, (h, s)
    engine.check_device_status()
    assert same >= 0.95 * voiced, (same, voiced)
    grp.close()


def test_stream_group_16_generator_fp16_gate(engine):
    """The opt-in half-precision generator for BASELINE C5's fp16 streaming (rvcx_rt_opts.gen_precision = 1: fp16
    operands, fp32 accumulation in the generator's weight-streamed convs and fused ResBlock pairs; RMVPE / HuBERT /
    TextEncoder / flow fp32-accurate), against the same fp32 reference fixture: gate v of SURVEY §8(d), per-hop
    spectrogram correlation >= 0.986 on every voiced hop; volumes (front end, fp32) stay exact. The setting travels
    with the hop: an fp32 hop and an offline call on the same context afterwards are unaffected."""
    from oracle.metrics import spectrogram_correlation
    from rvcx.config import SYNTH_48K_V2
    from rvcx.realtime import StreamGroup

    g = golden("stream_c5_16.npz")
    S, H, blk = int(g["n_streams"]), int(g["hops"]), int(g["block"])
    x = _inputs(g)
    grp = StreamGroup(engine, S, read_chunk_size=96, cross_fade_overlap_size=0.1, extra_convert_size=0.5,
                      silent_threshold=-90.0, sid=[int(v) for v in g["sids"]])
    # the same streams at fp32 on a second group: the fp16 hops must differ from them (the mode is active) by
    # fp16-operand rounding, not by more
    g32 = StreamGroup(engine, S, read_chunk_size=96, cross_fade_overlap_size=0.1, extra_convert_size=0.5,
                      silent_threshold=-90.0, sid=[int(v) for v in g["sids"]])
    T, I, upp = grp.geometry["frames"], SYNTH_48K_V2.inter_channels, SYNTH_48K_V2.upp
    rngs = [np.random.Generator(np.random.PCG64(int(g["noise_seed0"]) + s)) for s in range(S)]
    opts = grp.opts(f0_up_key=float(g["f0_up_key"]), protect=float(g["protect"]), index_rate=0.0,
                    gen_precision="fp16")
    opts32 = g32.opts(f0_up_key=float(g["f0_up_key"]), protect=float(g["protect"]), index_rate=0.0)
    corrs, dev16 = [], []
    for h in range(H):
        ez = np.empty((S, I, T), np.float32)
        es = np.empty((S, T * upp), np.float32)
        for s in range(S):
            ez[s] = rngs[s].standard_normal((1, I, T)).astype(np.float32)[0]
            es[s] = rngs[s].standard_normal((1, T * upp, 1)).astype(np.float32).reshape(-1)
        out, vol = grp.process(x[:, h * blk:(h + 1) * blk], opts, eps_z=ez, eps_src=es)
        out32, _ = g32.process(x[:, h * blk:(h + 1) * blk], opts32, eps_z=ez, eps_src=es)
        torch.cuda.synchronize()
        out, vol, out32 = out.cpu().numpy(), vol.cpu().numpy(), out32.cpu().numpy()
        for s in range(S):
            rv = float(g["vol"][s, h])
            assert abs(float(vol[s]) - rv) <= 1e-5 * max(rv, 1e-12), (h, s, vol[s], rv)
            if rv == 0.0:
                continue
            ref = g["out16"][s, h].astype(np.float32)
            c = spectrogram_correlation(out[s], ref)
            corrs.append(c)
            dev16.append(float(np.abs(out[s] - out32[s]).max() / max(float(np.abs(out32[s]).max()), 1e-12)))
            assert c >= 0.986, (h, s, c)
    engine.check_device_status()
    grp.close()
    g32.close()
    # the fp16 mode is active (the hops differ from the fp32 ones beyond fp32 rounding) and stays within fp16
    # operand rounding of them
    assert 1e-6 < max(dev16) < 5e-2, max(dev16)
    print(f"\ngenerator fp16: {len(corrs)} voiced hops, spec corr min {min(corrs):.5f} mean {np.mean(corrs):.5f}, "
          f"max rel diff to the fp32 hops {max(dev16):.2e}")


def test_generator_precision_stays_with_the_hop(engine):
    """the fp16 generator is a per-hop option, not context state. After fp16 hops on a context,
    an offline synthesizer call on the same context must stay fp32-accurate (bit-identical to the same call made
    before the fp16 hops)."""
    from rvcx import synthetic
    from rvcx.realtime import StreamGroup

    rng = np.random.Generator(np.random.PCG64(77))
    T = 48
    phone = rng.standard_normal((1, T, 768)).astype(np.float32)
    f0 = synthetic.f0_walk(1, T, seed=9)
    pitch = rng.integers(1, 256, size=(1, T)).astype(np.int64)
    ez = rng.standard_normal((1, 192, T)).astype(np.float32)
    es = rng.standard_normal((1, T * 480)).astype(np.float32)
    before = engine.synth_infer(phone, [T], pitch, f0, [0], eps_z=ez, eps_src=es).cpu().numpy()
    grp = StreamGroup(engine, 2, read_chunk_size=96, cross_fade_overlap_size=0.1, extra_convert_size=0.5,
                      silent_threshold=-90.0)
    x = np.stack([synthetic.speech_like(grp.block_frame, seed=3 + s, sr=48000).astype(np.float32) for s in range(2)])
    grp.process(x, grp.opts(gen_precision="fp16"))
    torch.cuda.synchronize()
    grp.close()
    after = engine.synth_infer(phone, [T], pitch, f0, [0], eps_z=ez, eps_src=es).cpu().numpy()
    assert np.array_equal(before, after)
