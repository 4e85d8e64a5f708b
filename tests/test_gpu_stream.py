"""Streaming path (rvcx.realtime: StreamGroup / VoiceChanger through rvcx_rt_process) vs the oracle
restatement of rvc/realtime (oracle/realtime.py), hop by hop, with the same injected noise.
Bar: geometry identical; vol rel <= 1e-5; SOLA offsets equal on >= 75 % of hops (a 1-sample move of
a flat correlation peak is a float32 tie); per-hop output spectrogram correlation >= 0.99 and the
silent-stream hops exact."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _noise(rng, B, I, T, upp):
    return (rng.standard_normal((B, I, T)).astype(np.float32), rng.standard_normal((B, T * upp)).astype(np.float32))


@pytest.mark.parametrize("protect,threshold", [(0.5, -90.0), (0.33, -45.0)])
def test_stream_group_matches_oracle(engine, synth_w, hubert_w, rmvpe_w, protect, threshold):
    from oracle.metrics import spectrogram_correlation
    from oracle.realtime import OracleVoiceChanger
    from rvcx import synthetic
    from rvcx.config import HUBERT_BASE, RMVPE_CFG, SYNTH_48K_V2
    from rvcx.realtime import StreamGroup

    B, hops = 3, 4
    grp = StreamGroup(engine, B, read_chunk_size=96, cross_fade_overlap_size=0.1, extra_convert_size=0.5,
                      silent_threshold=threshold, sid=[0, 1, 2])
    g = grp.geometry
    assert (g["block48"], g["block16"], g["convert16"], g["frames"], g["skip_head"], g["return_length"]) == \
        (12288, 4096, 13920, 87, 50, 37)
    block = g["block48"]
    audio = np.stack([synthetic.speech_like(block * hops, seed=60 + b, sr=48000).astype(np.float32)
                      for b in range(B)])
    audio[1, : 2 * block] *= 1e-4  # stream 1 is quiet for two hops (gated when threshold = -45 dB)
    orc = [OracleVoiceChanger(synth_w, SYNTH_48K_V2, hubert_w, HUBERT_BASE, rmvpe_w, RMVPE_CFG, read_chunk_size=96,
                              silent_threshold=threshold, sid=b) for b in range(B)]
    assert orc[0].convert_feature_size_16k == 87 and orc[0].skip_head == 50
    rng = np.random.default_rng(7)
    I, T, upp = SYNTH_48K_V2.inter_channels, g["frames"], SYNTH_48K_V2.upp
    same_off, n_off = 0, 0
    for h in range(hops):
        x = audio[:, h * block:(h + 1) * block]
        ez, es = _noise(rng, B, I, T, upp)
        out, vol = grp.process(x, grp.opts(protect=protect), eps_z=ez, eps_src=es)
        torch.cuda.synchronize()
        out, vol, offs = out.cpu().numpy(), vol.cpu().numpy(), grp.offs.cpu().numpy()
        for b in range(B):
            it = iter([torch.from_numpy(ez[b:b + 1]), torch.from_numpy(es[b:b + 1])])
            orc[b].noise_fn = lambda shape, which, it=it: next(it)
            ref, rvol = orc[b].on_request(x[b].copy(), protect=protect)
            assert abs(vol[b] - rvol) <= 1e-5 * max(rvol, 1e-12), (h, b, vol[b], rvol)
            if not np.any(ref):
                np.testing.assert_array_equal(out[b], ref)
                continue
            n_off += 1
            same_off += int(offs[b] == orc[b].last["sola_offset"])
            assert spectrogram_correlation(out[b], ref) > 0.99, (h, b)
    assert same_off >= 0.75 * n_off, (same_off, n_off)
    grp.close()


def test_voice_changer_api(engine):
    from rvcx import synthetic
    from rvcx.realtime import VoiceChanger

    vc = VoiceChanger(96, 0.1, 0.5, engine=engine, silent_threshold=-90)
    x = synthetic.speech_like(12288 * 2, seed=5, sr=48000).astype(np.float32)
    for h in range(2):
        res, vol, lat = vc.on_request(x[h * 12288:(h + 1) * 12288])
        assert res.shape == (12288,) and res.dtype == np.float32 and np.isfinite(res).all()
        assert vol > 0 and len(lat) == 3 and lat[1] > 0
    with pytest.raises(ValueError):
        vc.on_request(x[:1000])
    vc.close()
