"""split_audio on device (rvcx_split_audio: frame RMS on the GPU, librosa.effects.split edges) vs the oracle's
librosa restatement, and RVCX.convert(split_audio=True) (rvc/infer/infer.py:282-316)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("thresh,min_len", [(-60, 250), (-40, 250), (-50, 100)])
def test_split_intervals_vs_oracle(engine, thresh, min_len):
    from oracle import split_audio as osplit
    from rvcx import synthetic
    from rvcx.split import process_audio

    y = synthetic.speech_like(5 * 16000, seed=9)
    y[16000:30000] *= 1e-4  # quiet stretches of different depths
    y[50000:56000] = 0.0
    y[70000:] *= 1e-2
    segs, iv = process_audio(engine, y, 16000, thresh, min_len)
    _, iv_o = osplit.process_audio(y, 16000, thresh, min_len)
    np.testing.assert_array_equal(iv, iv_o)
    assert all(len(s) == e - b for s, (b, e) in zip(segs, iv))


def test_convert_split_audio(engine, synth_w, hubert_w, rmvpe_w):
    from rvcx import synthetic
    from rvcx.infer import RVCX
    from rvcx.split import merge_audio, process_audio

    rv = RVCX(synth_state=synth_w, hubert_state=hubert_w, rmvpe_state=rmvpe_w)
    try:
        y = synthetic.speech_like(6 * 16000, seed=4)
        y[2 * 16000:3 * 16000 + 8000] = 0.0
        out = rv.convert(y, split_audio=True)
        chunks, iv = process_audio(rv.engine, y, 16000)
        assert len(iv) == 2
        parts = [rv.convert(c) for c in chunks]
        np.testing.assert_array_equal(out, merge_audio(chunks, parts, iv, 16000, rv.tgt_sr))
        assert np.isfinite(out).all()
    finally:
        rv.close()
