"""split_audio (rvc/lib/tools/split_audio.py): the oracle's librosa.effects.split restatement on known answers,
and merge_audio's gap / duration-compensation arithmetic (rvcx.split, host output assembly)."""
import numpy as np

from oracle import split_audio as osplit


def test_effects_split_known_answer():
    sr = 16000
    t = np.arange(3 * sr) / sr
    y = 0.5 * np.sin(2 * np.pi * 220 * t)
    y[sr:2 * sr] = 0.0  # one second of digital silence in the middle
    segs, iv = osplit.process_audio(y, sr)
    # frames of 4000 every 2000 centred at 2000 k: silent where [2000k - 2000, 2000k + 2000) lies inside
    # [16000, 32000), i.e. k = 9..15; edges at frames 9 and 16 -> samples 18000 and 32000
    assert iv.tolist() == [[0, 18000], [32000, 48000]]
    assert len(segs) == 2 and len(segs[0]) == 18000


def test_merge_audio_gaps_and_compensation():
    from rvcx.split import merge_audio

    iv = np.array([[1600, 3200], [4800, 8000]])
    org = [np.ones(1600), np.ones(3200)]
    new = [np.full(4700, 2.0, np.float32), np.full(9700, 3.0, np.float32)]  # 48 kHz: -100 and +100 samples
    out = merge_audio(org, new, iv, 16000, 48000)
    # leading 4800 zeros, seg0, compensation after it (it got shorter), gap 14400 - 9600 = 4800 zeros,
    # compensation before seg1 (longer), seg1; compensation = int(|duration difference| * 48000) as the
    # reference computes it in float (99 here, not 100)
    c0 = int(abs(4700 / 48000 - 1600 / 16000) * 48000)
    c1 = int(abs(9700 / 48000 - 3200 / 16000) * 48000)
    assert out.dtype == np.float32
    assert len(out) == 4800 + 4700 + c0 + 4800 + c1 + 9700
    assert not out[:4800].any() and (out[4800:9500] == 2).all()
    z = 9500 + c0 + 4800 + c1
    assert not out[9500:z].any() and (out[z:] == 3).all()
