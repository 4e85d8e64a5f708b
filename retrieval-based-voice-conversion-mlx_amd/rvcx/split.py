"""split_audio (rvc/lib/tools/split_audio.py) on the device engine.

``process_audio(engine, audio, sr, silence_thresh, min_silence_len)`` -> (segments, intervals): the non-silent
intervals of librosa.effects.split (frame RMS on device, rvcx_split_audio) and the segments they cut.
``merge_audio(org, new, intervals, sr_orig, sr_new)`` re-assembles converted segments with the silent gaps
restored (split_audio.py:29-79; output assembly only: zeros and copies at the same offsets).
"""
from __future__ import annotations

import ctypes

import numpy as np


def split_intervals(engine, audio, sr: int = 16000, silence_thresh: float = -60, min_silence_len: int = 250):
    t = engine.torch
    a = engine._dev(audio, t.float64).reshape(-1)
    n = a.numel()
    frame = int(min_silence_len / 1000 * sr)
    cap = max(1, n // max(1, frame // 2) // 2 + 2)
    iv = np.zeros((cap, 2), dtype=np.int64)
    cnt = ctypes.c_int64(0)
    engine._check(engine.lib.rvcx_split_audio(engine.ctx, a.data_ptr(), n, int(sr), float(silence_thresh),
                                              int(min_silence_len), iv.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                              cap, ctypes.byref(cnt), engine.stream()), "split_audio")
    return iv[: cnt.value]


def process_audio(engine, audio, sr: int = 16000, silence_thresh: float = -60, min_silence_len: int = 250):
    """split_audio.process_audio (:5-27)."""
    intervals = split_intervals(engine, audio, sr, silence_thresh, min_silence_len)
    return [audio[s:e] for s, e in intervals], intervals


def merge_audio(audio_segments_org, audio_segments_new, intervals, sr_orig, sr_new):
    """split_audio.merge_audio (:29-79): leading silence, per-segment duration compensation (before the segment
    when it got shorter, after it when longer), the original gaps between segments, all at sr_new."""
    dt = np.asarray(audio_segments_new[0]).dtype
    parts = []
    ratio = sr_new / sr_orig
    for i, (start, end) in enumerate(intervals):
        start_new, end_new = int(start * ratio), int(end * ratio)
        diff = len(audio_segments_new[i]) / sr_new - len(audio_segments_org[i]) / sr_orig
        comp = np.zeros(int(abs(diff) * sr_new), dtype=dt)
        if i == 0 and start_new > 0:
            parts.append(np.zeros(start_new, dtype=dt))
        if diff > 0:
            parts.append(comp)
        parts.append(np.asarray(audio_segments_new[i], dtype=dt))
        if diff < 0:
            parts.append(comp)
        if i < len(intervals) - 1:
            gap = int(intervals[i + 1][0] * ratio) - end_new
            if gap > 0:
                parts.append(np.zeros(gap, dtype=dt))
    return np.concatenate(parts) if parts else np.array([], dtype=dt)
