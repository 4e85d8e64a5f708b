"""Oracle: split_audio.process_audio's interval search (rvc/lib/tools/split_audio.py:5-27).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). librosa 0.11.0 (uv.lock:1320-1321) is absent here, so its
effects.split / feature.rms / power_to_db / frames_to_samples are restated from their published algorithm
(center=True constant padding, mean |x|^2 per frame, 10 log10(max(amin, S)) - 10 log10(max(amin, max S)),
non-silent where > -top_db, edges at the flips, x hop, clipped). Parity against librosa itself is unpinned.
"""
import numpy as np


def rms(y, frame_length, hop_length):
    y = np.asarray(y, dtype=np.float64)
    yp = np.pad(y, frame_length // 2, mode="constant")
    nf = 1 + (len(yp) - frame_length) // hop_length
    idx = np.arange(frame_length)[None, :] + hop_length * np.arange(nf)[:, None]
    return np.sqrt(np.mean(np.abs(yp[idx]) ** 2, axis=1))


def effects_split(y, top_db=60, frame_length=2048, hop_length=512):
    mse = rms(y, frame_length, hop_length) ** 2
    db = 10.0 * np.log10(np.maximum(1e-10, mse)) - 10.0 * np.log10(np.maximum(1e-10, mse.max()))
    non_silent = db > -top_db
    edges = [np.flatnonzero(np.diff(non_silent.astype(int))) + 1]
    if non_silent[0]:
        edges.insert(0, [0])
    if non_silent[-1]:
        edges.append([len(non_silent)])
    edges = np.minimum(np.concatenate(edges).astype(np.int64) * hop_length, len(y))
    return edges.reshape((-1, 2))


def process_audio(audio, sr=16000, silence_thresh=-60, min_silence_len=250):
    frame_length = int(min_silence_len / 1000 * sr)
    intervals = effects_split(audio, top_db=-silence_thresh, frame_length=frame_length, hop_length=frame_length // 2)
    return [audio[s:e] for s, e in intervals], intervals
