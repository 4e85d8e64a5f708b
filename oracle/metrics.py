"""Parity metrics — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

``spectrogram_correlation`` restates benchmarks/benchmark_audio_parity.py:398-421
without librosa: |STFT| (n_fft 1024, hop 256, center=True with constant/zero
padding as librosa>=0.10 does, periodic Hann) -> power -> 80-band Slaney-scale,
Slaney-norm mel over 0..sr/2 -> power_to_db(ref=max, top_db=80) -> Pearson over
the flattened matrices; both signals trimmed to the shorter length first.
"""
from __future__ import annotations

import numpy as np

from oracle.rmvpe import mel_filterbank


def _stft_mag(y: np.ndarray, n_fft=1024, hop=256) -> np.ndarray:
    y = np.pad(np.asarray(y, dtype=np.float64), n_fft // 2, mode="constant")
    n = 1 + (len(y) - n_fft) // hop
    win = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n_fft) / n_fft)
    idx = np.arange(n_fft)[None, :] + hop * np.arange(n)[:, None]
    return np.abs(np.fft.rfft(y[idx] * win, axis=1)).T  # [1+n_fft/2, n]


def mel_db(y: np.ndarray, sr: int) -> np.ndarray:
    S = _stft_mag(y) ** 2
    fb = mel_filterbank(sr, 1024, 80, 0.0, sr / 2.0, htk=False).astype(np.float64)
    M = fb @ S
    db = 10.0 * np.log10(np.maximum(1e-10, M))
    db -= 10.0 * np.log10(np.maximum(1e-10, M.max()))
    return np.maximum(db, db.max() - 80.0)


def spectrogram_correlation(a: np.ndarray, b: np.ndarray, sr: int = 48000) -> float:
    n = min(len(a), len(b))
    A, B = mel_db(a[:n], sr).ravel(), mel_db(b[:n], sr).ravel()
    return float(np.corrcoef(A, B)[0, 1])


def waveform_correlation(a: np.ndarray, b: np.ndarray) -> float:
    n = min(len(a), len(b))
    return float(np.corrcoef(np.asarray(a[:n], np.float64), np.asarray(b[:n], np.float64))[0, 1])


def cents_agreement(f0_a: np.ndarray, f0_b: np.ndarray, tol_cents: float = 50.0):
    """(fraction of jointly-voiced frames within tol cents, voiced/unvoiced agreement)
    (tests/conftest.py:266-301 accuracy metric)."""
    va, vb = f0_a > 0, f0_b > 0
    vuv = float(np.mean(va == vb)) if len(va) else 1.0
    both = va & vb
    if not both.any():
        return 1.0, vuv
    c = 1200.0 * np.abs(np.log2(f0_a[both] / f0_b[both]))
    return float(np.mean(c <= tol_cents)), vuv
