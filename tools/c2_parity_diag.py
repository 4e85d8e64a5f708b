"""Diagnostic (GPU box): device pipeline vs the full-size C2 reference fixtures, stage by stage."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "retrieval-based-voice-conversion-mlx_amd"), ROOT, os.path.join(ROOT, "tests")]

import torch  # noqa: E402
from scipy import signal  # noqa: E402

from conftest import c2_audio, fixture_noise, golden  # noqa: E402
from oracle.metrics import cents_agreement, spectrogram_correlation, waveform_correlation  # noqa: E402
from rvcx import synthetic  # noqa: E402
from rvcx.config import SYNTH_48K_V2  # noqa: E402
from rvcx.engine import Engine  # noqa: E402
from rvcx.weights import normalize_state  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))


eng = Engine(0)
eng.load_synth(normalize_state(synthetic.synth_state(2)), SYNTH_48K_V2)
eng.load_hubert(normalize_state(synthetic.hubert_state(4)))
eng.load_rmvpe(normalize_state(synthetic.rmvpe_state(5)))
eng.set_pipeline_highpass()
bh, ah = signal.butter(N=5, Wn=48, btype="high", fs=16000)
for name in ("ios", "synth"):
    g = golden(f"pipeline_c2_{name}.npz")
    audio = c2_audio(name)
    ez, es = fixture_noise(g)
    out, f0 = eng.pipeline(audio, sid=0, protect=0.33, t_pad=16000, t_pad_tgt=48000, eps_z=ez, eps_src=es, want_f0=True)
    out = out.cpu().numpy()
    f0 = f0.cpu().numpy()
    ref = g["out"]
    fr = g["f0_raw"]
    acc, vuv = cents_agreement(f0[: len(fr)], fr, 50.0)
    eq = np.mean(f0[: len(fr)] == fr)
    close = np.abs(f0[: len(fr)] - fr) <= 1e-6 * np.abs(fr)
    print(f"[{name}] f0 exact {eq:.4f} close(1e-6) {close.mean():.4f} cents50 {acc:.4f} vuv {vuv:.4f}; "
          f"bad frames {np.flatnonzero(~close)[:20]}")
    x = np.pad(signal.filtfilt(bh, ah, audio), (16000, 16000), mode="reflect")
    h = eng.hubert(x.astype(np.float32)).cpu().numpy()
    print(f"[{name}] hubert rel {rel(h, g['feats16'].astype(np.float32)):.3e}")
    print(f"[{name}] pipeline: shape {out.shape} vs {ref.shape} spec_corr {spectrogram_correlation(out, ref):.6f} "
          f"rel {rel(out, ref):.3e} wave_corr {waveform_correlation(out, ref):.6f}")
    # staged: voice_conversion with the reference's pitch / pitchf and noise, then trim + normalise as the reference
    p_len = x.shape[0] // 160
    vc = eng.voice_conversion(x, g["pitch"][:p_len], g["f0_raw"][:p_len].astype(np.float32), 0, 0.33, eps_z=ez,
                              eps_src=es).cpu().numpy()
    vc = vc[48000:-48000]
    mx = np.abs(vc).max() / 0.99
    if mx > 1:
        vc = vc / mx
    print(f"[{name}] staged vc(ref pitch): spec_corr {spectrogram_correlation(vc, ref):.6f} rel {rel(vc, ref):.3e} "
          f"wave_corr {waveform_correlation(vc, ref):.6f}")
    d = np.abs(out - ref)
    print(f"[{name}] pipeline |diff| percentiles 50/99/99.9/max: {np.percentile(d, [50, 99, 99.9]).round(6)} {d.max():.4f}")
eng.close()
