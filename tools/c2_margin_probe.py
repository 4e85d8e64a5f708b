"""Margin of the C2 full-size parity (tests/test_gpu_c2_parity.py) on the GPU box: rel_err (bar 2e-3), spectrogram
correlation (bar 0.999) and where the largest sample difference sits, per clip. usage: python tools/c2_margin_probe.py"""
import os, sys
ROOT = "/root/repo" if os.path.isdir("/root/repo") else os.getcwd()
sys.path[:0] = [os.path.join(ROOT, "retrieval-based-voice-conversion-mlx_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np
from conftest import c2_audio, fixture_noise, golden
from oracle.metrics import spectrogram_correlation
from rvcx import synthetic
from rvcx.config import SYNTH_48K_V2
from rvcx.engine import Engine
from rvcx.weights import normalize_state
e = Engine(0)
e.load_synth(normalize_state(synthetic.synth_state(2)), SYNTH_48K_V2)
e.load_hubert(normalize_state(synthetic.hubert_state(4)))
e.load_rmvpe(normalize_state(synthetic.rmvpe_state(5)))
for clip in ("ios", "synth"):
    g = golden(f"pipeline_c2_{clip}.npz")
    ez, es = fixture_noise(g)
    e.set_pipeline_highpass()
    out = e.pipeline(c2_audio(clip), sid=0, semitones=0, protect=0.33, t_pad=16000, t_pad_tgt=48000, eps_z=ez, eps_src=es).cpu().numpy()
    ref = g["out"].astype(np.float64)
    d = np.abs(out - ref)
    print(clip, "rel_err %.3e" % (d.max() / np.abs(ref).max()), "spec_corr %.6f" % spectrogram_correlation(out, ref.astype(np.float32)), "argmax t=%d" % int(d.argmax()), "p99.9 %.3e" % (np.quantile(d, 0.999) / np.abs(ref).max()))
