"""Record how far an fp32 RMVPE salience may legitimately sit from exact arithmetic on each fixture clip.

Run:  python tests/golden/add_salience_noise.py        (CPU, a few minutes; adds `sal_fp32_noise` to the fixtures)

For the padded input of every fixture that stores a reference salience (pipeline_c2_{ios,synth}.npz,
pipeline_c4_30s.npz) the oracle E2E (oracle/rmvpe.py, the reference's RMVPE.py:13-564 restated in torch) runs in
fp32 (8 threads, the reference run's setting) and in fp64; `sal_fp32_noise` = max |fp32 - fp64| over the whole
[F, 360] matrix. An fp32 device computation and the fp32 reference each sit within about that of the exact
salience, so tests/rmvpe_parity.py allows the device-vs-reference salience error 3x this (triangle inequality with
a factor 2 for the device's different kernels and summation orders). Measured: C2 ios 8.7e-5, C2 synth 1.0e-4,
C4 1.5e-4; two fp32 thread counts of the same code differ by up to 1.2e-4 / 1.3e-4 / 1.5e-4.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch
from scipy import signal

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "retrieval-based-voice-conversion-mlx_amd"), REPO]
OUT = os.path.join(REPO, "tests", "golden")

from oracle import rmvpe as orm  # noqa: E402
from rvcx import synthetic  # noqa: E402
from rvcx.config import RMVPE_CFG  # noqa: E402
from rvcx.weights import normalize_state  # noqa: E402


def bigru_any_dtype(w, x):
    """orm.bigru with the GRU module in the input's dtype (the oracle's nn.GRU is created fp32)."""
    gru = torch.nn.GRU(x.shape[-1], 256, num_layers=1, batch_first=True, bidirectional=True).to(x.dtype)
    gru.load_state_dict({k[len("fc.0.gru."):]: w[k].to(x.dtype) for k in w if k.startswith("fc.0.gru.")})
    return gru.eval()(x)[0]


def clips():
    ios = np.load(os.path.join(OUT, "ios_kat.npz"))["input_audio"].astype(np.float64)
    return {"pipeline_c2_ios.npz": ios,
            "pipeline_c2_synth.npz": synthetic.speech_like(216100, seed=1000).astype(np.float32).astype(np.float64),
            "pipeline_c4_30s.npz": synthetic.speech_like(480000, seed=1000).astype(np.float32).astype(np.float64)}


def main():
    orm.bigru = bigru_any_dtype
    w = normalize_state(synthetic.rmvpe_state(5))
    bh, ah = signal.butter(N=5, Wn=48, btype="high", fs=16000)  # rvc/infer/pipeline.py:22-27, :439, :459
    for name, audio in clips().items():
        x = np.pad(signal.filtfilt(bh, ah, audio), (16000, 16000), mode="reflect").astype(np.float32)
        mel = orm.mel_spectrogram(torch.from_numpy(x)[None])
        hs = {}
        for dt in (torch.float32, torch.float64):
            torch.set_num_threads(8)
            wd = {k: torch.from_numpy(np.asarray(v)).to(dt) for k, v in w.items()}
            hs[dt] = orm.mel2hidden(wd, RMVPE_CFG, mel.to(dt)).squeeze(0).double().numpy()
        noise = float(np.abs(hs[torch.float32] - hs[torch.float64]).max())
        path = os.path.join(OUT, name)
        g = dict(np.load(path, allow_pickle=False))
        assert g["hidden16"].shape == hs[torch.float32].shape
        # the oracle fp32 salience is the reference's to within the same noise (it pins the fixture)
        d16 = float(np.abs(hs[torch.float32] - g["hidden16"].astype(np.float64)).max())
        assert d16 <= noise + 4.9e-4, (name, d16)
        g["sal_fp32_noise"] = np.float32(noise)
        np.savez_compressed(path, **g)
        print(f"{name}: sal_fp32_noise {noise:.3e} (oracle fp32 vs fixture fp16 {d16:.2e})")


if __name__ == "__main__":
    main()
