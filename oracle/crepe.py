"""Oracle: CREPE pitch estimator ("crepe" / "crepe-tiny" f0 methods).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). Restates the MLX reference
rvc_mlx/lib/mlx/crepe.py (CREPEModel :48-222, CREPE.get_f0 :282-325, _frame_audio :327-359,
_decode :387-441, _median_filter / _mean_filter :443-452) in torch-CPU / numpy. The network is
torchcrepe's (rvc/lib/predictors/f0.py:25-57 calls torchcrepe.predict); torchcrepe and mlx are
absent here, so parity against the reference's own run is UNPINNED: this file follows the MLX source
line by line and the device path is checked against it.

Weights use torchcrepe's state-dict names and torch layouts (conv{i}.weight [O][I][K][1],
conv{i}_BN.{weight,bias,running_mean,running_var}, classifier.weight [360][in_features]);
rvcx.weights.load_crepe_weights maps the MLX npz (tools/convert_crepe_weights.py) onto them.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

PITCH_BINS = 360
HOP_SIZE = 160  # crepe.py:23
WINDOW_SIZE = 1024  # crepe.py:24
CENTS = 20 * np.arange(PITCH_BINS) + 1997.3794084376191  # crepe.py:44
BN_EPS = 1e-3  # crepe.py:87 (nn.BatchNorm eps=1e-3)

CAPACITY = {"full": [1024, 128, 128, 128, 256, 512], "tiny": [128, 16, 16, 16, 32, 64]}  # crepe.py:66-75
KERNELS = [512, 64, 64, 64, 64, 64]  # crepe.py:78
STRIDES = [4, 1, 1, 1, 1, 1]  # crepe.py:79
PADS = [(254, 254)] + [(31, 32)] * 5  # crepe.py:196-205


def model_type(w) -> str:
    return "full" if w["conv1.weight"].shape[0] == 1024 else "tiny"


def frame_audio(audio: np.ndarray) -> np.ndarray:
    """_frame_audio (crepe.py:327-359): reflect pad 512, 1024-sample frames every 160, each frame minus its
    mean and divided by its (population) std when std > 1e-10. float32 as numpy computes it."""
    audio = np.asarray(audio, dtype=np.float32)
    pad = WINDOW_SIZE // 2
    ap = np.pad(audio, (pad, pad), mode="reflect")
    n_frames = 1 + (len(ap) - WINDOW_SIZE) // HOP_SIZE
    frames = np.zeros((n_frames, WINDOW_SIZE), dtype=np.float32)
    for i in range(n_frames):
        fr = ap[i * HOP_SIZE:i * HOP_SIZE + WINDOW_SIZE]
        fr = fr - np.mean(fr)
        sd = np.std(fr)
        if sd > 1e-10:
            fr = fr / sd
        frames[i] = fr
    return frames


def forward(w, frames: np.ndarray) -> np.ndarray:
    """CREPEModel.__call__ (crepe.py:184-222): 6 x (pad, conv, relu, BatchNorm, maxpool 2), flatten H-major
    then channels, Linear, sigmoid. frames [B][1024] -> probabilities [B][360] float32."""
    t = lambda k: torch.as_tensor(np.asarray(w[k], dtype=np.float32))  # noqa: E731
    x = torch.as_tensor(frames, dtype=torch.float32)[:, None, :]  # [B][C=1][H]
    for i in range(6):
        p = f"conv{i + 1}"
        x = F.pad(x, PADS[i])
        x = F.conv1d(x, t(p + ".weight")[..., 0], t(p + ".bias"), stride=STRIDES[i])
        x = torch.relu(x)
        bn = p + "_BN"
        inv = torch.rsqrt(t(bn + ".running_var") + BN_EPS)
        x = (x - t(bn + ".running_mean")[:, None]) * inv[:, None] * t(bn + ".weight")[:, None] + t(bn + ".bias")[:, None]
        x = F.max_pool1d(x, 2, 2)
    B = x.shape[0]
    x = x.permute(0, 2, 1).reshape(B, -1)  # (B, H, C) flatten, as MLX's (B, H, W=1, C)
    return torch.sigmoid(F.linear(x, t("classifier.weight"), t("classifier.bias"))).numpy()


def _f32_pairwise_sum(v: np.ndarray) -> np.float32:
    return np.float32(v.astype(np.float32).sum())


def decode(probs: np.ndarray, f0_min: float, f0_max: float):
    """_decode (crepe.py:387-441): bins outside [f0_min, f0_max] (in cents) zeroed, argmax, periodicity = the
    peak probability, cents = weighted mean of the +-4 bins around the peak (float64 products over float32
    weights), f0 = 10 * 2^(cents/1200) in float32. Returns (f0 float32, periodicity float32)."""
    probs = np.asarray(probs, dtype=np.float32)
    lo = 1200.0 * np.log2(f0_min / 10.0)
    hi = 1200.0 * np.log2(f0_max / 10.0)
    valid = (CENTS >= lo) & (CENTS <= hi)
    pm = probs.copy()
    pm[:, ~valid] = 0
    peak = np.argmax(pm, axis=1)
    periodicity = pm[np.arange(len(peak)), peak]
    cents = np.zeros(len(peak), dtype=np.float32)
    for i, pk in enumerate(peak):
        s, e = max(0, pk - 4), min(PITCH_BINS, pk + 4 + 1)
        pw = pm[i, s:e]
        tw = pw.sum()
        if tw > 0:
            cents[i] = (pw * CENTS[s:e]).sum() / tw
    f0 = 10.0 * (2 ** (cents / 1200.0))
    return f0.astype(np.float32), periodicity.astype(np.float32)


def get_f0(w, audio: np.ndarray, f0_min: float = 50.0, f0_max: float = 1100.0, threshold: float = 0.1,
           batch_size: int = 512, return_periodicity: bool = False):
    """CREPE.get_f0 (crepe.py:282-325): frames -> probabilities (batches of 512) -> decode -> median filter of
    the periodicity (scipy.ndimage.median_filter size 3) and mean filter of f0 (uniform_filter1d size 3), both
    mode 'reflect' -> f0 = 0 where periodicity < threshold."""
    from scipy.ndimage import median_filter, uniform_filter1d

    frames = frame_audio(audio)
    probs = np.concatenate([forward(w, frames[i:i + batch_size]) for i in range(0, len(frames), batch_size)])
    f0, per = decode(probs, f0_min, f0_max)
    per = median_filter(per, size=3)
    f0 = uniform_filter1d(f0, size=3)
    f0[per < threshold] = 0
    if return_periodicity:
        return f0, per, probs
    return f0
