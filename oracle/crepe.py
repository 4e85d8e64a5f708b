"""Oracle: CREPE pitch estimator ("crepe" / "crepe-tiny" f0 methods).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). Restates the MLX reference
rvc_mlx/lib/mlx/crepe.py (CREPEModel :48-222, CREPE.get_f0 :282-325, _frame_audio :327-359,
_decode :387-441, _median_filter / _mean_filter :443-452) in torch-CPU / numpy. The network is
torchcrepe's (rvc/lib/predictors/f0.py:25-57 calls torchcrepe.predict); torchcrepe and mlx are
absent here, so parity against the reference's own run is UNPINNED: this file follows the MLX source
line by line and the device path is checked against it.

get_f0_rvc restates the rvc/ side (rvc/lib/predictors/f0.py:31-55): torchcrepe.predict's framing (preprocess:
zero padding of 512, unbiased std), postprocess + decode.viterbi (softmax of the masked sigmoid outputs,
librosa.sequence.viterbi with the +-11-bin triangular transition matrix), convert.bins_to_frequency (with the
caller's dither values in place of scipy.stats.triang draws) and filter.median / filter.mean (window 3). These are
restated from torchcrepe's and librosa's published source (neither is importable here): UNPINNED as well.

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


# ---------------------------------------------------------------- rvc/ semantics (torchcrepe.predict + viterbi)
def frame_audio_torch(audio: np.ndarray) -> np.ndarray:
    """torchcrepe.preprocess (pad=True): zero pad 512 per side, 1024-sample frames every 160 (1 + n//160 of them),
    minus the mean, divided by max(1e-10, unbiased std). float32 as torch computes it."""
    a = torch.as_tensor(np.asarray(audio, dtype=np.float32))
    n_frames = 1 + len(audio) // HOP_SIZE
    ap = F.pad(a[None], (WINDOW_SIZE // 2, WINDOW_SIZE // 2))[0]
    frames = ap.unfold(0, WINDOW_SIZE, HOP_SIZE)[:n_frames].clone()
    frames -= frames.mean(dim=1, keepdim=True)
    frames /= torch.clamp(frames.std(dim=1, keepdim=True), min=1e-10)
    return frames.numpy()


def torchcrepe_bin_range(f0_min: float, f0_max: float):
    """postprocess: bins [frequency_to_bins(fmin) (floor), frequency_to_bins(fmax, ceil)) stay, the rest -inf."""
    lo = int(np.floor((1200.0 * np.log2(f0_min / 10.0) - 1997.3794084376191) / 20.0))
    hi = int(np.ceil((1200.0 * np.log2(f0_max / 10.0) - 1997.3794084376191) / 20.0))
    return max(0, min(PITCH_BINS, lo)), max(0, min(PITCH_BINS, hi))


RVC_CREPE_BATCH = 512  # rvc/lib/predictors/f0.py:38 (torchcrepe.predict batch_size)


def viterbi_bins(probs: np.ndarray, f0_min: float, f0_max: float, batch: int = RVC_CREPE_BATCH) -> np.ndarray:
    """torchcrepe.predict runs postprocess -- and so decode.viterbi -- once per batch of `batch` frames (f0.py:38-49),
    each batch a sequence of its own from the uniform initial state; the bin paths are concatenated."""
    probs = np.asarray(probs)
    return np.concatenate([_viterbi_seq(probs[i:i + batch], f0_min, f0_max)
                           for i in range(0, len(probs), batch)]) if len(probs) else np.zeros(0, np.int64)


def _viterbi_seq(probs: np.ndarray, f0_min: float, f0_max: float) -> np.ndarray:
    """decode.viterbi on the masked sigmoid outputs: softmax over the bins (float32), then
    librosa.sequence.viterbi(prob, transition): log(prob + tiny) float32, log(transition + tiny) float64, uniform
    p_init, values in float64, first argmax; returns the bin path [F]."""
    lo, hi = torchcrepe_bin_range(f0_min, f0_max)
    p = np.asarray(probs, dtype=np.float32).copy()
    p[:, :lo] = -np.inf
    p[:, hi:] = -np.inf
    seq = torch.softmax(torch.as_tensor(p), dim=1).numpy()
    eps = np.finfo(np.float32).tiny
    xx, yy = np.meshgrid(range(PITCH_BINS), range(PITCH_BINS))
    trans = np.maximum(12 - abs(xx - yy), 0)
    trans = trans / trans.sum(axis=1, keepdims=True)
    log_trans = np.log(trans + eps)
    log_prob = np.log(seq + eps)
    log_p_init = np.log(np.full(PITCH_BINS, 1.0 / PITCH_BINS) + eps)
    n = log_prob.shape[0]
    value = log_prob[0] + log_p_init
    ptr = np.zeros((n, PITCH_BINS), dtype=np.int64)
    rows = np.arange(PITCH_BINS)
    for t in range(1, n):
        trans_out = value[None, :] + log_trans.T  # [j][k] = value[k] + log_trans[k][j]
        ptr[t] = np.argmax(trans_out, axis=1)
        value = log_prob[t] + trans_out[rows, ptr[t]]
    state = np.zeros(n, dtype=np.int64)
    state[-1] = np.argmax(value)
    for t in range(n - 2, -1, -1):
        state[t] = ptr[t + 1, state[t + 1]]
    return state


def get_f0_rvc(w, audio: np.ndarray, f0_min: float = 50.0, f0_max: float = 1100.0, threshold: float = 0.1,
               dither=None, probs=None):
    """rvc/'s CREPE.get_f0: -> (f0 float32 [F], filtered periodicity float32 [F], probabilities [F][360]).
    probs: decode these instead of running the network (the device's own, to check the decode alone)."""
    if probs is None:
        probs = forward(w, frame_audio_torch(audio))
    probs = np.asarray(probs, dtype=np.float32)
    bins = viterbi_bins(probs, f0_min, f0_max)
    cents = (20 * bins).astype(np.float32) + np.float32(1997.3794084376191)
    if dither is not None:
        cents = cents + np.asarray(dither, dtype=np.float32)
    f0 = np.float32(10.0) * np.exp2(cents / np.float32(1200.0))
    per = probs[np.arange(len(bins)), bins]
    n = len(bins)
    pm = np.empty(n, dtype=np.float32)
    fm = np.empty(n, dtype=np.float32)
    for i in range(n):  # torchcrepe.filter.median / mean, window 3, edges over the 2 samples inside
        s, e = max(0, i - 1), min(n, i + 2)
        w3 = np.sort(per[s:e])
        pm[i] = w3[(len(w3) - 1) // 2]
        v = f0[s:e]
        fm[i] = ((v[0] + v[1]) + v[2]) / np.float32(3.0) if len(v) == 3 else (v.sum(dtype=np.float32) / np.float32(len(v)))
    fm[pm < threshold] = 0
    return fm, pm, probs
