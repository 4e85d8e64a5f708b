"""Oracle: RMVPE f0 predictor (mel -> E2E U-Net + BiGRU -> salience -> decode).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). Follows
rvc/lib/predictors/RMVPE.py (PyTorch path); librosa (absent here, pinned 0.11.0
at uv.lock:1320-1321) is restated for ``librosa.filters.mel(htk=True)``.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from oracle.synth import _t

N_CLASS = 360


# ----------------------------------------------------------------- librosa restatements
def hz_to_mel(f, htk: bool):
    f = np.asanyarray(f, dtype=np.float64)
    if htk:
        return 2595.0 * np.log10(1.0 + f / 700.0)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep, mels)


def mel_to_hz(m, htk: bool):
    m = np.asanyarray(m, dtype=np.float64)
    if htk:
        return 700.0 * (10.0 ** (m / 2595.0) - 1.0)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def mel_filterbank(sr: int, n_fft: int, n_mels: int, fmin: float, fmax: float, htk: bool) -> np.ndarray:
    """librosa.filters.mel(..., norm='slaney', dtype=float32) (librosa 0.11 filters.py)."""
    weights = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(fmin, htk), hz_to_mel(fmax, htk), n_mels + 2), htk)
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights


def rmvpe_mel_basis() -> np.ndarray:
    """MelSpectrogram(N_MELS=128, 16000, 1024, 160, None, 30, 8000) basis (RMVPE.py:371-379, :438-440)."""
    return mel_filterbank(16000, 1024, 128, 30, 8000, htk=True)


def mel_spectrogram(audio: torch.Tensor) -> torch.Tensor:
    """MelSpectrogram.forward(keyshift=0, speed=1, center=True) (RMVPE.py:388-417). audio [B, N]."""
    window = torch.hann_window(1024)
    fft = torch.stft(audio, n_fft=1024, hop_length=160, win_length=1024, window=window,
                     center=True, return_complex=True)
    mag = torch.sqrt(fft.real.pow(2) + fft.imag.pow(2))
    mel = torch.matmul(torch.from_numpy(rmvpe_mel_basis()), mag)
    return torch.log(torch.clamp(mel, min=1e-5))


# ----------------------------------------------------------------- E2E network
def _bn(w, p, x):
    return F.batch_norm(x, _t(w, p + ".running_mean"), _t(w, p + ".running_var"), _t(w, p + ".weight"),
                        _t(w, p + ".bias"), False, 0.0, 1e-5)


def conv_block_res(w, p, x):
    """ConvBlockRes.forward (RMVPE.py:13-57)."""
    y = F.conv2d(x, _t(w, p + ".conv.0.weight"), None, padding=1)
    y = torch.relu(_bn(w, p + ".conv.1", y))
    y = F.conv2d(y, _t(w, p + ".conv.3.weight"), None, padding=1)
    y = torch.relu(_bn(w, p + ".conv.4", y))
    if (p + ".shortcut.weight") in w:
        return y + F.conv2d(x, _t(w, p + ".shortcut.weight"), _t(w, p + ".shortcut.bias"))
    return y + x


def deep_unet(w, cfg, x):
    """DeepUnet.forward = Encoder -> Intermediate -> Decoder (RMVPE.py:94-286)."""
    x = _bn(w, "unet.encoder.bn", x)
    skips = []
    for i in range(cfg.en_de_layers):
        for b in range(cfg.n_blocks):
            x = conv_block_res(w, f"unet.encoder.layers.{i}.conv.{b}", x)
        skips.append(x)
        x = F.avg_pool2d(x, 2)
    for i in range(cfg.inter_layers):
        for b in range(cfg.n_blocks):
            x = conv_block_res(w, f"unet.intermediate.layers.{i}.conv.{b}", x)
    for i in range(cfg.en_de_layers):
        p = f"unet.decoder.layers.{i}"
        x = F.conv_transpose2d(x, _t(w, p + ".conv1.0.weight"), None, stride=2, padding=1, output_padding=1)
        x = torch.relu(_bn(w, p + ".conv1.1", x))
        x = torch.cat((x, skips[-1 - i]), dim=1)
        for b in range(cfg.n_blocks):
            x = conv_block_res(w, f"{p}.conv2.{b}", x)
    return x


def bigru(w, x):
    """BiGRU (RMVPE.py:543-564) = nn.GRU(384, 256, bidirectional, batch_first)."""
    gru = torch.nn.GRU(x.shape[-1], 256, num_layers=1, batch_first=True, bidirectional=True)
    sd = {k[len("fc.0.gru."):]: _t(w, k) for k in w if k.startswith("fc.0.gru.")}
    gru.load_state_dict(sd)
    gru.eval()
    return gru(x)[0]


def e2e(w, cfg, mel):
    """E2E.forward (RMVPE.py:335-339): mel [B,128,F] -> salience [B,F,360]."""
    x = mel.transpose(-1, -2).unsqueeze(1)
    x = deep_unet(w, cfg, x)
    x = F.conv2d(x, _t(w, "cnn.weight"), _t(w, "cnn.bias"), padding=1)
    x = x.transpose(1, 2).flatten(-2)
    x = bigru(w, x)
    x = F.linear(x, _t(w, "fc.1.weight"), _t(w, "fc.1.bias"))
    return torch.sigmoid(x)


def mel2hidden(w, cfg, mel, chunk_size: int = 32000):
    """RMVPE0Predictor.mel2hidden (RMVPE.py:445-482): reflect-pad frames to x32, chunked E2E."""
    with torch.no_grad():
        n = mel.shape[-1]
        mel = F.pad(mel, (0, 32 * ((n - 1) // 32 + 1) - n), mode="reflect")
        outs = []
        for s in range(0, mel.shape[-1], chunk_size):
            outs.append(e2e(w, cfg, mel[..., s:min(s + chunk_size, mel.shape[-1])]))
        hidden = torch.cat(outs, dim=1)
    return hidden[:, :n]


# ----------------------------------------------------------------- decode (numpy fp64)
CENTS_MAPPING = np.pad(20 * np.arange(N_CLASS) + 1997.3794084376191, (4, 4))


def to_local_average_cents(salience: np.ndarray, thred: float = 0.05) -> np.ndarray:
    """RMVPE0Predictor.to_local_average_cents (RMVPE.py:515-540), vectorised gather."""
    center = np.argmax(salience, axis=1)
    sal = np.pad(salience, ((0, 0), (4, 4)))
    center = center + 4
    idx = (center - 4)[:, None] + np.arange(9)[None, :]
    ts = np.take_along_axis(sal, idx, axis=1)
    tc = CENTS_MAPPING[idx]
    product_sum = np.sum(ts * tc, 1)
    weight_sum = np.sum(ts, 1)
    with np.errstate(invalid="ignore", divide="ignore"):
        devided = product_sum / weight_sum
    maxx = np.max(sal, axis=1)
    devided[maxx <= thred] = 0
    return devided


def decode(hidden: np.ndarray, thred: float = 0.03) -> np.ndarray:
    """RMVPE0Predictor.decode (RMVPE.py:484-495)."""
    cents = to_local_average_cents(hidden, thred=thred)
    f0 = 10 * (2 ** (cents / 1200))
    f0[f0 == 10] = 0
    return f0


def infer_from_audio(w, cfg, audio: np.ndarray, thred: float = 0.03):
    """RMVPE0Predictor.infer_from_audio (RMVPE.py:497-513). Returns (f0 fp64 [F], hidden f32 [F,360])."""
    a = torch.from_numpy(np.asarray(audio)).float().unsqueeze(0)
    mel = mel_spectrogram(a)
    hidden = mel2hidden(w, cfg, mel).squeeze(0).numpy()
    return decode(hidden, thred), hidden
