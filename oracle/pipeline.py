"""Oracle: Pipeline.pipeline / get_f0 / voice_conversion (rvc/infer/pipeline.py).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). Host DSP in numpy/scipy,
models from oracle.{hubert,rmvpe,synth}. RNG draws are injected through
``noise_fn(shape, which)`` so parity runs can share noise with the HIP path.
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np
import torch
import torch.nn.functional as F
from scipy import signal

from oracle import hubert as ohubert
from oracle import rmvpe as ormvpe
from oracle import synth as osynth

# pipeline.py:22-27
BH, AH = signal.butter(N=5, Wn=48, btype="high", fs=16000)

NOTE_DICT = [49.00, 51.91, 55.00, 58.27, 61.74, 65.41, 69.30, 73.42, 77.78, 82.41, 87.31, 92.50,
             98.00, 103.83, 110.00, 116.54, 123.47, 130.81, 138.59, 146.83, 155.56, 164.81,
             174.61, 185.00, 196.00, 207.65, 220.00, 233.08, 246.94, 261.63, 277.18, 293.66,
             311.13, 329.63, 349.23, 369.99, 392.00, 415.30, 440.00, 466.16, 493.88, 523.25,
             554.37, 587.33, 622.25, 659.25, 698.46, 739.99, 783.99, 830.61, 880.00, 932.33,
             987.77, 1046.50]


def autotune_f0(f0: np.ndarray, strength: float) -> np.ndarray:
    """Autotune.autotune_f0 (pipeline.py:151-162)."""
    out = np.zeros_like(f0)
    for i, freq in enumerate(f0):
        closest = min(NOTE_DICT, key=lambda x: abs(x - freq))
        out[i] = freq + (closest - freq) * strength
    return out


def coarse_pitch(f0: np.ndarray):
    """Mel quantisation to 1..255 (pipeline.py:281-291). Returns (coarse int64, f0bak)."""
    f0_mel_min = 1127 * np.log(1 + 50 / 700)
    f0_mel_max = 1127 * np.log(1 + 1100 / 700)
    f0bak = f0.copy()
    f0_mel = 1127 * np.log(1 + f0 / 700)
    pos = f0_mel > 0
    f0_mel[pos] = (f0_mel[pos] - f0_mel_min) * 254 / (f0_mel_max - f0_mel_min) + 1
    f0_mel[f0_mel <= 1] = 1
    f0_mel[f0_mel > 255] = 255
    return np.rint(f0_mel).astype(int), f0bak


def post_f0(f0: np.ndarray, pitch: int, f0_autotune=False, f0_autotune_strength=1.0,
            proposed_pitch=False, proposed_pitch_threshold=155.0):
    """f0 adjustments of Pipeline.get_f0 (pipeline.py:248-291)."""
    if f0_autotune is True:
        f0 = autotune_f0(f0, f0_autotune_strength)
    elif proposed_pitch is True:
        limit = 12
        valid = np.where(f0 > 0)[0]
        if len(valid) < 2:
            up_key = 0
        else:
            med = float(np.median(np.interp(np.arange(len(f0)), valid, f0[valid])))
            if med <= 0 or np.isnan(med):
                up_key = 0
            else:
                up_key = max(-limit, min(limit, int(np.round(12 * np.log2(proposed_pitch_threshold / med)))))
        f0 *= pow(2, (pitch + up_key) / 12)
    else:
        f0 *= pow(2, pitch / 12)
    return coarse_pitch(f0)


class OraclePipeline:
    """Pipeline (pipeline.py:165-558) over oracle models and fused weight dicts."""

    def __init__(self, tgt_sr: int, x_pad=1, x_query=6, x_center=38, x_max=41,
                 synth_w=None, synth_cfg=None, hubert_w=None, hubert_cfg=None, rmvpe_w=None, rmvpe_cfg=None,
                 noise_fn: Optional[Callable] = None):
        self.sample_rate = 16000
        self.window = 160
        self.tgt_sr = tgt_sr
        self.t_pad = int(self.sample_rate * x_pad)
        self.t_pad_tgt = int(tgt_sr * x_pad)
        self.t_pad2 = self.t_pad * 2
        self.t_query = int(self.sample_rate * x_query)
        self.t_center = int(self.sample_rate * x_center)
        self.t_max = int(self.sample_rate * x_max)
        self.sw, self.sc = synth_w, synth_cfg
        self.hw, self.hc = hubert_w, hubert_cfg
        self.rw, self.rc = rmvpe_w, rmvpe_cfg
        self.noise_fn = noise_fn or (lambda shape, which: torch.randn(shape))
        self.last = {}

    def get_f0(self, x, p_len, pitch=0, f0_autotune=False, f0_autotune_strength=1.0,
               proposed_pitch=False, proposed_pitch_threshold=155.0):
        f0, hidden = ormvpe.infer_from_audio(self.rw, self.rc, x, thred=0.03)
        self.last["f0_raw"], self.last["hidden"] = f0.copy(), hidden
        return post_f0(f0, pitch, f0_autotune, f0_autotune_strength, proposed_pitch, proposed_pitch_threshold)

    def voice_conversion(self, sid, audio0, pitch, pitchf, protect, version="v2", index=None, index_rate=0.0):
        """pipeline.py:293-376; ``index`` is an oracle.ivf.IvfFlat (faiss restatement), used when index_rate > 0."""
        with torch.no_grad():
            feats = torch.from_numpy(audio0).float().view(1, -1)
            feats = ohubert.hubert_forward(self.hw, self.hc, feats, version)
            feats0 = feats.clone()
            if index is not None and index_rate > 0:  # pipeline.py:338-342, :378-388
                from oracle import ivf

                big_npy = ivf.reconstruct_n(index, 0, index.ntotal)
                npy = feats[0].numpy()
                score, ix = ivf.search(index, npy, 8)
                self.last.setdefault("index_search", []).append((score, ix))
                feats = torch.from_numpy(ivf.retrieve_speaker_embeddings(npy, score, ix, big_npy,
                                                                         index_rate)).unsqueeze(0)
            feats = F.interpolate(feats.permute(0, 2, 1), scale_factor=2).permute(0, 2, 1)
            p_len = min(audio0.shape[0] // self.window, feats.shape[1])
            feats0 = F.interpolate(feats0.permute(0, 2, 1), scale_factor=2).permute(0, 2, 1)
            pitch, pitchf = pitch[:, :p_len], pitchf[:, :p_len]
            if protect < 0.5:
                pitchff = pitchf.clone()
                pitchff[pitchf > 0] = 1
                pitchff[pitchf < 1] = protect
                feats = feats * pitchff.unsqueeze(-1) + feats0 * (1 - pitchff.unsqueeze(-1))
            plen = torch.tensor([p_len]).long()
            T = feats.shape[1]
            eps_z = self.noise_fn((1, self.sc.inter_channels, T), "z")
            voc = getattr(self.sc, "vocoder", "HiFi-GAN")
            H = 9 if voc == "MRF HiFi-GAN" else 1  # source noise per decoder (include/rvcx.h layout)
            eps_src = self.noise_fn((1, T * self.sc.upp * H + (H if voc != "HiFi-GAN" else 0)), "src")
            o = osynth.synth_infer(self.sw, self.sc, feats.float(), plen, pitch, pitchf.float(), sid,
                                   eps_z, eps_src)[0]
            return o[0, 0].float().numpy()

    def pipeline(self, sid, audio, pitch=0, protect=0.33, volume_envelope=1.0, f0_autotune=False,
                 f0_autotune_strength=1.0, proposed_pitch=False, proposed_pitch_threshold=155.0, index=None,
                 index_rate=0.0):
        """pipeline.py:390-558 with pitch_guidance=True; ``index`` = the parsed file_index (oracle.ivf)."""
        vc_kw = dict(index=index, index_rate=index_rate)
        audio = signal.filtfilt(BH, AH, audio)
        audio_pad = np.pad(audio, (self.window // 2, self.window // 2), mode="reflect")
        opt_ts = []
        if audio_pad.shape[0] > self.t_max:
            audio_sum = np.zeros_like(audio)
            for i in range(self.window):
                audio_sum += audio_pad[i:i - self.window]
            for t in range(self.t_center, audio.shape[0], self.t_center):
                seg = np.abs(audio_sum[t - self.t_query:t + self.t_query])
                opt_ts.append(t - self.t_query + np.where(seg == seg.min())[0][0])
        s = 0
        audio_opt = []
        t = None
        audio_pad = np.pad(audio, (self.t_pad, self.t_pad), mode="reflect")
        p_len = audio_pad.shape[0] // self.window
        sid_t = torch.tensor(sid).unsqueeze(0).long()
        pitch_c, pitchf = self.get_f0(audio_pad, p_len, pitch, f0_autotune, f0_autotune_strength,
                                      proposed_pitch, proposed_pitch_threshold)
        pitch_c, pitchf = pitch_c[:p_len], pitchf[:p_len]
        pitch_t = torch.tensor(pitch_c).unsqueeze(0).long()
        pitchf_t = torch.tensor(pitchf).unsqueeze(0).float()
        self.last["pitch"], self.last["pitchf"] = pitch_c, pitchf
        for t in opt_ts:
            t = t // self.window * self.window
            audio_opt.append(self.voice_conversion(
                sid_t, audio_pad[s:t + self.t_pad2 + self.window],
                pitch_t[:, s // self.window:(t + self.t_pad2) // self.window],
                pitchf_t[:, s // self.window:(t + self.t_pad2) // self.window], protect,
                **vc_kw)[self.t_pad_tgt:-self.t_pad_tgt])
            s = t
        audio_opt.append(self.voice_conversion(
            sid_t, audio_pad[t:] if t is not None else audio_pad,
            pitch_t[:, t // self.window:] if t is not None else pitch_t,
            pitchf_t[:, t // self.window:] if t is not None else pitchf_t, protect,
            **vc_kw)[self.t_pad_tgt:-self.t_pad_tgt])
        audio_opt = np.concatenate(audio_opt)
        if volume_envelope != 1:
            audio_opt = change_rms(audio, self.sample_rate, audio_opt, self.tgt_sr, volume_envelope)
        audio_max = np.abs(audio_opt).max() / 0.99
        if audio_max > 1:
            audio_opt /= audio_max
        return audio_opt


def rms_frames(y: np.ndarray, frame_length: int, hop_length: int) -> np.ndarray:
    """librosa.feature.rms(y, frame_length, hop_length, center=True, pad_mode='constant') -> [1, n]."""
    y = np.pad(y, int(frame_length // 2), mode="constant")
    n = 1 + (len(y) - frame_length) // hop_length
    idx = np.arange(frame_length)[None, :] + hop_length * np.arange(n)[:, None]
    frames = y[idx]
    power = np.mean(np.abs(frames) ** 2, axis=1, keepdims=False)
    return np.sqrt(power)[None, :]


def change_rms(source_audio, source_rate, target_audio, target_rate, rate):
    """AudioProcessor.change_rms (pipeline.py:35-82)."""
    rms1 = rms_frames(source_audio, source_rate // 2 * 2, source_rate // 2)
    rms2 = rms_frames(target_audio, target_rate // 2 * 2, target_rate // 2)
    rms1 = F.interpolate(torch.from_numpy(rms1).float().unsqueeze(0), size=target_audio.shape[0],
                         mode="linear").squeeze()
    rms2 = F.interpolate(torch.from_numpy(rms2).float().unsqueeze(0), size=target_audio.shape[0],
                         mode="linear").squeeze()
    rms2 = torch.maximum(rms2, torch.zeros_like(rms2) + 1e-6)
    return target_audio * (torch.pow(rms1, 1 - rate) * torch.pow(rms2, rate - 1)).numpy()
