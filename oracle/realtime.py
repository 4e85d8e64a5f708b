"""Oracle: streaming (realtime) voice conversion -- rvc/realtime/{core,pipeline}.py.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates, over the oracle models:
  * ``Realtime.realloc`` (rvc/realtime/core.py:165-216): buffer geometry from the 48 kHz block;
  * ``Realtime.inference`` (core.py:217-326): 48k -> 16k resample, circular audio/convert buffers,
    RMS gate (silent_threshold), conversion, ``* sqrt(vol)``, 16k -> 48k output resample;
  * ``Realtime_Pipeline.voice_conversion`` / ``get_f0`` (rvc/realtime/pipeline.py:122-334): RMVPE on the
    convert buffer, f0 shift/autotune/proposed pitch, the realtime float32 coarse quantisation (which,
    unlike the offline pipeline, subtracts the Hz bounds 50/1100 from the mel value, :196-203), circular
    pitch buffers, HuBERT + repeated last frame, index retrieval from skip_head // 2 (:336-352), x2
    upsample [:p_len], protect, ``net_g.infer`` then clip to [-1, 1];
  * ``VoiceChanger.process_audio`` (core.py:404-451): SOLA offset search and the sin^2 crossfade.
  * ``torchaudio.transforms.Resample`` (third-party, torchaudio 2.x ``_get_sinc_resample_kernel`` /
    ``_apply_sinc_resample_kernel``; sinc_interp_hann, lowpass_filter_width 6, rolloff 0.99, kernel in
    float32 as core.py:99-108 request).
VAD (webrtcvad), noise gate (noisereduce) and pedalboard effects are out of scope (off by default).
"""
from __future__ import annotations

import math
from typing import Callable, Optional

import numpy as np
import torch
import torch.nn.functional as F

from oracle import hubert as ohubert
from oracle import rmvpe as ormvpe
from oracle import synth as osynth
from oracle.pipeline import autotune_f0

SAMPLE_RATE = 16000
AUDIO_SAMPLE_RATE = 48000


def sinc_resample_kernel(orig_freq: int, new_freq: int, lowpass_filter_width: int = 6, rolloff: float = 0.99,
                         dtype=torch.float32, resampling_method: str = "sinc_interp_hann", beta=None):
    """torchaudio.functional.functional._get_sinc_resample_kernel (sinc_interp_hann / sinc_interp_kaiser)."""
    gcd = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // gcd, int(new_freq) // gcd
    base_freq = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base_freq)
    idx = torch.arange(-width, width + orig, dtype=dtype)[None, None] / orig
    t = torch.arange(0, -new, -1, dtype=dtype)[:, None, None] / new + idx
    t *= base_freq
    t = t.clamp_(-lowpass_filter_width, lowpass_filter_width)
    if resampling_method == "sinc_interp_hann":
        window = torch.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    else:
        beta_tensor = torch.tensor(float(14.769656459379492 if beta is None else beta))
        window = torch.i0(beta_tensor * torch.sqrt(1 - (t / lowpass_filter_width) ** 2)) / torch.i0(beta_tensor)
    t *= math.pi
    scale = base_freq / orig
    kernels = torch.where(t == 0, torch.tensor(1.0).to(t), t.sin() / t)
    kernels *= window * scale
    return kernels, width, orig, new


def functional_resample(waveform: torch.Tensor, orig_freq: int, new_freq: int, lowpass_filter_width: int = 6,
                        rolloff: float = 0.99, resampling_method: str = "sinc_interp_hann", beta=None) -> torch.Tensor:
    """torchaudio.functional.resample (kernel in the waveform's dtype; any leading dims)."""
    if orig_freq == new_freq:
        return waveform
    kernel, width, orig, new = sinc_resample_kernel(orig_freq, new_freq, lowpass_filter_width, rolloff,
                                                    waveform.dtype, resampling_method, beta)
    shape = waveform.size()
    w = waveform.reshape(-1, shape[-1])
    length = w.shape[-1]
    w = F.pad(w, (width, width + orig))
    y = F.conv1d(w[:, None], kernel, stride=orig)
    y = y.transpose(1, 2).reshape(w.shape[0], -1)
    target = int(math.ceil(new * length / orig))
    return y[..., :target].reshape(shape[:-1] + (min(target, y.shape[-1]),))


def resample(x: torch.Tensor, orig_freq: int, new_freq: int) -> torch.Tensor:
    """torchaudio.transforms.Resample(orig, new, dtype=float32)(x) for a 1-D float32 waveform."""
    if orig_freq == new_freq:
        return x
    kernel, width, orig, new = sinc_resample_kernel(orig_freq, new_freq)
    length = x.shape[-1]
    w = F.pad(x.view(1, 1, -1), (width, width + orig))
    y = F.conv1d(w, kernel, stride=orig)
    y = y.transpose(1, 2).reshape(1, -1)
    target = int(math.ceil(new * length / orig))
    return y[0, :target]


def circular_write(new_data: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """rvc/realtime/utils/torch.py:4-8."""
    offset = new_data.shape[0]
    target[:-offset] = target[offset:].detach().clone()
    target[-offset:] = new_data
    return target


class OracleVoiceChanger:
    """VoiceChanger + Realtime + Realtime_Pipeline over the oracle models (one stream)."""

    def __init__(self, synth_w, synth_cfg, hubert_w, hubert_cfg, rmvpe_w, rmvpe_cfg, read_chunk_size: int = 192,
                 cross_fade_overlap_size: float = 0.1, extra_convert_size: float = 0.5, silent_threshold: int = 0,
                 sid: int = 0, version: str = "v2", index=None, noise_fn: Optional[Callable] = None):
        self.sw, self.sc = synth_w, synth_cfg
        self.hw, self.hc = hubert_w, hubert_cfg
        self.rw, self.rc = rmvpe_w, rmvpe_cfg
        self.version = version
        self.index = index
        self.big_npy = None
        if index is not None:
            from oracle import ivf

            self.big_npy = ivf.reconstruct_n(index, 0, index.ntotal)
        self.noise_fn = noise_fn or (lambda shape, which: torch.randn(shape))
        self.sid = torch.tensor([sid]).long()
        self.tgt_sr = synth_cfg.sr
        self.model_window = self.tgt_sr // 100
        # VoiceChanger.__init__ (core.py:329-374)
        self.block_frame = read_chunk_size * 128
        self.crossfade_frame = int(cross_fade_overlap_size * AUDIO_SAMPLE_RATE)
        self.extra_frame = int(extra_convert_size * AUDIO_SAMPLE_RATE)
        self.sola_search_frame = AUDIO_SAMPLE_RATE // 100
        # Realtime.__init__ (core.py:36-110)
        self.sample_rate = SAMPLE_RATE
        self.silence_front = 0
        self.input_sensitivity = 10 ** (silent_threshold / 20)
        self.window_size = self.sample_rate // 100
        self.realloc(self.block_frame, self.extra_frame, self.crossfade_frame, self.sola_search_frame)
        self.generate_strength()
        self.last = {}

    # ---------------------------------------------------------------- core.py:165-216
    def realloc(self, block_frame, extra_frame, crossfade_frame, sola_search_frame):
        block_frame_16k = int(block_frame / AUDIO_SAMPLE_RATE * self.sample_rate)
        crossfade_frame_16k = int(crossfade_frame / AUDIO_SAMPLE_RATE * self.sample_rate)
        sola_search_frame_16k = int(sola_search_frame / AUDIO_SAMPLE_RATE * self.sample_rate)
        extra_frame_16k = int(extra_frame / AUDIO_SAMPLE_RATE * self.sample_rate)
        convert_size_16k = block_frame_16k + sola_search_frame_16k + extra_frame_16k + crossfade_frame_16k
        if (modulo := convert_size_16k % self.window_size) != 0:
            convert_size_16k = convert_size_16k + (self.window_size - modulo)
        self.convert_feature_size_16k = convert_size_16k // self.window_size
        self.skip_head = extra_frame_16k // self.window_size
        self.return_length = self.convert_feature_size_16k - self.skip_head
        self.silence_front = extra_frame_16k - (self.window_size * 5) if self.silence_front else 0
        self.audio_buffer = torch.zeros(block_frame_16k + crossfade_frame_16k, dtype=torch.float32)
        self.convert_buffer = torch.zeros(convert_size_16k, dtype=torch.float32)
        self.pitch_buffer = torch.zeros(self.convert_feature_size_16k + 1, dtype=torch.int64)
        self.pitchf_buffer = torch.zeros(self.convert_feature_size_16k + 1, dtype=torch.float32)

    def generate_strength(self):
        """core.py:376-402."""
        self.fade_in_window = torch.sin(0.5 * np.pi * torch.linspace(0.0, 1.0, steps=self.crossfade_frame,
                                                                    dtype=torch.float32)) ** 2
        self.fade_out_window = 1 - self.fade_in_window
        self.sola_buffer = torch.zeros(self.crossfade_frame, dtype=torch.float32)

    # ---------------------------------------------------------------- pipeline.py:122-212
    def get_f0(self, x, pitch, pitchf, f0_up_key=0, f0_autotune=False, f0_autotune_strength=1.0,
               proposed_pitch=False, proposed_pitch_threshold=155.0):
        x = x.cpu().numpy()
        f0, _ = ormvpe.infer_from_audio(self.rw, self.rc, x, thred=0.03)
        if f0_autotune is True:
            f0 = autotune_f0(f0, f0_autotune_strength)
        elif proposed_pitch is True:
            valid = np.where(f0 > 0)[0]
            if len(valid) < 2:
                up_key = 0
            else:
                med = float(np.median(np.interp(np.arange(len(f0)), valid, f0[valid])))
                up_key = 0 if (med <= 0 or np.isnan(med)) else max(
                    -12, min(12, int(np.round(12 * np.log2(proposed_pitch_threshold / med)))))
            f0 *= pow(2, (f0_up_key + up_key) / 12)
        else:
            f0 *= pow(2, f0_up_key / 12)
        f0 = torch.from_numpy(f0).float()
        f0_mel = 1127.0 * torch.log(1.0 + f0 / 700.0)
        f0_mel = torch.clip((f0_mel - 50.0) * 254 / (1100.0 - 50.0) + 1, 1, 255, out=f0_mel)
        f0_coarse = torch.round(f0_mel, out=f0_mel).long()
        circular_write(f0_coarse, pitch)
        circular_write(f0, pitchf)
        return pitch.unsqueeze(0), pitchf.unsqueeze(0)

    # ---------------------------------------------------------------- pipeline.py:214-334
    def voice_conversion(self, audio, pitch, pitchf, f0_up_key=0, index_rate=0.5, p_len=0, silence_front=0,
                         skip_head=None, return_length=None, protect=0.5, volume_envelope=1, f0_autotune=False,
                         f0_autotune_strength=1, proposed_pitch=False, proposed_pitch_threshold=155.0):
        with torch.no_grad():
            formant_length = int(np.ceil(return_length * 1.0))
            pitch, pitchf = self.get_f0(audio[silence_front:], pitch, pitchf, f0_up_key, f0_autotune,
                                        f0_autotune_strength, proposed_pitch, proposed_pitch_threshold)
            feats = ohubert.hubert_forward(self.hw, self.hc, audio.view(1, -1), self.version)
            feats = torch.cat((feats, feats[:, -1:, :]), 1)
            feats0 = feats.detach().clone()
            if self.index is not None and index_rate > 0:
                from oracle import ivf

                skip_offset = skip_head // 2
                npy = feats[0][skip_offset:].cpu().numpy()
                score, ix = ivf.search(self.index, npy, 8)
                feats[0][skip_offset:] = torch.from_numpy(
                    ivf.retrieve_speaker_embeddings(npy, score, ix, self.big_npy, index_rate))
            feats = F.interpolate(feats.permute(0, 2, 1), scale_factor=2).permute(0, 2, 1)[:, :p_len, :]
            feats0 = F.interpolate(feats0.permute(0, 2, 1), scale_factor=2).permute(0, 2, 1)[:, :p_len, :]
            pitch, pitchf = pitch[:, -p_len:], pitchf[:, -p_len:] * (formant_length / return_length)
            if protect < 0.5:
                pitchff = pitchf.detach().clone()
                pitchff[pitchf > 0] = 1
                pitchff[pitchf < 1] = protect
                feats = feats * pitchff.unsqueeze(-1) + feats0 * (1 - pitchff.unsqueeze(-1))
            T = feats.shape[1]
            eps_z = self.noise_fn((1, self.sc.inter_channels, T), "z")
            eps_src = self.noise_fn((1, T * self.sc.upp), "src")
            out = osynth.synth_infer(self.sw, self.sc, feats.float(), torch.tensor([p_len]).long(), pitch,
                                     pitchf.float(), self.sid, eps_z, eps_src)[0][0, 0]
            out = torch.clip(out, -1.0, 1.0)
            if volume_envelope != 1:
                from oracle.pipeline import change_rms

                out = torch.as_tensor(change_rms(audio.cpu().numpy(), self.sample_rate, out.numpy(), self.tgt_sr,
                                                 volume_envelope))
            return out

    # ---------------------------------------------------------------- core.py:217-326
    def inference(self, audio_input, f0_up_key=0, index_rate=0.5, protect=0.5, volume_envelope=1,
                  f0_autotune=False, f0_autotune_strength=1, proposed_pitch=False, proposed_pitch_threshold=155.0):
        audio_input_16k = resample(torch.as_tensor(audio_input, dtype=torch.float32), AUDIO_SAMPLE_RATE,
                                   self.sample_rate)
        circular_write(audio_input_16k, self.audio_buffer)
        vol_t = torch.sqrt(torch.square(self.audio_buffer).mean())
        vol = max(vol_t.item(), 0)
        args = (f0_up_key, index_rate, self.convert_feature_size_16k, self.silence_front, self.skip_head,
                self.return_length, protect, volume_envelope, f0_autotune, f0_autotune_strength, proposed_pitch,
                proposed_pitch_threshold)
        if vol < self.input_sensitivity:
            audio_model = self.voice_conversion(self.convert_buffer, self.pitch_buffer, self.pitchf_buffer, *args)
            return torch.zeros(audio_model.shape, dtype=torch.float32), vol
        circular_write(audio_input_16k, self.convert_buffer)
        audio_model = self.voice_conversion(self.convert_buffer, self.pitch_buffer, self.pitchf_buffer, *args)
        audio_out = resample(audio_model * torch.sqrt(vol_t), self.tgt_sr, AUDIO_SAMPLE_RATE)
        return audio_out, vol

    # ---------------------------------------------------------------- core.py:404-451
    def process_audio(self, audio_input, f0_up_key=0, index_rate=0.5, protect=0.5, volume_envelope=1,
                      f0_autotune=False, f0_autotune_strength=1, proposed_pitch=False, proposed_pitch_threshold=155.0):
        block_size = audio_input.shape[0]
        audio, vol = self.inference(audio_input, f0_up_key, index_rate, protect, volume_envelope, f0_autotune,
                                    f0_autotune_strength, proposed_pitch, proposed_pitch_threshold)
        conv_input = audio[None, None, : self.crossfade_frame + self.sola_search_frame]
        cor_nom = F.conv1d(conv_input, self.sola_buffer[None, None, :])
        cor_den = torch.sqrt(F.conv1d(conv_input ** 2, torch.ones(1, 1, self.crossfade_frame)) + 1e-8)
        sola_offset = torch.argmax(cor_nom[0, 0] / cor_den[0, 0])
        self.last["sola_offset"] = int(sola_offset)
        audio = audio[sola_offset:]
        audio[: self.crossfade_frame] *= self.fade_in_window
        audio[: self.crossfade_frame] += self.sola_buffer * self.fade_out_window
        self.sola_buffer[:] = audio[block_size: block_size + self.crossfade_frame]
        return audio[:block_size].detach().cpu().numpy(), vol

    def on_request(self, audio_input, *a, **kw):
        """core.py:453-484 (latency entry omitted)."""
        with torch.no_grad():
            return self.process_audio(audio_input, *a, **kw)
