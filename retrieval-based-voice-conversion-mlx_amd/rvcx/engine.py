"""Device engine: one rvcx context (weights + workspace in HBM) driven through the C-ABI.

torch is used only for device memory and the current HIP stream; every computation runs in
librvcx.so (HIP kernels for gfx950).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Mapping, Optional

import numpy as np

from . import _lib
from .config import SYNTH_48K_V2, SynthConfig
from .weights import normalize_state


def _ptr(t) -> Optional[int]:
    return None if t is None else t.data_ptr()


class Engine:
    """Owns an ``rvcx_ctx`` on one GPU. Not thread-safe (one host thread at a time)."""

    def __init__(self, device: int = 0):
        import torch

        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise RuntimeError("rvcx needs a ROCm GPU: torch.cuda.is_available() is False")
        self.torch = torch
        self.device_index = int(device)
        self.device = torch.device(f"cuda:{self.device_index}")
        ctx = ctypes.c_void_p()
        rc = self.lib.rvcx_create(ctypes.byref(ctx), self.device_index)
        if rc != 0:
            raise _lib.RvcxError(rc, f"rvcx_create(device={device}) failed")
        self.ctx = ctx
        self.synth_cfg: Optional[SynthConfig] = None
        self.loaded = {"synth": False, "hubert": False, "rmvpe": False, "crepe": None}

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.rvcx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ plumbing
    def _check(self, rc: int, what: str):
        if rc != 0:
            msg = self.lib.rvcx_last_error(self.ctx)
            raise _lib.RvcxError(rc, f"{what}: {msg.decode() if msg else ''}")

    def check_device_status(self):
        """Synchronise the current stream and raise RvcxError(RVCX_E_HIP) if a kernel of an earlier call raised
        a device-side fault flag (e.g. the RMVPE BiGRU hand-off timed out: that call's outputs are invalid)."""
        self._check(self.lib.rvcx_device_status(self.ctx, self.stream()), "device status")

    def host(self, t):
        """Device tensor -> numpy at the API edge: synchronises, then raises RvcxError if a kernel of this (or an
        earlier) call raised a device-side fault flag, so a faulted result never leaves as data."""
        self.check_device_status()
        return t.cpu().numpy()

    def stream(self) -> int:
        return self.torch.cuda.current_stream(self.device).cuda_stream

    def _dev(self, x, dtype):
        t = self.torch
        if isinstance(x, t.Tensor):
            return x.to(device=self.device, dtype=dtype).contiguous()
        return t.as_tensor(np.ascontiguousarray(x), dtype=dtype, device=self.device).contiguous()

    # ------------------------------------------------------------------ weights
    def set_synth_config(self, cfg: SynthConfig = SYNTH_48K_V2):
        d = _lib.SynthDesc()
        d.inter_channels, d.hidden_channels, d.filter_channels = cfg.inter_channels, cfg.hidden_channels, \
            cfg.filter_channels
        d.n_heads, d.n_layers, d.kernel_size = cfg.n_heads, cfg.n_layers, cfg.kernel_size
        d.n_resblocks = len(cfg.resblock_kernel_sizes)
        d.n_dilations = len(cfg.resblock_dilation_sizes[0])
        for j, k in enumerate(cfg.resblock_kernel_sizes):
            d.resblock_kernel_sizes[j] = k
            for m, dd in enumerate(cfg.resblock_dilation_sizes[j]):
                d.resblock_dilation_sizes[j][m] = dd
        d.n_upsample = len(cfg.upsample_rates)
        for i, (u, k) in enumerate(zip(cfg.upsample_rates, cfg.upsample_kernel_sizes)):
            d.upsample_rates[i] = u
            d.upsample_kernel_sizes[i] = k
        d.upsample_initial_channel = cfg.upsample_initial_channel
        d.spk_embed_dim, d.gin_channels, d.sr = cfg.spk_embed_dim, cfg.gin_channels, cfg.sr
        d.text_enc_hidden_dim = cfg.text_enc_hidden_dim
        d.no_f0 = 0 if cfg.use_f0 else 1
        if cfg.vocoder not in _lib.VOCODERS:
            raise ValueError(f"unknown vocoder {cfg.vocoder!r}; expected one of {sorted(_lib.VOCODERS)}")
        d.vocoder = _lib.VOCODERS[cfg.vocoder]
        self._check(self.lib.rvcx_set_synth_config(self.ctx, ctypes.byref(d)), "set_synth_config")
        self.synth_cfg = cfg

    def upload_state(self, model: int, state: Mapping[str, np.ndarray]):
        """Upload a fused fp32 state dict (reference names and layouts) and finalize it."""
        for name, arr in state.items():
            a = np.ascontiguousarray(arr, dtype=np.float32)
            shape = (ctypes.c_int64 * max(1, a.ndim))(*a.shape)
            self._check(self.lib.rvcx_upload(self.ctx, model, name.encode(), a.ctypes.data, shape, a.ndim),
                        f"upload {name}")
        self._check(self.lib.rvcx_finalize(self.ctx, model), "finalize")

    def load_synth(self, state: Mapping[str, np.ndarray], cfg: SynthConfig = SYNTH_48K_V2):
        self.set_synth_config(cfg)
        st = {k: v for k, v in normalize_state(state).items() if not k.startswith("enc_q.")}
        self.upload_state(_lib.RVCX_MODEL_SYNTH, st)
        self.loaded["synth"] = True

    def load_hubert(self, state: Mapping[str, np.ndarray]):
        st = {k: v for k, v in normalize_state(state).items() if k != "masked_spec_embed"}
        self.upload_state(_lib.RVCX_MODEL_HUBERT, st)
        self.loaded["hubert"] = True

    def load_rmvpe(self, state: Mapping[str, np.ndarray]):
        self.upload_state(_lib.RVCX_MODEL_RMVPE, normalize_state(state))
        self.loaded["rmvpe"] = True

    def load_crepe(self, state: Mapping[str, np.ndarray], key=None):
        """CREPE weights under torchcrepe's names (rvcx.weights.load_crepe_weights); the context holds one CREPE
        model at a time (full or tiny, told apart by conv1's filter count). `key` names what was loaded so callers
        can skip a reload."""
        self.upload_state(_lib.RVCX_MODEL_CREPE, {k: v for k, v in state.items() if not k.endswith("num_batches_tracked")})
        self.loaded["crepe"] = key if key is not None else ("full" if np.shape(state["conv1.weight"])[0] == 1024
                                                           else "tiny")

    def crepe(self, audio, f0_min: float = 50.0, f0_max: float = 1100.0, threshold: float = 0.1,
              want_periodicity: bool = False, want_probs: bool = False, semantics: str = "mlx", dither=None):
        """CREPE.get_f0 (rvc_mlx/lib/mlx/crepe.py:282-325): audio [N] (16 kHz) -> f0 fp32 [1 + N//160] on device
        (and the filtered periodicity [F], the probabilities [F, 360]). semantics="rvc": rvc/'s CREPE.get_f0
        (torchcrepe.predict + viterbi, rvc/lib/predictors/f0.py:31-55; rvcx_crepe_ex); dither: its [F] cents noise
        (torchcrepe draws scipy.stats.triang(c=0.5, loc=-20, scale=40)), None = none."""
        t = self.torch
        a = self._dev(audio, t.float32).reshape(-1)
        n = a.numel()
        F = 1 + n // 160
        f0 = t.empty((F,), dtype=t.float32, device=self.device)
        per = t.empty((F,), dtype=t.float32, device=self.device) if want_periodicity else None
        probs = t.empty((F, 360), dtype=t.float32, device=self.device) if want_probs else None
        fo = ctypes.c_int64(0)
        sem = {"mlx": 0, "rvc": 1}[semantics]
        d = None if dither is None else self._dev(dither, t.float32).reshape(-1)
        if d is not None and d.numel() != F:
            raise ValueError(f"dither needs {F} values")
        self._check(self.lib.rvcx_crepe_ex(self.ctx, a.data_ptr(), n, float(f0_min), float(f0_max), float(threshold),
                                           sem, _ptr(d), f0.data_ptr(), _ptr(per), _ptr(probs), F, ctypes.byref(fo),
                                           self.stream()), "crepe")
        out = [f0]
        if want_periodicity:
            out.append(per)
        if want_probs:
            out.append(probs)
        return out[0] if len(out) == 1 else tuple(out)

    def crepe_decode(self, probs, f0_min: float = 50.0, f0_max: float = 1100.0, threshold: float = 0.1,
                     semantics: str = "rvc", dither=None):
        """rvcx_crepe_decode: the decode + filters alone on probabilities [F][360] -> (f0 [F], periodicity [F])."""
        t = self.torch
        p = self._dev(probs, t.float32).contiguous()
        F = int(p.shape[0])
        f0 = t.empty((F,), dtype=t.float32, device=self.device)
        per = t.empty((F,), dtype=t.float32, device=self.device)
        d = None if dither is None else self._dev(dither, t.float32).reshape(-1)
        self._check(self.lib.rvcx_crepe_decode(self.ctx, p.data_ptr(), F, float(f0_min), float(f0_max),
                                               float(threshold), {"mlx": 0, "rvc": 1}[semantics], _ptr(d),
                                               f0.data_ptr(), per.data_ptr(), self.stream()), "crepe_decode")
        return f0, per

    @property
    def upp(self) -> int:
        return int(self.lib.rvcx_synth_upp(self.ctx))

    # ------------------------------------------------------------------ compute
    def hubert(self, audio, version: str = "v2"):
        """audio [N] (16 kHz) -> feats [L, 768] (v2) / [L, 256] (v1), fp32 on device."""
        t = self.torch
        a = self._dev(audio, t.float32).reshape(-1)
        n = a.numel()
        cap = n // 320 + 8
        D = 256 if version == "v1" else 768
        out = t.empty((cap, D), dtype=t.float32, device=self.device)
        rows = ctypes.c_int64(0)
        self._check(self.lib.rvcx_hubert(self.ctx, a.data_ptr(), n, 1 if version == "v1" else 2, out.data_ptr(), cap,
                                         ctypes.byref(rows), self.stream()), "hubert")
        return out[: rows.value]

    def rmvpe(self, audio, thred: float = 0.03, want_hidden: bool = False):
        """audio [N] (16 kHz) -> f0 fp64 [1 + N//160] on device (and salience [F, 360])."""
        t = self.torch
        a = self._dev(audio, t.float32).reshape(-1)
        n = a.numel()
        F = 1 + n // 160
        f0 = t.empty((F,), dtype=t.float64, device=self.device)
        hid = t.empty((F, 360), dtype=t.float32, device=self.device) if want_hidden else None
        fo = ctypes.c_int64(0)
        self._check(self.lib.rvcx_rmvpe(self.ctx, a.data_ptr(), n, float(thred), f0.data_ptr(), F, ctypes.byref(fo),
                                        _ptr(hid), self.stream()), "rmvpe")
        return (f0, hid) if want_hidden else f0

    def hubert_batch(self, audio, version: str = "v2"):
        """audio [B, N] (16 kHz, equal lengths) -> feats [B, L, D] on device in one batched pass."""
        t = self.torch
        a = self._dev(audio, t.float32)
        B, n = int(a.shape[0]), int(a.shape[1])
        D = 256 if version == "v1" else 768
        cap = n // 320 + 8
        out = t.empty((B, cap, D), dtype=t.float32, device=self.device)
        rows = ctypes.c_int64(0)
        self._check(self.lib.rvcx_hubert_batch(self.ctx, a.data_ptr(), n, n, B, 1 if version == "v1" else 2,
                                               out.data_ptr(), cap, ctypes.byref(rows), self.stream()), "hubert_batch")
        L = rows.value
        return out.reshape(-1)[: B * L * D].reshape(B, L, D)

    def rmvpe_batch(self, audio, thred: float = 0.03, want_hidden: bool = False):
        """audio [B, N] (16 kHz, equal lengths) -> f0 fp64 [B, 1 + N//160] (and salience [B, F, 360])."""
        t = self.torch
        a = self._dev(audio, t.float32)
        B, n = int(a.shape[0]), int(a.shape[1])
        F = 1 + n // 160
        f0 = t.empty((B, F), dtype=t.float64, device=self.device)
        hid = t.empty((B, F, 360), dtype=t.float32, device=self.device) if want_hidden else None
        fo = ctypes.c_int64(0)
        self._check(self.lib.rvcx_rmvpe_batch(self.ctx, a.data_ptr(), n, n, B, float(thred), f0.data_ptr(), F,
                                              ctypes.byref(fo), _ptr(hid), self.stream()), "rmvpe_batch")
        return (f0, hid) if want_hidden else f0

    def rmvpe_decode(self, hidden, thred: float = 0.03):
        """RMVPE0Predictor.decode on device: salience [F, 360] -> f0 fp64 [F]."""
        t = self.torch
        h = self._dev(hidden, t.float32).reshape(-1, 360)
        f0 = t.empty((h.shape[0],), dtype=t.float64, device=self.device)
        self._check(self.lib.rvcx_rmvpe_decode(self.ctx, h.data_ptr(), h.shape[0], float(thred), f0.data_ptr(),
                                               self.stream()), "rmvpe_decode")
        return f0

    def f0_post(self, f0, semitones: float):
        """Pitch shift + coarse quantisation on device: (coarse int32, pitchf fp32, f0 fp64)."""
        t = self.torch
        f = self._dev(f0, t.float64).reshape(-1)
        F = f.numel()
        coarse = t.empty((F,), dtype=t.int32, device=self.device)
        pitchf = t.empty((F,), dtype=t.float32, device=self.device)
        fs = t.empty((F,), dtype=t.float64, device=self.device)
        self._check(self.lib.rvcx_f0_post(self.ctx, f.data_ptr(), F, float(semitones), coarse.data_ptr(),
                                          pitchf.data_ptr(), fs.data_ptr(), self.stream()), "f0_post")
        return coarse, pitchf, fs

    def synth_infer(self, phone, lengths, pitch, pitchf, sid, eps_z=None, eps_src=None, seed: int = 0,
                    want_latents: bool = False):
        t = self.torch
        ph = self._dev(phone, t.float32)
        B, T = int(ph.shape[0]), int(ph.shape[1])
        ln = self._dev(lengths, t.int32).reshape(B)
        pc = None if pitch is None else self._dev(pitch, t.int32).reshape(B, T)
        pf = None if pitchf is None else self._dev(pitchf, t.float32).reshape(B, T)
        sd = self._dev(sid, t.int32).reshape(B)
        ez = None if eps_z is None else self._dev(eps_z, t.float32)
        es = None if eps_src is None else self._dev(eps_src, t.float32)
        out = t.empty((B, T * self.upp), dtype=t.float32, device=self.device)
        I = self.synth_cfg.inter_channels
        zp = t.empty((B, T, I), dtype=t.float32, device=self.device) if want_latents else None
        z = t.empty((B, T, I), dtype=t.float32, device=self.device) if want_latents else None
        self._check(self.lib.rvcx_synth_infer(self.ctx, B, T, ph.data_ptr(), ln.data_ptr(), _ptr(pc),
                                              _ptr(pf), sd.data_ptr(), _ptr(ez), _ptr(es),
                                              ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), out.data_ptr(), _ptr(zp),
                                              _ptr(z), self.stream()), "synth_infer")
        return (out, zp, z) if want_latents else out

    def synth_infer_ex(self, phone, lengths, pitch, pitchf, sid, rate=None, eps_z=None, eps_src=None, seed: int = 0):
        """Synthesizer.infer with rate and the full return value (rvcx_synth_infer_ex): -> (out [B][T' upp],
        z_p [B][T'][I], z [B][T'][I], m_p [B][T][I], logs_p [B][T][I]) with T' = T - int(T (1 - rate))."""
        t = self.torch
        ph = self._dev(phone, t.float32)
        B, T = int(ph.shape[0]), int(ph.shape[1])
        ln = self._dev(lengths, t.int32).reshape(B)
        pc = None if pitch is None else self._dev(pitch, t.int32).reshape(B, T)
        pf = None if pitchf is None else self._dev(pitchf, t.float32).reshape(B, T)
        sd = self._dev(sid, t.int32).reshape(B)
        ez = None if eps_z is None else self._dev(eps_z, t.float32)
        es = None if eps_src is None else self._dev(eps_src, t.float32)
        I = self.synth_cfg.inter_channels
        out = t.empty((B, T * self.upp), dtype=t.float32, device=self.device)
        zp = t.empty((B, T, I), dtype=t.float32, device=self.device)
        z = t.empty((B, T, I), dtype=t.float32, device=self.device)
        mp = t.empty((B, T, I), dtype=t.float32, device=self.device)
        lp = t.empty((B, T, I), dtype=t.float32, device=self.device)
        tn = ctypes.c_int(0)
        self._check(self.lib.rvcx_synth_infer_ex(self.ctx, B, T, ph.data_ptr(), ln.data_ptr(), _ptr(pc), _ptr(pf),
                                                 sd.data_ptr(), -1.0 if rate is None else float(rate), _ptr(ez),
                                                 _ptr(es), ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), out.data_ptr(),
                                                 zp.data_ptr(), z.data_ptr(), mp.data_ptr(), lp.data_ptr(),
                                                 ctypes.byref(tn), self.stream()), "synth_infer_ex")
        Tn = int(tn.value)
        return (out.reshape(-1)[: B * Tn * self.upp].reshape(B, Tn * self.upp), zp.reshape(-1)[: B * Tn * I].reshape(B, Tn, I),
                z.reshape(-1)[: B * Tn * I].reshape(B, Tn, I), mp, lp)

    def dec_only(self, z, f0, sid, eps_src=None, seed: int = 0):
        t = self.torch
        zz = self._dev(z, t.float32)
        B, I, T = zz.shape
        f = None if f0 is None else self._dev(f0, t.float32).reshape(B, T)
        sd = self._dev(sid, t.int32).reshape(B)
        es = None if eps_src is None else self._dev(eps_src, t.float32)
        out = t.empty((B, T * self.upp), dtype=t.float32, device=self.device)
        self._check(self.lib.rvcx_dec_only(self.ctx, B, T, zz.data_ptr(), _ptr(f), sd.data_ptr(), _ptr(es),
                                           ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), out.data_ptr(),
                                           self.stream()), "dec_only")
        return out

    def voice_conversion(self, audio_pad, pitch, pitchf, sid: int, protect: float, eps_z=None, eps_src=None,
                         seed: int = 0, index_rate: float = 0.0):
        """HuBERT -> x2 upsample -> protect -> Synthesizer.infer on one padded chunk (device in/out)."""
        t = self.torch
        a = self._dev(audio_pad, t.float32).reshape(-1)
        n = a.numel()
        pc = None if pitch is None else self._dev(pitch, t.int32).reshape(-1)
        pf = None if pitchf is None else self._dev(pitchf, t.float32).reshape(-1)
        cap = (n // 160) * self.upp
        out = t.empty((cap,), dtype=t.float32, device=self.device)
        no = ctypes.c_int64(0)
        ez = None if eps_z is None else self._dev(eps_z, t.float32)
        es = None if eps_src is None else self._dev(eps_src, t.float32)
        self._check(self.lib.rvcx_voice_conversion(self.ctx, a.data_ptr(), n, _ptr(pc), _ptr(pf), int(sid),
                                                   float(protect), float(index_rate), _ptr(ez), _ptr(es),
                                                   ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), out.data_ptr(), cap,
                                                   ctypes.byref(no), self.stream()), "voice_conversion")
        return out[: no.value]

    # ------------------------------------------------------------------ whole pipeline
    def set_highpass(self, b, a, zi, sos=None):
        """The pipeline's high-pass (pipeline.py:22-27) as transfer function (+ lfilter_zi) and, when given,
        as second-order sections (run as a chunk-parallel scan)."""
        b = np.ascontiguousarray(b, dtype=np.float64)
        a = np.ascontiguousarray(a, dtype=np.float64)
        zi = np.ascontiguousarray(zi, dtype=np.float64)
        self._check(self.lib.rvcx_set_highpass(self.ctx, b.ctypes.data, a.ctypes.data, zi.ctypes.data, len(a) - 1),
                    "set_highpass")
        if sos is not None:
            q = np.ascontiguousarray(sos, dtype=np.float64).reshape(-1, 6)
            self._check(self.lib.rvcx_set_highpass_sos(self.ctx, q.ctypes.data, q.shape[0]), "set_highpass_sos")
        self._hp = (b, a, zi)

    def set_pipeline_highpass(self, sr: int = 16000):
        """signal.butter(N=5, Wn=48, btype='high', fs=16000) as rvc/infer/pipeline.py:22-27 designs it."""
        from scipy import signal

        b, a = signal.butter(N=5, Wn=48, btype="high", fs=sr)
        sos = signal.butter(N=5, Wn=48, btype="high", fs=sr, output="sos")
        self.set_highpass(b, a, signal.lfilter_zi(b, a), sos)

    def highpass_pad(self, audio, t_pad: int):
        """filtfilt + reflect pad on device: fp64 [n] -> (fp64, fp32) [n + 2 t_pad]."""
        t = self.torch
        a = self._dev(audio, t.float64).reshape(-1)
        n = a.numel()
        p64 = t.empty((n + 2 * t_pad,), dtype=t.float64, device=self.device)
        p32 = t.empty((n + 2 * t_pad,), dtype=t.float32, device=self.device)
        self._check(self.lib.rvcx_highpass_pad(self.ctx, a.data_ptr(), n, int(t_pad), p64.data_ptr(), p32.data_ptr(),
                                               self.stream()), "highpass_pad")
        return p64, p32

    def pipeline(self, audio, sid: int = 0, semitones: float = 0.0, protect: float = 0.33, t_pad: int = 16000,
                 t_pad_tgt: int = 48000, eps_z=None, eps_src=None, seed: int = 0, out=None, want_f0: bool = False):
        """One utterance (padded length <= t_max) through the whole device pipeline.
        audio: fp64 [n] @16 kHz (device tensor or numpy). Returns fp32 [n_out] on device."""
        t = self.torch
        a = self._dev(audio, t.float64).reshape(-1)
        n = a.numel()
        m = n + 2 * t_pad
        cap = (m // 160) * self.upp
        if out is None:
            out = t.empty((cap,), dtype=t.float32, device=self.device)
        f0 = t.empty((1 + m // 160,), dtype=t.float64, device=self.device) if want_f0 else None
        no = ctypes.c_int64(0)
        ez = None if eps_z is None else self._dev(eps_z, t.float32)
        es = None if eps_src is None else self._dev(eps_src, t.float32)
        self._check(self.lib.rvcx_pipeline(self.ctx, a.data_ptr(), n, int(sid), float(semitones), float(protect),
                                           int(t_pad), int(t_pad_tgt), _ptr(ez), _ptr(es),
                                           ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), out.data_ptr(), out.numel(),
                                           ctypes.byref(no), _ptr(f0), self.stream()), "pipeline")
        res = out[: no.value]
        return (res, f0) if want_f0 else res

    def config_info(self) -> dict:
        """The effective configuration (rvcx_config_info): contraction arithmetic, whether RVCX_* developer knobs are
        honoured (RVCX_EXPERIMENTAL=1), and each RVCX_* variable of the environment."""
        import json

        n = ctypes.c_int64(0)
        self.lib.rvcx_config_info(self.ctx, None, 0, ctypes.byref(n))
        buf = ctypes.create_string_buffer(int(n.value) + 1)
        self._check(self.lib.rvcx_config_info(self.ctx, ctypes.cast(buf, ctypes.c_void_p), len(buf), ctypes.byref(n)),
                    "config_info")
        return json.loads(buf.value.decode())

    def set_generator_precision(self, precision):
        """Removed in round 4: the fp16 streaming generator is a per-hop option (StreamGroup.process(...,
        gen_precision=...), rvcx_rt_opts.gen_precision). Raises RvcxError(RVCX_E_INVALID) with that message."""
        self._check(self.lib.rvcx_set_generator_precision(self.ctx, int(precision)), "set_generator_precision")

    def workspace_bytes(self, n: int, B: int = 1, opts=None) -> int:
        """Device scratch a pipeline call of B utterances of n samples takes (rvcx_workspace_bytes: one call on zero
        audio from an empty pool; the pool is released after)."""
        o = opts if opts is not None else self.pipeline_opts()
        v = ctypes.c_int64(0)
        self._check(self.lib.rvcx_workspace_bytes(self.ctx, int(B), int(n), ctypes.byref(o), ctypes.byref(v),
                                                  self.stream()), "workspace_bytes")
        return int(v.value)

    def set_workspace(self, arena=None):
        """Carve the context's scratch from a caller-owned device tensor (rvcx_set_workspace; None: back to internal
        allocation). The tensor is kept referenced here for as long as it is attached."""
        base = 0 if arena is None else arena.data_ptr()
        nbytes = 0 if arena is None else arena.numel() * arena.element_size()
        self._check(self.lib.rvcx_set_workspace(self.ctx, ctypes.c_void_p(base or None), int(nbytes)),
                    "set_workspace")
        self._arena = arena

    def workspace_info(self):
        """(bytes the pool holds, arena bytes, arena bytes carved)."""
        v = [ctypes.c_int64(0) for _ in range(3)]
        self._check(self.lib.rvcx_workspace_info(self.ctx, *(ctypes.byref(x) for x in v)), "workspace_info")
        return tuple(int(x.value) for x in v)

    def pipeline_opts(self, **kw) -> "_lib.PipelineOpts":
        """rvcx_pipeline_opts with the C defaults, overridden by keyword (field names of the struct)."""
        o = _lib.PipelineOpts()
        self.lib.rvcx_pipeline_default_opts(ctypes.byref(o))
        names = {f[0] for f in _lib.PipelineOpts._fields_}
        for k, v in kw.items():
            if k not in names:
                raise TypeError(f"unknown pipeline option {k!r}")
            setattr(o, k, v)
        return o

    def pipeline_ex(self, audio, opts: "_lib.PipelineOpts", eps_z=None, eps_src=None, seed: int = 0, out=None,
                    want_f0: bool = False):
        """Pipeline.pipeline on device with long-input splitting, f0 adjustments and volume envelope.
        audio: fp64 [n] @16 kHz. Returns fp32 [n_out] on device (and the adjusted f0 when want_f0)."""
        t = self.torch
        a = self._dev(audio, t.float64).reshape(-1)
        n = a.numel()
        m = n + 2 * int(opts.t_pad)
        n_split = n // int(opts.t_center) if opts.t_max > 0 and opts.t_center > 0 else 0
        cap = (m // 160 + n_split + 2) * self.upp
        if out is None or out.numel() < cap:
            out = t.empty((cap,), dtype=t.float32, device=self.device)
        f0 = t.empty((1 + m // 160,), dtype=t.float64, device=self.device) if want_f0 else None
        no = ctypes.c_int64(0)
        ez = None if eps_z is None else self._dev(eps_z, t.float32)
        es = None if eps_src is None else self._dev(eps_src, t.float32)
        self._check(self.lib.rvcx_pipeline_ex(self.ctx, a.data_ptr(), n, ctypes.byref(opts), _ptr(ez), _ptr(es),
                                              ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), out.data_ptr(), out.numel(),
                                              ctypes.byref(no), _ptr(f0), self.stream()), "pipeline_ex")
        res = out[: no.value]
        return (res, f0) if want_f0 else res

    def pipeline_batch(self, audio, opts: "_lib.PipelineOpts", sids=0, eps_z=None, eps_src=None, seed: int = 0,
                       out=None, want_f0: bool = False, want_hidden: bool = False):
        """B equal-length utterances (fp64 [B, n] @16 kHz, each within t_max) through one batched pass.
        Returns fp32 [B, n_out] on device (row b = Pipeline.pipeline of utterance b); with want_f0 / want_hidden
        also the rows' adjusted f0 fp64 [B, F] / RMVPE salience fp32 [B, F, 360]."""
        t = self.torch
        a = self._dev(audio, t.float64)
        B, n = int(a.shape[0]), int(a.shape[1])
        m = n + 2 * int(opts.t_pad)
        ldo = (m // 160) * self.upp
        if out is None or out.numel() < B * ldo:
            out = t.empty((B, ldo), dtype=t.float32, device=self.device)
        sid = np.broadcast_to(np.asarray(sids, dtype=np.int32), (B,))
        sarr = (ctypes.c_int32 * B)(*[int(v) for v in sid])
        no = ctypes.c_int64(0)
        ez = None if eps_z is None else self._dev(eps_z, t.float32)
        es = None if eps_src is None else self._dev(eps_src, t.float32)
        F = 1 + m // 160
        f0 = t.empty((B, F), dtype=t.float64, device=self.device) if want_f0 else None
        hid = t.empty((B, F, 360), dtype=t.float32, device=self.device) if want_hidden else None
        self._check(self.lib.rvcx_pipeline_batch(self.ctx, a.data_ptr(), n, n, B, ctypes.byref(opts), sarr, _ptr(ez),
                                                 _ptr(es), ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF),
                                                 out.data_ptr(), ldo, ctypes.byref(no), _ptr(f0), _ptr(hid),
                                                 self.stream()),
                    "pipeline_batch")
        y = out.reshape(-1)[: B * ldo].reshape(B, ldo)[:, : no.value]
        extra = [v for v, w in ((f0, want_f0), (hid, want_hidden)) if w]
        return (y, *extra) if extra else y

    def f0_autotune(self, f0, strength: float = 1.0, skip_unvoiced: bool = False):
        """Autotune.autotune_f0 on device; returns a new fp64 tensor."""
        t = self.torch
        f = self._dev(f0, t.float64).reshape(-1).clone()
        self._check(self.lib.rvcx_f0_autotune(self.ctx, f.data_ptr(), f.numel(), float(strength),
                                              1 if skip_unvoiced else 0, self.stream()), "f0_autotune")
        return f

    # ------------------------------------------------------------------ feature index (FAISS IVFFlat)
    def index_load(self, data: bytes):
        """Parse a faiss IndexIVFFlat file image and keep it in HBM (faiss.read_index, pipeline.py:430-434)."""
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        self._check(self.lib.rvcx_index_load(self.ctx, buf, len(data)), "index_load")
        self.index_info()

    def index_unload(self):
        self._check(self.lib.rvcx_index_unload(self.ctx), "index_unload")

    def index_info(self):
        """-> dict(d, ntotal, nlist, nprobe), or None when no index is loaded."""
        v = [ctypes.c_int64(0) for _ in range(4)]
        rc = self.lib.rvcx_index_info(self.ctx, *[ctypes.byref(x) for x in v])
        if rc == -5:
            return None
        self._check(rc, "index_info")
        return dict(zip(("d", "ntotal", "nlist", "nprobe"), (x.value for x in v)))

    def index_set_nprobe(self, nprobe: int):
        self._check(self.lib.rvcx_index_set_nprobe(self.ctx, int(nprobe)), "index_set_nprobe")

    def index_search(self, x, k: int = 8):
        """index.search(x, k) on device -> (dist fp32 [n, k], ids int64 [n, k]) device tensors."""
        t = self.torch
        xx = self._dev(x, t.float32)
        xx = xx.reshape(-1, xx.shape[-1])
        n = xx.shape[0]
        dist = t.empty((n, k), dtype=t.float32, device=self.device)
        ids = t.empty((n, k), dtype=t.int64, device=self.device)
        self._check(self.lib.rvcx_index_search(self.ctx, xx.data_ptr(), n, int(k), dist.data_ptr(), ids.data_ptr(),
                                               self.stream()), "index_search")
        return dist, ids

    def index_reconstruct_n(self, i0: int, ni: int):
        info = self.index_info()
        if info is None:
            raise _lib.RvcxError(-5, "no feature index loaded")
        out = self.torch.empty((int(ni), info["d"]), dtype=self.torch.float32, device=self.device)
        self._check(self.lib.rvcx_index_reconstruct_n(self.ctx, int(i0), int(ni), out.data_ptr(), self.stream()),
                    "index_reconstruct_n")
        return out

    def index_retrieve(self, feats, index_rate: float):
        """Pipeline._retrieve_speaker_embeddings on device: feats [L, d] -> blended [L, d]."""
        t = self.torch
        f = self._dev(feats, t.float32)
        f = f.reshape(-1, f.shape[-1])
        out = t.empty_like(f)
        self._check(self.lib.rvcx_index_retrieve(self.ctx, f.data_ptr(), f.shape[0], f.shape[1], float(index_rate),
                                                 out.data_ptr(), self.stream()), "index_retrieve")
        return out

    # ------------------------------------------------------------------ kernel timing
    def set_conv_math(self, mode: str):
        """Contraction arithmetic of this context: "h16" (the default: fp32 via three bf16 planes on bf16 MFMA, the
        generator's weight-streamed convs and fused ResBlock pairs via two fp16 planes), "split" (three bf16 planes
        everywhere) or "f32" (fp32-input MFMA) (rvcx_set_conv_math)."""
        m = {"default": 0, "f32": 1, "split": 2, "h16": 3}[mode]
        self._check(self.lib.rvcx_set_conv_math(self.ctx, m), "set_conv_math")

    def conv1d(self, x, w, bias=None, dilation: int = 1, padding: int = 0, stride: int = 1, math: str = "default"):
        """torch.nn.functional.conv1d(x.T[None], w, bias, stride, padding, dilation)[0].T on the device kernel:
        x [T][C_in] (time-major), w [N][C_in][taps] (torch layout) -> [T_out][N] fp32 (rvcx_conv1d)."""
        torch = self.torch
        x = self._dev(x, torch.float32)
        w = torch.as_tensor(w, dtype=torch.float32)
        N, C, K = (int(v) for v in w.shape)
        wk = self._dev(w.permute(2, 0, 1).contiguous(), torch.float32)
        b = self._dev(bias, torch.float32) if bias is not None else None
        T = int(x.shape[0])
        T_out = (T + 2 * padding - dilation * (K - 1) - 1) // stride + 1
        y = torch.empty((T_out, N), dtype=torch.float32, device=self.device)
        m = {"default": 0, "f32": 1, "split": 2, "wsb": 3, "gs": 4, "h16": 5, "f16": 6, "gs_h16": 7}[math]
        self._check(self.lib.rvcx_conv1d(self.ctx, _ptr(x), T, C, _ptr(wk), _ptr(b), N, K, dilation, padding, stride,
                                         m, _ptr(y), T_out, self.stream()), "conv1d")
        return y

    def conv1d_gen(self, x, w, bias=None, dilation: int = 1, padding: int = 0, pre_slope: float = 0.1,
                   slope=None, res=None, acc=None, acc_mode: int = 0, acc_div: float = 1.0,
                   kernel: str = "policy"):
        """The generator's fused conv (rvcx_conv1d_gen): y = acc(act(conv1d(pre(x), w, bias)) + res), pre = leaky
        ReLU(pre_slope) unless pre_slope is None, act = leaky ReLU(slope) unless slope is None, acc_mode 0 store / 1 add
        / 2 add-then-divide into `acc` (the
        initial y); kernel "policy", "wsb" (weight-streamed) or "wst" (weight-stationary). x [T][C_in], w [N][C_in][taps]
        -> [T_out][N] fp32 in the two-plane fp16 split."""
        torch = self.torch
        x = self._dev(x, torch.float32)
        w = torch.as_tensor(w, dtype=torch.float32)
        N, C, K = (int(v) for v in w.shape)
        wk = self._dev(w.permute(2, 0, 1).contiguous(), torch.float32)
        b = self._dev(bias, torch.float32) if bias is not None else None
        r = self._dev(res, torch.float32) if res is not None else None
        T = int(x.shape[0])
        T_out = T + 2 * padding - dilation * (K - 1)
        if acc is not None:
            y = self._dev(acc, torch.float32).clone()
        else:
            y = torch.empty((T_out, N), dtype=torch.float32, device=self.device)
        kn = {"policy": 0, "wsb": 1, "wst": 2}[kernel]
        self._check(self.lib.rvcx_conv1d_gen(self.ctx, _ptr(x), T, C, _ptr(wk), _ptr(b), N, K, dilation, padding,
                                             0 if pre_slope is None else 1,
                                             0.0 if pre_slope is None else float(pre_slope), 0 if slope is None else 1,
                                             0.0 if slope is None else float(slope), _ptr(r), int(acc_mode),
                                             float(acc_div), kn, _ptr(y), self.stream()), "conv1d_gen")
        return y

    def conv2d3x3(self, x, w, bias=None, relu: bool = False, math: str = "default"):
        """torch.nn.functional.conv2d(x.permute(2, 0, 1)[None], w, bias, padding=1)[0].permute(1, 2, 0) on the device
        kernel: x [H][W][C_in] (NHWC), w [N][C_in][3][3] (torch layout) -> [H][W][N] fp32 (rvcx_conv2d3x3); math
        "default" = the context's arithmetic, "f32" = exact fp32, "gsw" = the U-Net deep levels' windowed kernel in the
        fp16 split (K split over workgroups)."""
        torch = self.torch
        x = self._dev(x, torch.float32)
        w = torch.as_tensor(w, dtype=torch.float32)
        N, C = int(w.shape[0]), int(w.shape[1])
        wk = self._dev(w.permute(2, 3, 0, 1).reshape(9, N, C).contiguous(), torch.float32)
        b = self._dev(bias, torch.float32) if bias is not None else None
        H, W = int(x.shape[0]), int(x.shape[1])
        y = torch.empty((H, W, N), dtype=torch.float32, device=self.device)
        m = {"default": 0, "f32": 1, "gsw": 2}[math]
        self._check(self.lib.rvcx_conv2d3x3(self.ctx, _ptr(x), H, W, C, _ptr(wk), _ptr(b), N, 1 if relu else 0, m,
                                            _ptr(y), self.stream()), "conv2d3x3")
        return y

    def convtranspose2d_s2(self, x, w, bias=None, relu: bool = False, math: str = "default"):
        """torch.nn.functional.conv_transpose2d(x.permute(2, 0, 1)[None], w, bias, stride=2, padding=1,
        output_padding=1)[0].permute(1, 2, 0) on the device (rvcx_convtranspose2d_s2, the U-Net decoder's up-conv as
        the pipeline runs it): x [H][W][C_in] (NHWC), w [C_in][N][3][3] (torch layout) -> [2H][2W][N] fp32; math
        "default" = the context's arithmetic, "f32" = exact fp32."""
        torch = self.torch
        x = self._dev(x, torch.float32)
        wd = self._dev(torch.as_tensor(w, dtype=torch.float32).contiguous(), torch.float32)
        C, N = int(wd.shape[0]), int(wd.shape[1])
        b = self._dev(bias, torch.float32) if bias is not None else None
        H, W = int(x.shape[0]), int(x.shape[1])
        y = torch.empty((2 * H, 2 * W, N), dtype=torch.float32, device=self.device)
        m = {"default": 0, "f32": 1}[math]
        self._check(self.lib.rvcx_convtranspose2d_s2(self.ctx, _ptr(x), H, W, C, _ptr(wd), _ptr(b), N,
                                                     1 if relu else 0, m, _ptr(y), self.stream()), "convtranspose2d_s2")
        return y

    def flash_attention(self, qkv, n_heads: int, qscale: float, rel_k=None, rel_v=None, window: int = 0, mask=None):
        """The fused attention core (rvcx_flash_attention): qkv [B][T][3 H] time-major (q | k | v, heads of dk inside
        each), optional relative tables rel_k / rel_v [2 window + 1][dk] and key/query mask [B][T] -> [B][T][H]."""
        torch = self.torch
        q = self._dev(qkv, torch.float32)
        B, T, H3 = (int(v) for v in q.shape)
        dk = H3 // 3 // n_heads
        rk = None if rel_k is None else self._dev(rel_k, torch.float32)
        rv = None if rel_v is None else self._dev(rel_v, torch.float32)
        mk = None if mask is None else self._dev(mask, torch.float32)
        y = torch.empty((B, T, H3 // 3), dtype=torch.float32, device=self.device)
        self._check(self.lib.rvcx_flash_attention(self.ctx, _ptr(q), B, T, int(n_heads), dk, float(qscale), _ptr(rk),
                                                  _ptr(rv), int(window), _ptr(mk), _ptr(y), self.stream()),
                    "flash_attention")
        return y

    def resblock_pair(self, x, w1, b1, w2, b2, dilation: int, acc=None, acc_mode: int = 0, acc_div: float = 1.0,
                      cfg: int = 0):
        """One ResBlock dilation pair on the fused kernel (rvcx_resblock_pair): x [B][T][C] time-major, w1/w2
        [C][C][k] (torch layout) -> conv2(lrelu(conv1_d(lrelu(x)) + b1)) + b2 + x, stored (acc_mode 0) or
        accumulated into `acc` (1: acc + out, 2: (acc + out) / acc_div)."""
        torch = self.torch
        x = self._dev(x, torch.float32)
        B, T, C = (int(v) for v in x.shape)
        k = int(np.shape(w1)[2])
        w1k = self._dev(torch.as_tensor(w1, dtype=torch.float32).permute(2, 0, 1).contiguous(), torch.float32)
        w2k = self._dev(torch.as_tensor(w2, dtype=torch.float32).permute(2, 0, 1).contiguous(), torch.float32)
        b1d, b2d = self._dev(b1, torch.float32), self._dev(b2, torch.float32)
        y = (self._dev(acc, torch.float32).clone() if acc is not None
             else torch.empty((B, T, C), dtype=torch.float32, device=self.device))
        self._check(self.lib.rvcx_resblock_pair(self.ctx, _ptr(x), B, T, C, _ptr(w1k), _ptr(b1d), _ptr(w2k), _ptr(b2d),
                                                k, dilation, acc_mode, float(acc_div), cfg, _ptr(y), self.stream()),
                    "resblock_pair")
        return y

    def profile(self, enable: bool):
        self._check(self.lib.rvcx_profile(self.ctx, 1 if enable else 0), "profile")

    def profile_read(self, with_ceiling: bool = False):
        """(summed conv-GEMM kernel ms, summed algorithmic FLOPs, launches) since the last read; with_ceiling adds
        the same launches' time at their arithmetic's MFMA ceiling (ms, rvcx_profile_read_ex)."""
        ms, fl, n, cm = ctypes.c_double(0), ctypes.c_double(0), ctypes.c_int64(0), ctypes.c_double(0)
        self._check(self.lib.rvcx_profile_read_ex(self.ctx, ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(n),
                                                  ctypes.byref(cm)), "profile_read")
        return (ms.value, fl.value, n.value, cm.value) if with_ceiling else (ms.value, fl.value, n.value)

    def profile_read_kinds(self):
        """((ms, flops, launches, ceiling_ms) totals, {kernel family: {ms, flops, ceiling_ms, bytes, launches}}) since
        the last read (rvcx_profile_read_kinds: grouped by the kernel each launch actually ran)."""
        K = 10  # RVCX_PROF_KINDS
        arr = lambda T: (T * K)()  # noqa: E731
        kms, kfl, kcm, kby, kn = arr(ctypes.c_double), arr(ctypes.c_double), arr(ctypes.c_double), \
            arr(ctypes.c_double), arr(ctypes.c_int64)
        ms, fl, n, cm = ctypes.c_double(0), ctypes.c_double(0), ctypes.c_int64(0), ctypes.c_double(0)
        self._check(self.lib.rvcx_profile_read_kinds(self.ctx, ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(n),
                                                     ctypes.byref(cm), K, kms, kfl, kcm, kby, kn), "profile_read_kinds")
        fam = {}
        for k in range(K):
            if kn[k]:
                fam[self.lib.rvcx_profile_kind_name(k).decode()] = {"ms": kms[k], "flops": kfl[k], "ceiling_ms": kcm[k],
                                                                    "bytes": kby[k], "launches": int(kn[k])}
        return (ms.value, fl.value, n.value, cm.value), fam
