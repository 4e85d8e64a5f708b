"""Streaming voice conversion on MI355X (config C5) -- the rvc/realtime surface.

Mirrors rvc/realtime/core.py (``VoiceChanger`` :329-484 with ``process_audio`` / ``on_request``,
``Realtime`` :36-326) and the per-hop semantics of rvc/realtime/pipeline.py (``Realtime_Pipeline``
:99-352). The MLX port of this path (rvc_mlx/realtime) is not functional, so the
PyTorch path's behaviour is the contract.

``StreamGroup`` converts B concurrent streams of one geometry per hop in one device call
(``rvcx_rt_process``: resample, circular buffers, RMS gate, RMVPE, HuBERT, retrieval, one batched
Synthesizer.infer, SOLA crossfade -- all HIP kernels). ``VoiceChanger`` is the one-stream, numpy-in /
numpy-out object of the reference. Audio I/O, VAD, noise gate and pedalboard effects are not part of
this path.
"""
from __future__ import annotations

import ctypes
import time
from typing import Optional, Sequence

import numpy as np

from . import _lib
from .engine import Engine

GEOMETRY_FIELDS = ("n_streams", "block48", "block16", "convert16", "frames", "skip_head", "return_length",
                   "crossfade48", "sola_search48", "extra48", "resampled_block16", "silence_front")


def _ptr(t):
    return None if t is None else t.data_ptr()


class StreamGroup:
    """B streams sharing one buffer geometry, converted together each hop on one Engine."""

    def __init__(self, engine: Engine, n_streams: int = 1, read_chunk_size: int = 192,
                 cross_fade_overlap_size: float = 0.1, extra_convert_size: float = 0.5,
                 silent_threshold: float = -90.0, sid=0):
        self.engine = engine
        lib = engine.lib
        d = _lib.RtDesc()
        lib.rvcx_rt_default_desc(ctypes.byref(d))
        d.n_streams, d.read_chunk_size = int(n_streams), int(read_chunk_size)
        d.cross_fade_overlap_size, d.extra_convert_size = float(cross_fade_overlap_size), float(extra_convert_size)
        d.silent_threshold = float(silent_threshold)
        h = ctypes.c_void_p()
        engine._check(lib.rvcx_rt_create(engine.ctx, ctypes.byref(d), ctypes.byref(h)), "rt_create")
        self.handle = h
        g = (ctypes.c_int64 * 12)()
        engine._check(lib.rvcx_rt_geometry(h, g), "rt_geometry")
        self.geometry = dict(zip(GEOMETRY_FIELDS, list(g)))
        self.n_streams = self.geometry["n_streams"]
        self.block_frame = self.geometry["block48"]
        sids = np.broadcast_to(np.asarray(sid, dtype=np.int32), (self.n_streams,))
        self.sids = (ctypes.c_int32 * self.n_streams)(*[int(v) for v in sids])
        t = engine.torch
        self.out = t.empty((self.n_streams, self.block_frame), dtype=t.float32, device=engine.device)
        self.vol = t.empty((self.n_streams,), dtype=t.float32, device=engine.device)
        self.offs = t.empty((self.n_streams,), dtype=t.int32, device=engine.device)

    def close(self):
        if getattr(self, "handle", None):
            self.engine.lib.rvcx_rt_destroy(self.engine.ctx, self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        self.engine._check(self.engine.lib.rvcx_rt_reset(self.engine.ctx, self.handle, self.engine.stream()),
                           "rt_reset")

    def opts(self, f0_up_key=0, index_rate=0.5, protect=0.5, volume_envelope=1.0, f0_autotune=False,
             f0_autotune_strength=1.0, proposed_pitch=False, proposed_pitch_threshold=155.0,
             gen_precision: str = "fp32") -> _lib.RtOpts:
        """Per-hop options (rvcx_rt_opts). gen_precision "fp16" runs this hop's generator on fp16 operands (BASELINE
        C5's half precision); the f0 / feature front end, TextEncoder and flow stay fp32-accurate either way."""
        o = _lib.RtOpts()
        self.engine.lib.rvcx_rt_default_opts(ctypes.byref(o))
        # rvc/realtime only retrieves when an index is loaded (pipeline.py:264); index_rate alone does not
        loaded = self.engine.index_info() is not None
        o.f0_up_key, o.index_rate, o.protect = float(f0_up_key), float(index_rate) if loaded else 0.0, float(protect)
        o.volume_envelope, o.f0_autotune = float(volume_envelope), int(bool(f0_autotune))
        o.f0_autotune_strength, o.proposed_pitch = float(f0_autotune_strength), int(bool(proposed_pitch))
        o.proposed_pitch_threshold = float(proposed_pitch_threshold)
        o.gen_precision = {"fp32": 0, "fp16": 1}[gen_precision]
        return o

    def process(self, audio_in, opts: Optional[_lib.RtOpts] = None, eps_z=None, eps_src=None, seed: int = 0):
        """One hop for every stream: audio_in [B, block48] @48 kHz (device tensor or numpy) ->
        (out [B, block48] device tensor, vol [B] device tensor). Asynchronous on the current stream."""
        eng = self.engine
        t = eng.torch
        x = eng._dev(audio_in, t.float32).reshape(self.n_streams, self.block_frame)
        ez = None if eps_z is None else eng._dev(eps_z, t.float32)
        es = None if eps_src is None else eng._dev(eps_src, t.float32)
        o = opts if opts is not None else self.opts()
        eng._check(eng.lib.rvcx_rt_process(eng.ctx, self.handle, x.data_ptr(), self.sids, ctypes.byref(o), _ptr(ez),
                                           _ptr(es), ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), self.out.data_ptr(),
                                           self.vol.data_ptr(), self.offs.data_ptr(), eng.stream()), "rt_process")
        return self.out, self.vol


class VoiceChanger:
    """One realtime stream with the reference's API (rvc/realtime/core.py:329-484).

    ``VoiceChanger(read_chunk_size, cross_fade_overlap_size, extra_convert_size, engine=..., sid=0,
    silent_threshold=0)`` then ``on_request(audio_input @48k) -> (audio_out np.float32 [block], vol, [0, ms, 0])``.
    Models come from the Engine (``rvcx.infer.RVCX(...).engine`` or an Engine loaded by hand); an index
    loaded on that Engine (``rvcx.infer.read_index``) is used when index_rate > 0.
    """

    def __init__(self, read_chunk_size: int, cross_fade_overlap_size: float, extra_convert_size: float,
                 engine: Engine = None, silent_threshold: int = 0, sid: int = 0, **_unused):
        if engine is None:
            raise ValueError("VoiceChanger needs an rvcx Engine with the synthesizer, HuBERT and RMVPE loaded")
        self.group = StreamGroup(engine, 1, read_chunk_size, cross_fade_overlap_size, extra_convert_size,
                                 silent_threshold, sid)
        g = self.group.geometry
        self.block_frame, self.crossfade_frame = g["block48"], g["crossfade48"]
        self.sola_search_frame, self.extra_frame = g["sola_search48"], g["extra48"]
        self.seed = 0

    def process_audio(self, audio_input: np.ndarray, f0_up_key=0, index_rate=0.5, protect=0.5, volume_envelope=1,
                      f0_autotune=False, f0_autotune_strength=1, proposed_pitch=False, proposed_pitch_threshold=155.0,
                      eps_z=None, eps_src=None):
        if audio_input.shape[0] != self.block_frame:
            raise ValueError(f"block must be {self.block_frame} samples (read_chunk_size * 128)")
        o = self.group.opts(f0_up_key, index_rate, protect, volume_envelope, f0_autotune, f0_autotune_strength,
                            proposed_pitch, proposed_pitch_threshold)
        out, vol = self.group.process(np.asarray(audio_input, dtype=np.float32)[None], o, eps_z, eps_src, self.seed)
        self.seed += 1
        out0 = self.group.engine.host(out[0])
        return out0, float(vol[0].item())

    def on_request(self, audio_input: np.ndarray, f0_up_key=0, index_rate=0.5, protect=0.5, volume_envelope=1,
                   f0_autotune=False, f0_autotune_strength=1, proposed_pitch=False, proposed_pitch_threshold=155.0):
        start = time.perf_counter()
        result, vol = self.process_audio(audio_input, f0_up_key, index_rate, protect, volume_envelope, f0_autotune,
                                         f0_autotune_strength, proposed_pitch, proposed_pitch_threshold)
        end = time.perf_counter()
        return result, vol, [0, (end - start) * 1000, 0]

    def close(self):
        self.group.close()
