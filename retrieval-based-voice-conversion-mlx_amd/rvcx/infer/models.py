"""Model handles with the duck types the reference pipeline injects.

All three share one device ``Engine`` (one rvcx context = weights + workspace in HBM):

  HubertModel        hubert_model(audio[1, N]) -> feats [1, L, 768]   (pipeline_mlx.py:172-173)
  RMVPE0Predictor    .infer_from_audio(audio, thred) -> f0 [1 + N//160] (rvc/lib/predictors/RMVPE.py:497-513,
                                                                        rvc_mlx/lib/mlx/rmvpe.py:408-412)
  Synthesizer        .infer(phone, lengths, pitch, nsff0, sid) -> (o [B, 1, T*upp], x_mask, (z, z_p, None, None))
                     .dec.upp                                          (synthesizers.py:206-243, pipeline_mlx.py:349-351)

Inputs may be numpy arrays or torch tensors; outputs are numpy at this API edge (like the MLX path).
The compute runs in librvcx.so; there is no CPU fallback.
"""
from __future__ import annotations

import os
from types import SimpleNamespace

import numpy as np

from ..engine import Engine


def _fingerprint(state) -> str:
    """Content hash of a weight dict (a reload key that cannot collide the way id() of a freed dict can)."""
    import hashlib

    h = hashlib.sha1()
    for k in sorted(state):
        a = np.ascontiguousarray(_np(state[k]), dtype=np.float32)
        h.update(k.encode())
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def _np(x):
    if hasattr(x, "detach"):
        return x.detach().cpu().numpy()
    return np.asarray(x)


class HubertModel:
    """ContentVec/HuBERT base feature extractor on device."""

    def __init__(self, engine: Engine, version: str = "v2"):
        self.engine = engine
        self.version = version

    def __call__(self, audio):
        a = _np(audio).reshape(-1)
        feats = self.engine.hubert(a, self.version)
        return self.engine.host(feats.unsqueeze(0))


class RMVPE0Predictor:
    """RMVPE pitch predictor on device."""

    def __init__(self, engine: Engine):
        self.engine = engine

    def infer_from_audio(self, audio, thred: float = 0.03):
        f0 = self.engine.rmvpe(_np(audio).reshape(-1), thred)
        return self.engine.host(f0)

    def infer_from_audio_with_hidden(self, audio, thred: float = 0.03):
        f0, hidden = self.engine.rmvpe(_np(audio).reshape(-1), thred, want_hidden=True)
        return self.engine.host(f0), self.engine.host(hidden)


class Synthesizer:
    """SynthesizerTrnMs768NSFsid (v2, 48 kHz by default) inference on device."""

    def __init__(self, engine: Engine):
        self.engine = engine
        self.dec = SimpleNamespace(upp=engine.upp)
        self.upp = engine.upp

    def infer(self, phone, phone_lengths, pitch, nsff0, sid, rate=None, eps_z=None, eps_src=None, seed: int = 0):
        """synthesizers.py:206-243: -> (o [B][1][T' upp], x_mask [B][1][T'], (z, z_p, m_p, logs_p)) with z / z_p
        [B][I][T'] and m_p / logs_p [B][I][T]; rate (a float or a one-element tensor) slices z_p, x_mask and nsff0
        [:, head:] before the flow with head = int(T (1 - rate)) and Python's slice semantics (rate > 1: a negative
        head keeps the last -head frames; T' = T without a rate)."""
        ph = _np(phone).astype(np.float32)
        B, T = ph.shape[0], ph.shape[1]
        guided = bool(self.engine.synth_cfg.use_f0)  # synthesizers.py:233-239: pitch ignored without f0
        r = None if rate is None else float(np.asarray(_np(rate)).reshape(-1)[0])
        out, zp, z, mp, lp = self.engine.synth_infer_ex(ph, _np(phone_lengths).reshape(B),
                                                        _np(pitch).reshape(B, T) if guided else None,
                                                        _np(nsff0).reshape(B, T) if guided else None,
                                                        _np(sid).reshape(B), rate=r, eps_z=eps_z, eps_src=eps_src,
                                                        seed=seed)
        head = T - zp.shape[1]
        lengths = _np(phone_lengths).reshape(B)
        x_mask = (np.arange(T)[None, :] < lengths[:, None]).astype(np.float32)[:, None, head:]
        o = self.engine.host(out)[:, None, :]
        h = self.engine.host
        return o, x_mask, (h(z.transpose(1, 2)), h(zp.transpose(1, 2)), h(mp.transpose(1, 2)), h(lp.transpose(1, 2)))


class CREPE:
    """rvc_mlx/lib/mlx/crepe.py CREPE (:224-325) on device: CREPE(model, weights_path).get_f0(audio, f0_min,
    f0_max, return_periodicity, threshold). Weights: the MLX npz (crepe_{model}.npz) or torchcrepe's .pth; the
    default location is $RVCX_CREPE_DIR/crepe_{model}.npz (the reference looks in rvc_mlx/weights, :260-268)
    and a missing file raises FileNotFoundError as the reference does (:252-256)."""

    def __init__(self, model: str = "full", weights_path=None, engine: Engine = None, state=None):
        if model not in ("full", "tiny"):
            raise ValueError(f"Model {model} is not supported. Use 'full' or 'tiny'.")
        if engine is None:
            raise TypeError("CREPE needs the rvcx Engine it runs on (engine=...)")
        self.model_type = model
        self.engine = engine
        key = ("crepe", model, weights_path) if state is None else ("crepe", model, "state", _fingerprint(state))
        if engine.loaded.get("crepe") != key:
            if state is None:
                from ..weights import load_crepe_weights
                path = weights_path or os.path.join(os.environ.get("RVCX_CREPE_DIR", "weights"), f"crepe_{model}.npz")
                if not os.path.exists(path):
                    raise FileNotFoundError(f"CREPE weights not found. Expected at: {path}")
                state = load_crepe_weights(path)
            engine.load_crepe(state, key=key)

    def get_f0(self, audio, f0_min: float = 50.0, f0_max: float = 1100.0, return_periodicity: bool = False,
               threshold: float = 0.1):
        f0, per = self.engine.crepe(_np(audio).reshape(-1).astype(np.float32), f0_min, f0_max, threshold,
                                    want_periodicity=True)
        if return_periodicity:
            return self.engine.host(f0), self.engine.host(per)
        return self.engine.host(f0)


class FCPE:
    """rvc_mlx/lib/mlx/fcpe.py FCPE (:50-163): the reference's MLX FCPE is a stub that runs RMVPE with threshold x 5
    (:129-132); this keeps exactly that behaviour on the device RMVPE."""

    def __init__(self, engine: Engine):
        self.engine = engine

    def get_f0(self, audio, f0_min: float = 50.0, f0_max: float = 1100.0, threshold: float = 0.006, **kw):
        return self.engine.host(self.engine.rmvpe(_np(audio).reshape(-1).astype(np.float32), threshold * 5))


class PitchExtractor:
    """rvc_mlx/lib/mlx/pitch_extractors.py PitchExtractor (:19-216) for the methods this path runs on device:
    rmvpe, crepe, crepe-tiny, fcpe (the pyworld methods dio/pm/harvest are CPU algorithms outside this path)."""

    METHODS = ["rmvpe", "crepe", "crepe-tiny", "fcpe"]

    def __init__(self, method: str = "rmvpe", sample_rate: int = 16000, hop_size: int = 160, engine: Engine = None,
                 crepe_weights=None):
        if method not in self.METHODS:
            raise ValueError(f"Unknown method: {method}")
        self.method, self.sample_rate, self.hop_size, self.engine = method, sample_rate, hop_size, engine
        if method in ("crepe", "crepe-tiny"):
            self._model = CREPE("tiny" if method == "crepe-tiny" else "full", crepe_weights, engine=engine)
        elif method == "fcpe":
            self._model = FCPE(engine)
        else:
            self._model = RMVPE0Predictor(engine)

    def extract(self, audio, f0_min: float = 50.0, f0_max: float = 1100.0, **kwargs):
        audio = _np(audio)
        if audio.ndim > 1:
            audio = audio.mean(axis=-1)
        if self.method == "rmvpe":
            return self._model.infer_from_audio(audio, thred=kwargs.get("threshold", 0.03))
        if self.method == "fcpe":
            return self._model.get_f0(audio, f0_min=f0_min, f0_max=f0_max, threshold=kwargs.get("threshold", 0.006))
        return self._model.get_f0(audio, f0_min=f0_min, f0_max=f0_max, **kwargs)
