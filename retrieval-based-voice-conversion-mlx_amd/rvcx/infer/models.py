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

from types import SimpleNamespace

import numpy as np

from ..engine import Engine


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
        return feats.unsqueeze(0).cpu().numpy()


class RMVPE0Predictor:
    """RMVPE pitch predictor on device."""

    def __init__(self, engine: Engine):
        self.engine = engine

    def infer_from_audio(self, audio, thred: float = 0.03):
        f0 = self.engine.rmvpe(_np(audio).reshape(-1), thred)
        return f0.cpu().numpy()

    def infer_from_audio_with_hidden(self, audio, thred: float = 0.03):
        f0, hidden = self.engine.rmvpe(_np(audio).reshape(-1), thred, want_hidden=True)
        return f0.cpu().numpy(), hidden.cpu().numpy()


class Synthesizer:
    """SynthesizerTrnMs768NSFsid (v2, 48 kHz by default) inference on device."""

    def __init__(self, engine: Engine):
        self.engine = engine
        self.dec = SimpleNamespace(upp=engine.upp)
        self.upp = engine.upp

    def infer(self, phone, phone_lengths, pitch, nsff0, sid, rate=None, eps_z=None, eps_src=None, seed: int = 0):
        if rate is not None:
            raise NotImplementedError("Synthesizer.infer(rate=...) (partial re-synthesis) is not supported")
        ph = _np(phone).astype(np.float32)
        B, T = ph.shape[0], ph.shape[1]
        guided = bool(self.engine.synth_cfg.use_f0)  # synthesizers.py:233-239: pitch ignored without f0
        out, zp, z = self.engine.synth_infer(ph, _np(phone_lengths).reshape(B),
                                             _np(pitch).reshape(B, T) if guided else None,
                                             _np(nsff0).reshape(B, T) if guided else None,
                                             _np(sid).reshape(B), eps_z=eps_z,
                                             eps_src=eps_src, seed=seed, want_latents=True)
        lengths = _np(phone_lengths).reshape(B)
        x_mask = (np.arange(T)[None, :] < lengths[:, None]).astype(np.float32)[:, None, :]
        o = out.cpu().numpy()[:, None, :]
        return o, x_mask, (z.transpose(1, 2).cpu().numpy(), zp.transpose(1, 2).cpu().numpy(), None, None)
