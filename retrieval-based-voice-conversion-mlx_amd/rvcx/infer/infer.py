"""RVC_MLX-compatible front end on MI355X (rvc_mlx/infer/infer_mlx.py:106-343).

``RVCX(model_path).infer(audio_input, audio_output, pitch, f0_method, index_path, index_rate,
volume_envelope, protect, f0_autotune, f0_autotune_strength)`` loads a voice model, converts a
WAV file and writes the result at the model's sample rate. Attributes kept from the reference:
``tgt_sr``, ``net_g``, ``hubert_model``, ``rmvpe_model``, ``pipeline``.

Model files (all loaded without executing anything from the file):
  * RVC ``.pth`` (``weight``/``config``/``version``; rvc/train/process/extract_model.py:57-109) via
    torch.load(weights_only=True), weight-norm pairs fused exactly like torch.
  * MLX ``.npz`` / ``.safetensors`` written by tools/convert_rvc_model.py (remapped names, MLX
    layouts, already fused) plus an optional sibling ``.json`` config list (infer_mlx.py:146-205).
HuBERT/ContentVec and RMVPE weights come from local files only (no download: the reference's
``load_embedding``/``from_pretrained`` fetch over the network, rvc/lib/utils.py:125-153): the MLX tree's
``hubert_mlx.npz`` / ``rmvpe_mlx.npz`` (tools/convert_hubert.py, tools/convert_rmvpe.py layouts) or the
torch ``pytorch_model.bin`` / ``model.safetensors`` / ``rmvpe.pt`` (``HUBERT_CANDIDATES``, ``RMVPE_CANDIDATES``).
"""
from __future__ import annotations

import json
import os
from typing import Dict, Mapping, Optional

import numpy as np

from ..config import SynthConfig
from ..engine import Engine
from ..weights import load_rvc_checkpoint, load_state_file, normalize_state, unmap_mlx_keys
from .models import HubertModel, RMVPE0Predictor, Synthesizer
from .pipeline import Config, PipelineRVCX

# infer_mlx.py:130-176 defaults when an MLX file has no config (40 kHz v2)
_MLX_DEFAULT_40K = SynthConfig(upsample_rates=(10, 10, 2, 2), upsample_kernel_sizes=(16, 16, 4, 4), sr=40000)

# Searched relative to the working directory, the MLX tree's own files first, as RVC_MLX does
# (infer_mlx.py:258-264 for HuBERT; RMVPE0Predictor's default, rvc_mlx/lib/mlx/rmvpe.py:256-258), then the
# rvc/ torch files (rvc/lib/utils.py:125-153, RMVPE.py:429-434).
HUBERT_CANDIDATES = ("rvc_mlx/models/embedders/contentvec/hubert_mlx.npz",
                     "rvc/models/embedders/contentvec/hubert_mlx.npz",
                     "rvc/models/embedders/contentvec/pytorch_model.bin",
                     "rvc/models/embedders/contentvec/model.safetensors")
RMVPE_CANDIDATES = ("rvc_mlx/models/predictors/rmvpe_mlx.npz",
                    "rvc/models/predictors/rmvpe.pt")


def mlx_to_reference_state(weights: Mapping[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """Undo tools/convert_rvc_model.py:340-392: names back to reference keys, MLX layouts back to torch
    (Conv1d (O,K,I) -> (O,I,K); ConvTranspose1d (O,K,I) -> (I,O,K); Conv2d (O,H,W,I) -> (O,I,H,W))."""
    names = unmap_mlx_keys(weights.keys())
    out = {}
    for k, v in weights.items():
        n = names[k]
        a = np.asarray(v, dtype=np.float32)
        if a.ndim == 4:
            a = a.transpose(0, 3, 1, 2)
        elif a.ndim == 3 and "emb_rel" not in n:
            a = a.transpose(2, 0, 1) if n.startswith("dec.ups.") else a.transpose(0, 2, 1)
        out[n] = np.ascontiguousarray(a)
    return out


def load_voice_model(path: str):
    """-> (fused reference-name state, SynthConfig, version)."""
    import dataclasses

    if path.endswith(".pth"):
        state, cfg_list, meta = load_rvc_checkpoint(path)
        version = meta.get("version") or "v1"
        cfg = SynthConfig.from_list(cfg_list)
        if version == "v1":
            cfg = dataclasses.replace(cfg, text_enc_hidden_dim=256)
        cfg = dataclasses.replace(cfg, use_f0=bool(meta.get("f0", 1)),
                                  vocoder=str(meta.get("vocoder") or "HiFi-GAN"))
        return state, cfg, version
    if path.endswith(".npz") or path.endswith(".safetensors"):
        if path.endswith(".npz"):
            with np.load(path, allow_pickle=False) as z:
                raw = {k: z[k] for k in z.files}
        else:
            from safetensors.numpy import load_file

            raw = load_file(path)
        state = normalize_state(mlx_to_reference_state(raw))
        cfg = _MLX_DEFAULT_40K
        cfg_path = os.path.splitext(path)[0] + ".json"
        if os.path.exists(cfg_path):
            cfg = SynthConfig.from_json(cfg_path)
        if "emb_g.weight" in state:
            import dataclasses

            cfg = dataclasses.replace(cfg, spk_embed_dim=int(state["emb_g.weight"].shape[0]))
        emb = state.get("enc_p.emb_phone.weight")
        version = "v1" if emb is not None and emb.shape[1] == 256 else "v2"
        if version == "v1":
            import dataclasses

            cfg = dataclasses.replace(cfg, text_enc_hidden_dim=256)
        return state, cfg, version
    raise ValueError(f"unsupported voice model format: {path}")


def _first_existing(cands):
    for c in cands:
        if os.path.exists(c):
            return c
    return None


def load_audio(file_path: str, sr: int = 16000) -> np.ndarray:
    """WAV -> mono float64 @sr (infer_mlx.py:91-104; resampling by polyphase filtering)."""
    from math import gcd

    from scipy import signal
    from scipy.io import wavfile

    rate, data = wavfile.read(file_path)
    if np.issubdtype(data.dtype, np.integer):
        data = data.astype(np.float64) / float(np.iinfo(data.dtype).max + 1)
    data = np.asarray(data, dtype=np.float64)
    if data.ndim > 1:
        data = data.mean(axis=1)
    if rate != sr:
        g = gcd(int(rate), int(sr))
        data = signal.resample_poly(data, sr // g, int(rate) // g)
    return data


class RVCX:
    def __init__(self, model_path: Optional[str] = None, config=None, hubert_path: Optional[str] = None,
                 rmvpe_path: Optional[str] = None, device: int = 0, semantics: str = "rvc", *,
                 synth_state: Optional[Mapping[str, np.ndarray]] = None, synth_cfg: Optional[SynthConfig] = None,
                 hubert_state: Optional[Mapping[str, np.ndarray]] = None,
                 rmvpe_state: Optional[Mapping[str, np.ndarray]] = None, version: str = "v2"):
        self.config = config
        self.model_path = model_path
        if synth_state is None:
            if model_path is None:
                raise ValueError("model_path or synth_state is required")
            synth_state, synth_cfg, version = load_voice_model(model_path)
        if hubert_state is None:
            hp = hubert_path or _first_existing(HUBERT_CANDIDATES)
            if hp is None:
                raise FileNotFoundError("HuBERT/ContentVec weights not found; pass hubert_path (no download)")
            hubert_state = load_state_file(hp)
        if rmvpe_state is None:
            rp = rmvpe_path or _first_existing(RMVPE_CANDIDATES)
            if rp is None:
                raise FileNotFoundError("RMVPE weights not found; pass rmvpe_path (no download)")
            rmvpe_state = load_state_file(rp)
        self.version = version
        self.engine = Engine(device)
        self.engine.load_synth(synth_state, synth_cfg or SynthConfig())
        self.engine.load_hubert(hubert_state)
        self.engine.load_rmvpe(rmvpe_state)
        self.tgt_sr = self.engine.synth_cfg.sr
        self.use_f0 = bool(self.engine.synth_cfg.use_f0)  # pitch_guidance of infer.py:300
        self.net_g = Synthesizer(self.engine)
        self.hubert_model = HubertModel(self.engine, version)
        self.rmvpe_model = RMVPE0Predictor(self.engine)
        self.pipeline_config = config or Config()
        self.pipeline = PipelineRVCX(self.tgt_sr, self.pipeline_config, self.hubert_model, self.rmvpe_model,
                                     semantics=semantics)

    def convert(self, audio: np.ndarray, pitch=0, f0_method="rmvpe", index_path=None, index_rate=0.75,
                volume_envelope=1.0, protect=0.5, f0_autotune=False, f0_autotune_strength=1.0, sid=0,
                proposed_pitch=False, proposed_pitch_threshold=155.0, seed: int = 0,
                split_audio: bool = False) -> np.ndarray:
        """16 kHz mono audio -> converted float32 audio @tgt_sr (the body of infer_mlx.py:287-336). split_audio
        converts the non-silent intervals one by one and merges them back with the gaps restored
        (rvc/infer/infer.py:282-316)."""
        from ..split import merge_audio, process_audio

        chunks, intervals = process_audio(self.engine, audio, 16000) if split_audio else ([audio], None)
        outs = [self.pipeline.pipeline(self.hubert_model, self.net_g, sid, c, pitch, f0_method, index_path,
                                       index_rate, self.use_f0, volume_envelope, self.version, protect, f0_autotune,
                                       f0_autotune_strength, proposed_pitch, proposed_pitch_threshold, seed=seed)
                for c in chunks]
        return merge_audio(chunks, outs, intervals, 16000, self.tgt_sr) if split_audio else outs[0]

    def infer(self, audio_input, audio_output, pitch=0, f0_method="rmvpe", index_path=None, index_rate=0.75,
              volume_envelope=1.0, protect=0.5, f0_autotune=False, f0_autotune_strength=1.0, split_audio=False):
        from scipy.io import wavfile

        audio = load_audio(audio_input)
        out = self.convert(audio, pitch, f0_method, index_path, index_rate, volume_envelope, protect, f0_autotune,
                           f0_autotune_strength, split_audio=split_audio)
        wavfile.write(audio_output, self.tgt_sr, out.astype(np.float32))
        return out

    def close(self):
        self.engine.close()


RVC_MLX = RVCX
