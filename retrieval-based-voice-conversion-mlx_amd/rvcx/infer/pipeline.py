"""PipelineMLX-compatible conversion pipeline on MI355X.

Mirrors the plugin surface of rvc_mlx/infer/pipeline_mlx.py (PipelineMLX, :84-373) and the
semantics of its PyTorch oracle rvc/infer/pipeline.py (Pipeline, :165-558): same constructor,
same ``pipeline`` / ``get_f0`` / ``voice_conversion`` signatures, numpy in and out. The work
runs in librvcx.so on the GPU (see include/rvcx.h); this module only converts arguments.

Semantics: ``semantics="rvc"`` (default) follows rvc/infer/pipeline.py -- t_pad = x_pad * 16000,
autotune replaces the pitch shift, long inputs are split at quiet points (x_query/x_center/x_max).
``semantics="mlx"`` applies the two documented deltas of the MLX port that are pure pipeline
policy: t_pad forced to 1600 samples (pipeline_mlx.py:318) and the MLX get_f0 order (autotune
skips f0 <= 0, then the shift is applied; pipeline_mlx.py:142-147). Differences the reference
marks as port bugs (zeroed flow noise, no opt_ts split) are not reproduced.

Errors raise (the reference prints and continues, pipeline_mlx.py:280-281).
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np

from .models import CREPE, HubertModel, RMVPE0Predictor, Synthesizer, _np


class Config:
    """rvc_mlx/configs/config.py:7-20 (x_pad, x_query, x_center, x_max in seconds)."""

    def __init__(self, x_pad=1, x_query=6, x_center=38, x_max=41):
        self.device = "rocm"
        self.gpu_name = "AMD Instinct MI355X"
        self.x_pad, self.x_query, self.x_center, self.x_max = x_pad, x_query, x_center, x_max
        self.is_half = False

    def device_config(self):
        return self.x_pad, self.x_query, self.x_center, self.x_max


class PipelineRVCX:
    # pipeline_mlx.py:82 / pitch_extractors.py:44 minus the pyworld CPU methods (dio, pm, harvest). "crepe" and
    # "crepe-tiny" run CREPE as each side defines it: semantics="mlx" as rvc_mlx/lib/mlx/crepe.py (reflect padding,
    # biased std, weighted-argmax decode), semantics="rvc" as rvc/lib/predictors/f0.py:31-55 (torchcrepe.predict:
    # zero padding, unbiased std, viterbi decode; its triangular dither of the decoded cents only with
    # crepe_dither=True in get_f0, as it is random; pipeline() decodes without it). "fcpe" is the MLX stub's RMVPE with threshold 0.006 x 5
    # (rvc_mlx/lib/mlx/fcpe.py:129-132) and needs semantics="mlx" (rvc/'s torchfcpe model is not available).
    SUPPORTED_F0_METHODS = ("rmvpe", "crepe", "crepe-tiny", "fcpe")

    def __init__(self, tgt_sr, config, hubert_model: Optional[HubertModel] = None,
                 rmvpe_model: Optional[RMVPE0Predictor] = None, f0_method: str = "rmvpe", semantics: str = "rvc",
                 crepe_weights=None, crepe_dither: bool = False):
        if semantics not in ("rvc", "mlx"):
            raise ValueError("semantics must be 'rvc' or 'mlx'")
        self.x_pad, self.x_query, self.x_center, self.x_max = config.x_pad, config.x_query, config.x_center, \
            config.x_max
        self.sample_rate = 16000
        self.tgt_sr = int(tgt_sr)
        self.window = 160
        self.t_pad = int(self.sample_rate * self.x_pad)
        self.t_pad_tgt = int(self.tgt_sr * self.x_pad)
        self.t_pad2 = self.t_pad * 2
        self.t_query = int(self.sample_rate * self.x_query)
        self.t_center = int(self.sample_rate * self.x_center)
        self.t_max = int(self.sample_rate * self.x_max)
        self.time_step = self.window / self.sample_rate * 1000
        self.f0_min, self.f0_max = 50, 1100
        self.f0_mel_min = 1127 * np.log(1 + self.f0_min / 700)
        self.f0_mel_max = 1127 * np.log(1 + self.f0_max / 700)
        self.hubert_model = hubert_model
        self.rmvpe_model = rmvpe_model
        self.semantics = semantics
        self.crepe_dither = bool(crepe_dither)
        # {"full": path-or-state, "tiny": ...} (or one path for "full"); None = $RVCX_CREPE_DIR/crepe_{model}.npz
        self.crepe_weights = crepe_weights if isinstance(crepe_weights, dict) or crepe_weights is None \
            else {"full": crepe_weights}
        self._check_method(f0_method)
        self._f0_method = f0_method
        self.engine = (hubert_model or rmvpe_model).engine if (hubert_model or rmvpe_model) else None
        self.last_f0 = None

    # ------------------------------------------------------------------ helpers
    def _check_method(self, m):
        if m not in self.SUPPORTED_F0_METHODS:
            raise ValueError(f"f0_method {m!r} is not supported on this path (supported: {self.SUPPORTED_F0_METHODS})")
        if m == "fcpe" and self.semantics != "mlx":
            raise ValueError("f0_method 'fcpe' needs torchfcpe's model on the rvc/ path (rvc/lib/predictors/f0.py:60-89); "
                             "semantics='mlx' runs the MLX port's FCPE (its RMVPE fallback)")

    def _crepe(self, eng, f0_method):
        """Load the CREPE weights f0_method names into the engine (once per model kind)."""
        kind = "tiny" if f0_method == "crepe-tiny" else "full"
        src = (self.crepe_weights or {}).get(kind)
        if isinstance(src, dict):
            return CREPE(kind, None, engine=eng, state=src)
        return CREPE(kind, src, engine=eng)

    def _f0_opts(self, eng, f0_method):
        """(f0_method, rmvpe_threshold) of rvcx_pipeline_opts for an f0 method name."""
        if f0_method in ("crepe", "crepe-tiny"):
            self._crepe(eng, f0_method)
            return (1 if self.semantics == "mlx" else 2), 0.03
        if f0_method == "fcpe":
            return 0, 0.006 * 5
        return 0, 0.03

    @staticmethod
    def _check_guidance(eng, pitch_guidance: bool):
        """pitch_guidance must match the loaded model (infer.py:300 passes cpt["f0"]): the reference fails on a
        mismatch (pitchf.float() on None, pipeline.py:370; dec(z, None) for an NSF decoder); here it raises."""
        model_f0 = bool(eng.synth_cfg.use_f0)
        if pitch_guidance != model_f0:
            raise ValueError(f"pitch_guidance={pitch_guidance} but the loaded model has f0={int(model_f0)}")

    def _engine(self, *models):
        for mdl in models + (self.hubert_model, self.rmvpe_model):
            if mdl is not None and getattr(mdl, "engine", None) is not None:
                return mdl.engine
        if self.engine is None:
            raise RuntimeError("no rvcx Engine: pass models created by rvcx.infer (HubertModel/RMVPE0Predictor)")
        return self.engine

    def _ensure_highpass(self, eng):
        if getattr(eng, "_hp", None) is None:
            eng.set_pipeline_highpass(self.sample_rate)  # pipeline.py:22-27

    def load_index(self, file_index: str, eng=None):
        """faiss.read_index + reconstruct_n (pipeline.py:430-434), cached per (path, mtime, size)."""
        from .index import IndexIVFFlat

        eng = eng or self._engine()
        st = os.stat(file_index)
        key = (os.path.abspath(file_index), st.st_mtime_ns, st.st_size, id(eng))
        if getattr(self, "_index_key", None) != key or eng.index_info() is None:
            self.index = IndexIVFFlat(eng, path=file_index)
            self._index_key = key
        return self.index

    # ------------------------------------------------------------------ API (pipeline_mlx.py:135-373)
    def get_f0(self, x, p_len, f0_method="rmvpe", pitch=0, f0_autotune=False, f0_autotune_strength=1.0,
               proposed_pitch=False, proposed_pitch_threshold=155.0):
        """-> (f0_coarse int64 [F], f0 float64 [F]) with F = 1 + len(x)//160 (pipeline.py:200-291)."""
        self._check_method(f0_method)
        eng = self._engine()
        method, thr = self._f0_opts(eng, f0_method)
        xa = np.asarray(x, dtype=np.float32).reshape(-1)
        if method == 1:  # PitchExtractor.extract -> CREPE.get_f0(x, f0_min=50, f0_max=1100) (pipeline_mlx.py:140)
            f0 = eng.crepe(xa, self.f0_min, self.f0_max, 0.1).double()
        elif method == 2:  # CREPE(...).get_f0(x, self.f0_min, self.f0_max, p_len, model) (pipeline.py:223-234)
            dither = None
            if self.crepe_dither:  # torchcrepe.convert.dither: scipy.stats.triang(c=0.5, loc=-20, scale=40)
                dither = np.random.default_rng().triangular(-20.0, 0.0, 20.0, size=1 + len(xa) // 160)
            f0 = eng.crepe(xa, self.f0_min, self.f0_max, 0.1, semantics="rvc", dither=dither).double()
        else:
            f0 = eng.rmvpe(xa, thr)
        shift = float(pitch)
        if f0_autotune:
            f0 = eng.f0_autotune(f0, f0_autotune_strength, skip_unvoiced=self.semantics == "mlx")
            if self.semantics == "rvc":
                shift = 0.0
        elif proposed_pitch and self.semantics == "rvc":
            shift += proposed_key(eng.host(f0), proposed_pitch_threshold)
        coarse, _, fs = eng.f0_post(f0, shift)
        return eng.host(coarse).astype(np.int64), eng.host(fs)

    def voice_conversion(self, model, net_g, sid, audio0, pitch, pitchf, index=None, big_npy=None, index_rate=0.0,
                         version="v2", protect=0.33, eps_z=None, eps_src=None, seed: int = 0):
        """One padded chunk: HuBERT -> x2 -> protect -> Synthesizer.infer. -> float32 [p_len * upp].
        pitch / pitchf None = pitch_guidance False (pipeline.py:324): no protect, the model's f0-less decoder."""
        eng = self._engine(model)
        self._check_guidance(eng, pitch is not None and pitchf is not None)
        rate = 0.0
        if index is not None and index_rate > 0:  # pipeline.py:338-342 (big_npy is the index's own rows)
            if getattr(index, "engine", None) is not eng:
                raise TypeError("index must be an rvcx IndexIVFFlat loaded on this pipeline's engine (read_index)")
            index._bound()
            rate = float(index_rate)
        out = eng.voice_conversion(np.asarray(audio0, dtype=np.float32).reshape(-1),
                                   None if pitch is None else _np(pitch).reshape(-1),
                                   None if pitchf is None else _np(pitchf).reshape(-1), int(_np(sid).reshape(-1)[0]),
                                   float(protect),
                                   eps_z=eps_z, eps_src=eps_src, seed=seed, index_rate=rate)
        return eng.host(out)

    def pipeline(self, model, net_g, sid, audio, pitch=0, f0_method="rmvpe", file_index=None, index_rate=0.0,
                 pitch_guidance=True, volume_envelope=1.0, version="v2", protect=0.33, f0_autotune=False,
                 f0_autotune_strength=1.0, proposed_pitch=False, proposed_pitch_threshold=155.0, eps_z=None,
                 eps_src=None, seed: int = 0):
        """Whole utterance -> float32 [N_out] @tgt_sr (pipeline.py:390-558)."""
        self._check_method(f0_method)
        eng = self._engine(model)
        self._check_guidance(eng, bool(pitch_guidance))
        # pipeline.py:430-436: the index is used only when the file exists and index_rate > 0 (a missing
        # file means no retrieval, as in the reference); a file that does not parse raises here.
        rate = 0.0
        if file_index and os.path.exists(file_index) and index_rate > 0:
            self.load_index(file_index, eng)
            rate = float(index_rate)
        self._ensure_highpass(eng)
        method, thr = self._f0_opts(eng, f0_method)
        mlx = self.semantics == "mlx"
        t_pad = 1600 if mlx else self.t_pad
        t_pad_tgt = int(t_pad * self.tgt_sr / self.sample_rate) if mlx else self.t_pad_tgt
        opts = eng.pipeline_opts(
            sid=int(_np(sid).reshape(-1)[0]), version={"v1": 1, "v2": 2}.get(version, 0), pitch=float(pitch),
            protect=float(protect), t_pad=t_pad, t_pad_tgt=t_pad_tgt, t_query=self.t_query,
            t_center=self.t_center, t_max=0 if mlx else self.t_max, f0_autotune=int(bool(f0_autotune)),
            f0_autotune_strength=float(f0_autotune_strength),
            proposed_pitch=int(bool(proposed_pitch) and not mlx),
            proposed_pitch_threshold=float(proposed_pitch_threshold), volume_envelope=float(volume_envelope),
            mlx_semantics=int(mlx), index_rate=rate, f0_method=method, rmvpe_threshold=thr)
        y, f0 = eng.pipeline_ex(np.asarray(audio, dtype=np.float64).reshape(-1), opts, eps_z=eps_z,
                                eps_src=eps_src, seed=seed, want_f0=True)
        self.last_f0 = f0
        return eng.host(y)


PipelineMLX = PipelineRVCX


def proposed_key(f0: np.ndarray, threshold: float, limit: int = 12) -> int:
    """Key offset of proposed_pitch (rvc/infer/pipeline.py:250-277)."""
    valid = np.where(f0 > 0)[0]
    if len(valid) < 2:
        return 0
    med = float(np.median(np.interp(np.arange(len(f0)), valid, f0[valid])))
    if med <= 0 or np.isnan(med):
        return 0
    return max(-limit, min(limit, int(np.round(12 * np.log2(threshold / med)))))
