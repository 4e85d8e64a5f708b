"""ctypes binding of librvcx.so (the C-ABI declared in include/rvcx.h).

There is no CPU fallback: if the HIP library is missing or cannot be loaded, importing
the compute path raises ``RvcxLibraryError``.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RVCX_LIB", os.path.join(_HERE, "librvcx.so"))

RVCX_MODEL_SYNTH, RVCX_MODEL_HUBERT, RVCX_MODEL_RMVPE, RVCX_MODEL_CREPE = 0, 1, 2, 3

STATUS = {
    0: "RVCX_OK", -1: "RVCX_E_INVALID", -2: "RVCX_E_SHAPE", -3: "RVCX_E_HIP", -4: "RVCX_E_OOM",
    -5: "RVCX_E_STATE", -6: "RVCX_E_CAPACITY",
}

EXPORTS = [
    "rvcx_create", "rvcx_destroy", "rvcx_set_generator_precision", "rvcx_config_info", "rvcx_profile_read_kinds",
    "rvcx_profile_kind_name", "rvcx_synth_infer_ex", "rvcx_last_error", "rvcx_set_synth_config", "rvcx_upload", "rvcx_finalize",
    "rvcx_hubert", "rvcx_rmvpe", "rvcx_f0_post", "rvcx_synth_infer", "rvcx_dec_only", "rvcx_voice_conversion",
    "rvcx_synth_upp", "rvcx_set_highpass", "rvcx_pipeline", "rvcx_pipeline_default_opts", "rvcx_pipeline_ex",
    "rvcx_f0_autotune", "rvcx_rmvpe_decode", "rvcx_profile", "rvcx_profile_read", "rvcx_profile_read_ex", "rvcx_index_load",
    "rvcx_index_unload", "rvcx_index_info", "rvcx_index_set_nprobe", "rvcx_index_search", "rvcx_index_reconstruct_n",
    "rvcx_index_retrieve", "rvcx_rt_default_desc", "rvcx_rt_default_opts", "rvcx_rt_create", "rvcx_rt_destroy",
    "rvcx_rt_geometry", "rvcx_rt_reset", "rvcx_rt_process", "rvcx_hubert_batch", "rvcx_rmvpe_batch",
    "rvcx_pipeline_batch", "rvcx_set_highpass_sos", "rvcx_highpass_pad", "rvcx_device_status", "rvcx_index_parse",
    "rvcx_set_conv_math", "rvcx_conv1d", "rvcx_conv1d_gen", "rvcx_conv2d3x3", "rvcx_convtranspose2d_s2", "rvcx_flash_attention", "rvcx_resblock_pair", "rvcx_crepe", "rvcx_split_audio",
    "rvcx_workspace_bytes", "rvcx_set_workspace", "rvcx_workspace_info", "rvcx_crepe_ex",
    "rvcx_crepe_decode",
]


class RvcxLibraryError(ImportError):
    pass


class RvcxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code


class SynthDesc(ctypes.Structure):
    _fields_ = [
        ("inter_channels", ctypes.c_int), ("hidden_channels", ctypes.c_int), ("filter_channels", ctypes.c_int),
        ("n_heads", ctypes.c_int), ("n_layers", ctypes.c_int), ("kernel_size", ctypes.c_int),
        ("n_resblocks", ctypes.c_int), ("resblock_kernel_sizes", ctypes.c_int * 4),
        ("resblock_dilation_sizes", (ctypes.c_int * 4) * 4), ("n_dilations", ctypes.c_int),
        ("n_upsample", ctypes.c_int), ("upsample_rates", ctypes.c_int * 8),
        ("upsample_initial_channel", ctypes.c_int), ("upsample_kernel_sizes", ctypes.c_int * 8),
        ("spk_embed_dim", ctypes.c_int), ("gin_channels", ctypes.c_int), ("sr", ctypes.c_int),
        ("text_enc_hidden_dim", ctypes.c_int), ("no_f0", ctypes.c_int), ("vocoder", ctypes.c_int),
    ]


VOCODERS = {"HiFi-GAN": 0, "MRF HiFi-GAN": 1, "RefineGAN": 2}


class PipelineOpts(ctypes.Structure):
    """rvcx_pipeline_opts (include/rvcx.h)."""
    _fields_ = [
        ("sid", ctypes.c_int), ("version", ctypes.c_int), ("pitch", ctypes.c_double), ("protect", ctypes.c_float),
        ("rmvpe_threshold", ctypes.c_float), ("t_pad", ctypes.c_int64), ("t_pad_tgt", ctypes.c_int64),
        ("t_query", ctypes.c_int64), ("t_center", ctypes.c_int64), ("t_max", ctypes.c_int64),
        ("f0_autotune", ctypes.c_int), ("f0_autotune_strength", ctypes.c_double), ("proposed_pitch", ctypes.c_int),
        ("proposed_pitch_threshold", ctypes.c_double), ("volume_envelope", ctypes.c_double),
        ("mlx_semantics", ctypes.c_int), ("index_rate", ctypes.c_double), ("f0_method", ctypes.c_int),
    ]


class RtDesc(ctypes.Structure):
    """rvcx_rt_desc (include/rvcx.h)."""
    _fields_ = [("n_streams", ctypes.c_int), ("read_chunk_size", ctypes.c_int),
                ("cross_fade_overlap_size", ctypes.c_double), ("extra_convert_size", ctypes.c_double),
                ("silent_threshold", ctypes.c_double)]


class RtOpts(ctypes.Structure):
    """rvcx_rt_opts (include/rvcx.h)."""
    _fields_ = [("f0_up_key", ctypes.c_double), ("index_rate", ctypes.c_double), ("protect", ctypes.c_float),
                ("volume_envelope", ctypes.c_double), ("f0_autotune", ctypes.c_int),
                ("f0_autotune_strength", ctypes.c_double), ("proposed_pitch", ctypes.c_int),
                ("proposed_pitch_threshold", ctypes.c_double), ("gen_precision", ctypes.c_int)]


_lib: Optional[ctypes.CDLL] = None


def load(path: Optional[str] = None) -> ctypes.CDLL:
    """Load librvcx.so and declare every prototype. Raises RvcxLibraryError when absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RvcxLibraryError(f"librvcx.so not found at {p}; build it with __graft_entry__.build() "
                               "(make -C retrieval-based-voice-conversion-mlx_amd/csrc)")
    try:
        lib = ctypes.CDLL(p)
    except OSError as e:
        raise RvcxLibraryError(f"cannot load {p}: {e}") from e
    vp, i64, i32, f32, f64, u64 = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_double,
                                   ctypes.c_uint64)
    P = ctypes.POINTER
    sig = {
        "rvcx_create": (i32, [P(vp), i32]),
        "rvcx_destroy": (i32, [vp]),
        "rvcx_last_error": (ctypes.c_char_p, [vp]),
        "rvcx_set_synth_config": (i32, [vp, P(SynthDesc)]),
        "rvcx_upload": (i32, [vp, i32, ctypes.c_char_p, vp, P(i64), i32]),
        "rvcx_finalize": (i32, [vp, i32]),
        "rvcx_hubert": (i32, [vp, vp, i64, i32, vp, i64, P(i64), vp]),
        "rvcx_rmvpe": (i32, [vp, vp, i64, f32, vp, i64, P(i64), vp, vp]),
        "rvcx_f0_post": (i32, [vp, vp, i64, f64, vp, vp, vp, vp]),
        "rvcx_synth_infer": (i32, [vp, i32, i32, vp, vp, vp, vp, vp, vp, vp, u64, vp, vp, vp, vp]),
        "rvcx_synth_infer_ex": (i32, [vp, i32, i32, vp, vp, vp, vp, vp, f64, vp, vp, u64, vp, vp, vp, vp, vp, P(i32),
                                      vp]),
        "rvcx_dec_only": (i32, [vp, i32, i32, vp, vp, vp, vp, u64, vp, vp]),
        "rvcx_voice_conversion": (i32, [vp, vp, i64, vp, vp, i32, f32, f64, vp, vp, u64, vp, i64, P(i64), vp]),
        "rvcx_synth_upp": (i32, [vp]),
        "rvcx_set_highpass": (i32, [vp, vp, vp, vp, i32]),
        "rvcx_profile": (i32, [vp, i32]),
        "rvcx_profile_read": (i32, [vp, P(f64), P(f64), P(i64)]),
        "rvcx_profile_read_ex": (i32, [vp, P(f64), P(f64), P(i64), P(f64)]),
        "rvcx_pipeline": (i32, [vp, vp, i64, i32, f64, f32, i64, i64, vp, vp, u64, vp, i64, P(i64), vp, vp]),
        "rvcx_pipeline_default_opts": (i32, [P(PipelineOpts)]),
        "rvcx_pipeline_ex": (i32, [vp, vp, i64, P(PipelineOpts), vp, vp, u64, vp, i64, P(i64), vp, vp]),
        "rvcx_f0_autotune": (i32, [vp, vp, i64, f64, i32, vp]),
        "rvcx_rmvpe_decode": (i32, [vp, vp, i64, f32, vp, vp]),
        "rvcx_crepe": (i32, [vp, vp, i64, f32, f32, f32, vp, vp, vp, i64, P(i64), vp]),
        "rvcx_crepe_ex": (i32, [vp, vp, i64, f32, f32, f32, i32, vp, vp, vp, vp, i64, P(i64), vp]),
        "rvcx_crepe_decode": (i32, [vp, vp, i64, f32, f32, f32, i32, vp, vp, vp, vp]),
        "rvcx_split_audio": (i32, [vp, vp, i64, i32, f64, i32, P(i64), i64, P(i64), vp]),
        "rvcx_index_load": (i32, [vp, vp, i64]),
        "rvcx_index_unload": (i32, [vp]),
        "rvcx_index_info": (i32, [vp, P(i64), P(i64), P(i64), P(i64)]),
        "rvcx_index_set_nprobe": (i32, [vp, i64]),
        "rvcx_index_search": (i32, [vp, vp, i64, i32, vp, vp, vp]),
        "rvcx_index_reconstruct_n": (i32, [vp, i64, i64, vp, vp]),
        "rvcx_index_retrieve": (i32, [vp, vp, i64, i32, f64, vp, vp]),
        "rvcx_pipeline_batch": (i32, [vp, vp, i64, i64, i32, P(PipelineOpts), P(ctypes.c_int32), vp, vp, u64, vp, i64,
                                      P(i64), vp, vp, vp]),
        "rvcx_set_highpass_sos": (i32, [vp, vp, i32]),
        "rvcx_workspace_bytes": (i32, [vp, i32, i64, P(PipelineOpts), P(i64), vp]),
        "rvcx_set_workspace": (i32, [vp, vp, i64]),
        "rvcx_workspace_info": (i32, [vp, P(i64), P(i64), P(i64)]),
        "rvcx_highpass_pad": (i32, [vp, vp, i64, i64, vp, vp, vp]),
        "rvcx_hubert_batch": (i32, [vp, vp, i64, i64, i32, i32, vp, i64, P(i64), vp]),
        "rvcx_rmvpe_batch": (i32, [vp, vp, i64, i64, i32, f32, vp, i64, P(i64), vp, vp]),
        "rvcx_rt_default_desc": (i32, [P(RtDesc)]),
        "rvcx_rt_default_opts": (i32, [P(RtOpts)]),
        "rvcx_rt_create": (i32, [vp, P(RtDesc), P(vp)]),
        "rvcx_rt_destroy": (i32, [vp, vp]),
        "rvcx_rt_geometry": (i32, [vp, P(i64)]),
        "rvcx_rt_reset": (i32, [vp, vp, vp]),
        "rvcx_rt_process": (i32, [vp, vp, vp, P(ctypes.c_int32), P(RtOpts), vp, vp, u64, vp, vp, vp, vp]),
        "rvcx_device_status": (i32, [vp, vp]),
        "rvcx_index_parse": (i32, [vp, i64, P(i64), P(i64), P(i64), P(i64), ctypes.c_char_p, i64]),
        "rvcx_set_conv_math": (i32, [vp, i32]),
        "rvcx_set_generator_precision": (i32, [vp, i32]),
        "rvcx_config_info": (i32, [vp, vp, i64, P(i64)]),
        "rvcx_profile_read_kinds": (i32, [vp, P(f64), P(f64), P(i64), P(f64), i32, P(f64), P(f64), P(f64), P(f64),
                                          P(i64)]),
        "rvcx_profile_kind_name": (ctypes.c_char_p, [i32]),
        "rvcx_conv1d": (i32, [vp, vp, i64, i32, vp, vp, i32, i32, i32, i32, i32, i32, vp, i64, vp]),
        "rvcx_conv1d_gen": (i32, [vp, vp, i64, i32, vp, vp, i32, i32, i32, i32, i32, f32, i32, f32, vp, i32, f32, i32,
                                  vp, vp]),
        "rvcx_conv2d3x3": (i32, [vp, vp, i32, i32, i32, vp, vp, i32, i32, i32, vp, vp]),
        "rvcx_convtranspose2d_s2": (i32, [vp, vp, i32, i32, i32, vp, vp, i32, i32, i32, vp, vp]),
        "rvcx_flash_attention": (i32, [vp, vp, i32, i32, i32, i32, ctypes.c_float, vp, vp, i32, vp, vp, vp]),
        "rvcx_resblock_pair": (i32, [vp, vp, i32, i64, i32, vp, vp, vp, vp, i32, i32, i32, f32, i32, vp, vp]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(lib, name):  # reported by exported_symbols(); an older build lacks newer entry points
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def exported_symbols(path: Optional[str] = None):
    """Names of the C-ABI entry points that resolve in the library (no compute call)."""
    lib = load(path)
    return [n for n in EXPORTS if hasattr(lib, n)]


def index_parse(data: bytes) -> dict:
    """Validate a faiss IndexIVFFlat file image on the host (rvcx_index_parse; no context, no GPU).
    Returns dict(d, ntotal, nlist, nprobe); raises RvcxError for anything the loader would refuse."""
    lib = load()
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    v = [ctypes.c_int64(0) for _ in range(4)]
    err = ctypes.create_string_buffer(512)
    rc = lib.rvcx_index_parse(buf, len(data), *[ctypes.byref(x) for x in v], err, 512)
    if rc != 0:
        raise RvcxError(rc, err.value.decode(errors="replace"))
    return dict(zip(("d", "ntotal", "nlist", "nprobe"), (x.value for x in v)))
