"""Host-side logic of the drop-in API (no GPU): weight ingestion formats, MLX layout inversion,
proposed-pitch key, audio loading, and the rvcx_pipeline_opts struct layout shared with C."""
import os

import numpy as np
import pytest
import torch


def _mlx_forward(state):
    """Forward layout conversion of tools/convert_rvc_model.py:340-392 restated for the round trip:
    Conv2d (O,I,H,W)->(O,H,W,I); ConvTranspose1d (I,O,K)->(O,K,I); Conv1d (O,I,K)->(O,K,I)."""
    import re

    rules = [
        (r"^dec\.resblocks\.(\d+)\.convs([12])\.(\d+)\.(.*)$", r"dec.resblock_\1.c\2_\3.\4"),
        (r"^dec\.ups\.(\d+)\.(.*)$", r"dec.up_\1.\2"),
        (r"^dec\.noise_convs\.(\d+)\.(.*)$", r"dec.noise_conv_\1.\2"),
        (r"^enc_p\.encoder\.attn_layers\.(\d+)\.(.*)$", r"enc_p.encoder.attn_\1.\2"),
        (r"^enc_p\.encoder\.norm_layers_1\.(\d+)\.(.*)$", r"enc_p.encoder.norm1_\1.\2"),
        (r"^enc_p\.encoder\.norm_layers_2\.(\d+)\.(.*)$", r"enc_p.encoder.norm2_\1.\2"),
        (r"^enc_p\.encoder\.ffn_layers\.(\d+)\.(.*)$", r"enc_p.encoder.ffn_\1.\2"),
        (r"^flow\.flows\.(\d+)\.enc\.in_layers\.(\d+)\.(.*)$", r"flow.flow_\1.enc.in_layer_\2.\3"),
        (r"^flow\.flows\.(\d+)\.enc\.res_skip_layers\.(\d+)\.(.*)$", r"flow.flow_\1.enc.res_skip_layer_\2.\3"),
        (r"^flow\.flows\.(\d+)\.(.*)$", r"flow.flow_\1.\2"),
    ]
    out = {}
    for k, v in state.items():
        n = k
        for pat, rep in rules:
            if re.match(pat, n):
                n = re.sub(pat, rep, n)
                break
        n = n.replace(".gamma", ".weight").replace(".beta", ".bias")
        if v.ndim == 4:
            v = v.transpose(0, 2, 3, 1)
        elif v.ndim == 3 and "emb_rel" not in k:
            v = v.transpose(1, 2, 0) if k.startswith("dec.ups.") else v.transpose(0, 2, 1)
        out[n] = np.ascontiguousarray(v)
    return out


def test_mlx_state_round_trip(synth_w):
    from rvcx.infer.infer import mlx_to_reference_state

    back = mlx_to_reference_state(_mlx_forward(synth_w))
    assert set(back) == set(synth_w)
    for k, v in synth_w.items():
        assert back[k].shape == v.shape, k
        assert np.array_equal(back[k], v), k


def test_load_rvc_pth_and_npz(tmp_path, synth_w):
    from rvcx import synthetic
    from rvcx.config import SYNTH_48K_V2
    from rvcx.infer.infer import load_voice_model

    raw = synthetic.synth_state(2)
    cpt = {"weight": {k: torch.from_numpy(np.asarray(v)).half() for k, v in raw.items()},
           "config": SYNTH_48K_V2.as_list(), "version": "v2", "f0": 1, "sr": "48k"}
    p = tmp_path / "voice.pth"
    torch.save(cpt, p)
    st, cfg, ver = load_voice_model(str(p))
    assert ver == "v2" and cfg.upsample_rates == SYNTH_48K_V2.upsample_rates and cfg.sr == 48000
    assert set(st) == set(synth_w)
    for k in ("dec.ups.0.weight", "enc_p.emb_phone.weight", "flow.flows.0.enc.in_layers.0.weight"):
        ref = synth_w[k]
        assert np.abs(st[k] - ref).max() <= 2e-3 * np.abs(ref).max() + 1e-3, k  # fp16 storage
    q = tmp_path / "voice.npz"
    np.savez(q, **_mlx_forward(synth_w))
    with open(tmp_path / "voice.json", "w") as f:
        import json

        json.dump(SYNTH_48K_V2.as_list(), f)
    st2, cfg2, ver2 = load_voice_model(str(q))
    assert ver2 == "v2" and cfg2.sr == 48000
    assert all(np.array_equal(st2[k], synth_w[k]) for k in synth_w)


def test_proposed_key_matches_oracle():
    from oracle.pipeline import post_f0
    from rvcx.infer.pipeline import proposed_key

    rng = np.random.default_rng(0)
    for thr in (155.0, 220.0, 90.0):
        f0 = np.where(rng.random(400) < 0.3, 0.0, rng.uniform(80, 400, 400))
        key = proposed_key(f0, thr)
        _, shifted = post_f0(f0.copy(), 1, proposed_pitch=True, proposed_pitch_threshold=thr)
        v = f0 > 0
        ratio = np.median(shifted[v] / f0[v])
        assert abs(ratio - 2 ** ((1 + key) / 12)) < 1e-12
    assert proposed_key(np.zeros(10), 155.0) == 0


def test_load_audio_resamples(tmp_path):
    from scipy.io import wavfile

    from rvcx.infer.infer import load_audio

    t = np.arange(44100) / 44100.0
    x = (0.5 * np.sin(2 * np.pi * 440 * t) * 32767).astype(np.int16)
    wavfile.write(tmp_path / "a.wav", 44100, np.stack([x, x], 1))
    y = load_audio(str(tmp_path / "a.wav"))
    assert y.dtype == np.float64 and y.shape == (16000,)
    assert abs(np.abs(y[1000:-1000]).max() - 0.5) < 0.01


def test_pipeline_opts_layout_and_defaults():
    """The ctypes mirror of rvcx_pipeline_opts must match the C struct: the library fills it."""
    import ctypes

    from rvcx import _lib

    lib = _lib.load()
    o = _lib.PipelineOpts()
    assert lib.rvcx_pipeline_default_opts(ctypes.byref(o)) == 0
    assert (o.t_pad, o.t_pad_tgt, o.t_query, o.t_center, o.t_max) == (16000, 48000, 96000, 608000, 656000)
    assert abs(o.protect - 0.33) < 1e-7 and abs(o.rmvpe_threshold - 0.03) < 1e-7
    assert o.f0_autotune_strength == 1.0 and o.proposed_pitch_threshold == 155.0 and o.volume_envelope == 1.0
    assert o.sid == 0 and o.version == 0 and o.mlx_semantics == 0


def test_api_names_exist():
    import rvcx.infer as ri

    for name in ("RVC_MLX", "PipelineMLX", "Config", "HubertModel", "RMVPE0Predictor", "Synthesizer"):
        assert hasattr(ri, name)
    assert ri.PipelineMLX.SUPPORTED_F0_METHODS == ("rmvpe", "crepe", "crepe-tiny", "fcpe")
    for m in ("pipeline", "get_f0", "voice_conversion"):
        assert callable(getattr(ri.PipelineMLX, m))
