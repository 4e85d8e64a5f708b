"""Weight ingestion end to end: model files on disk in the reference's own formats, loaded
through ``RVC_MLX(...)`` with the non-executing loaders and run through the device pipeline.

Files written here (seeded synthetic weights of the real architectures):
  * an RVC ``.pth`` exactly as rvc/train/process/extract_model.py:57-109 writes it: ``weight`` (fp16 tensors,
    ``enc_q`` dropped, weight-norm as ``*.weight_g`` / ``*.weight_v``), the 18-element ``config`` list, ``f0``,
    ``version``, ``sr`` and the bookkeeping keys;
  * a ContentVec HF state dict ``pytorch_model.bin`` (HF names, positional-conv weight norm over dim 2,
    ``final_proj``; the file rvc/lib/utils.py:125-153 would fetch);
  * an ``rmvpe.pt`` state dict (BatchNorm buffers included; RMVPE.py:429-434);
  * the MLX pair ``model.npz`` + ``model.json`` as tools/convert_rvc_model.py:250-392 writes it (remapped names,
    MLX layouts: Conv1d (O,K,I), ConvTranspose1d (O,K,I), LayerNorm weight/bias), read by infer_mlx.py:130-244.
Checks: the .pth-loaded context equals a context fed the same tensors from memory (bit-identical output), the
MLX-loaded context equals the .pth-loaded one, and the .pth-loaded context matches the CPU oracle on the
fp16-rounded fused weights (spectrogram correlation >= 0.999, rel <= 2e-3, the pipeline test's bar).
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def _ref_to_mlx_name(k: str) -> str:
    """Reference state-dict name -> the MLX converter's name (the forward of infer_mlx.py:17-89 remap_keys)."""
    p = k.split(".")
    if k.startswith("dec.resblocks."):
        k = f"dec.resblock_{p[2]}.{'c1' if p[3] == 'convs1' else 'c2'}_{p[4]}.{'.'.join(p[5:])}"
    elif k.startswith("dec.ups."):
        k = f"dec.up_{p[2]}.{'.'.join(p[3:])}"
    elif k.startswith("dec.noise_convs."):
        k = f"dec.noise_conv_{p[2]}.{'.'.join(p[3:])}"
    elif k.startswith("enc_p.encoder.attn_layers."):
        k = f"enc_p.encoder.attn_{p[3]}.{'.'.join(p[4:])}"
    elif k.startswith("enc_p.encoder.norm_layers_1."):
        k = f"enc_p.encoder.norm1_{p[3]}.{'.'.join(p[4:])}"
    elif k.startswith("enc_p.encoder.norm_layers_2."):
        k = f"enc_p.encoder.norm2_{p[3]}.{'.'.join(p[4:])}"
    elif k.startswith("enc_p.encoder.ffn_layers."):
        k = f"enc_p.encoder.ffn_{p[3]}.{'.'.join(p[4:])}"
    elif k.startswith("flow.flows."):
        if "in_layers" in k:
            k = f"flow.flow_{p[2]}.enc.in_layer_{p[5]}.{'.'.join(p[6:])}"
        elif "res_skip_layers" in k:
            k = f"flow.flow_{p[2]}.enc.res_skip_layer_{p[5]}.{'.'.join(p[6:])}"
        else:
            k = f"flow.flow_{p[2]}.{'.'.join(p[3:])}"
    if k.endswith(".gamma"):
        k = k[: -len(".gamma")] + ".weight"
    elif k.endswith(".beta"):
        k = k[: -len(".beta")] + ".bias"
    return k


def _ref_to_mlx_layout(name: str, a: np.ndarray) -> np.ndarray:
    if a.ndim == 3 and "emb_rel" not in name:
        return a.transpose(1, 2, 0) if name.startswith("dec.ups.") else a.transpose(0, 2, 1)
    return a


@pytest.fixture(scope="module")
def model_files(tmp_path_factory):
    from rvcx import synthetic
    from rvcx.config import SYNTH_48K_V2

    d = tmp_path_factory.mktemp("models")
    c = SYNTH_48K_V2
    cfg_list = [c.spec_channels, c.segment_size, c.inter_channels, c.hidden_channels, c.filter_channels, c.n_heads,
                c.n_layers, c.kernel_size, c.p_dropout, c.resblock, list(c.resblock_kernel_sizes),
                [list(x) for x in c.resblock_dilation_sizes], list(c.upsample_rates), c.upsample_initial_channel,
                list(c.upsample_kernel_sizes), c.spk_embed_dim, c.gin_channels, c.sr]
    raw = synthetic.synth_state(2)
    pth = {"weight": {k: torch.from_numpy(np.ascontiguousarray(v)).half() for k, v in raw.items()},
           "config": cfg_list, "epoch": 1, "step": 1, "sr": "48k", "f0": 1, "version": "v2",
           "creation_date": "2026-01-01T00:00:00", "model_hash": "0" * 64, "overtrain_info": "None",
           "dataset_length": 0, "model_name": "synthetic", "author": "tests", "embedder_model": "contentvec",
           "speakers_id": 0, "vocoder": "HiFi-GAN"}
    torch.save(pth, d / "voice.pth")
    torch.save({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in synthetic.hubert_state(4).items()},
               d / "pytorch_model.bin")
    torch.save({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in synthetic.rmvpe_state(5).items()},
               d / "rmvpe.pt")
    # what the .pth carries, as the oracle and the in-memory context see it: fp16-rounded, then fused
    from rvcx.weights import normalize_state

    raw16 = {k: v.astype(np.float16).astype(np.float32) for k, v in raw.items()}
    fused16 = normalize_state(raw16)
    mlx = {_ref_to_mlx_name(k): _ref_to_mlx_layout(k, v) for k, v in fused16.items()}
    np.savez(d / "voice_mlx.npz", **mlx)
    with open(d / "voice_mlx.json", "w") as f:
        json.dump(cfg_list, f)
    return {"dir": str(d), "fused16": fused16}


def _run(engine, g):
    engine.set_pipeline_highpass()
    return engine.pipeline(g["audio"], sid=0, semitones=0, protect=0.33, t_pad=16000, t_pad_tgt=48000,
                           eps_z=g["eps_z"], eps_src=g["eps_src"]).cpu().numpy()


def test_rvc_pth_contentvec_rmvpe_files_end_to_end(model_files, hubert_w, rmvpe_w):
    from oracle.metrics import spectrogram_correlation
    from oracle.pipeline import OraclePipeline
    from rvcx.config import HUBERT_BASE, RMVPE_CFG, SYNTH_48K_V2
    from rvcx.engine import Engine
    from rvcx.infer import RVC_MLX

    d = model_files["dir"]
    g = golden("pipeline_2p5s.npz")
    rvc = RVC_MLX(os.path.join(d, "voice.pth"), hubert_path=os.path.join(d, "pytorch_model.bin"),
                  rmvpe_path=os.path.join(d, "rmvpe.pt"))
    try:
        assert rvc.tgt_sr == 48000 and rvc.version == "v2"
        out_file = _run(rvc.engine, g)
        rvc.engine.check_device_status()
    finally:
        rvc.close()
    mem = Engine(0)
    try:
        mem.load_synth(model_files["fused16"], SYNTH_48K_V2)
        mem.load_hubert(hubert_w)
        mem.load_rmvpe(rmvpe_w)
        out_mem = _run(mem, g)
    finally:
        mem.close()
    assert np.array_equal(out_file, out_mem), "file-loaded weights differ from the same tensors uploaded from memory"

    noise = {"z": torch.from_numpy(g["eps_z"]).float(), "src": torch.from_numpy(g["eps_src"]).float()}
    orc = OraclePipeline(48000, synth_w=model_files["fused16"], synth_cfg=SYNTH_48K_V2, hubert_w=hubert_w,
                         hubert_cfg=HUBERT_BASE, rmvpe_w=rmvpe_w, rmvpe_cfg=RMVPE_CFG,
                         noise_fn=lambda shape, which: noise[which].reshape(shape))
    ref = orc.pipeline(0, g["audio"].astype(np.float64).copy(), protect=0.33)
    assert out_file.shape == ref.shape
    corr = spectrogram_correlation(out_file, ref)
    rel = float(np.abs(out_file - ref).max() / np.abs(ref).max())
    assert corr >= 0.999 and rel <= 2e-3, (corr, rel)


def test_mlx_npz_model_matches_pth(model_files, hubert_w, rmvpe_w):
    from rvcx.infer import RVC_MLX

    d = model_files["dir"]
    g = golden("pipeline_2p5s.npz")
    outs = []
    for name in ("voice.pth", "voice_mlx.npz"):
        rvc = RVC_MLX(os.path.join(d, name), hubert_state=hubert_w, rmvpe_state=rmvpe_w)
        try:
            assert rvc.tgt_sr == 48000 and rvc.version == "v2"
            outs.append(_run(rvc.engine, g))
        finally:
            rvc.close()
    assert np.array_equal(outs[0], outs[1])


def test_mlx_tree_hubert_rmvpe_files(model_files, monkeypatch):
    """RVC_MLX(voice_mlx.npz) with the MLX tree's own hubert_mlx.npz / rmvpe_mlx.npz found where
    the reference looks for them (infer_mlx.py:258-264, rvc_mlx/lib/mlx/rmvpe.py:256-258), written by the numpy
    restatement of tools/convert_hubert.py / tools/convert_rmvpe.py (tests/mlx_convert.py). The pipeline output
    must be bit-identical to the same voice with the torch ContentVec .bin and rmvpe.pt."""
    from mlx_convert import hubert_to_mlx, rmvpe_to_mlx
    from rvcx import synthetic
    from rvcx.infer import RVC_MLX

    d = model_files["dir"]
    root = os.path.join(d, "mlx_tree")
    os.makedirs(os.path.join(root, "rvc_mlx/models/embedders/contentvec"), exist_ok=True)
    os.makedirs(os.path.join(root, "rvc_mlx/models/predictors"), exist_ok=True)
    np.savez(os.path.join(root, "rvc_mlx/models/embedders/contentvec/hubert_mlx.npz"),
             **hubert_to_mlx(synthetic.hubert_state(4)))
    np.savez(os.path.join(root, "rvc_mlx/models/predictors/rmvpe_mlx.npz"), **rmvpe_to_mlx(synthetic.rmvpe_state(5)))
    g = golden("pipeline_2p5s.npz")
    voice = os.path.join(d, "voice_mlx.npz")
    ref = RVC_MLX(voice, hubert_path=os.path.join(d, "pytorch_model.bin"), rmvpe_path=os.path.join(d, "rmvpe.pt"))
    try:
        out_torch = _run(ref.engine, g)
    finally:
        ref.close()
    monkeypatch.chdir(root)
    rvc = RVC_MLX(voice)
    try:
        out_mlx = _run(rvc.engine, g)
        rvc.engine.check_device_status()
    finally:
        rvc.close()
    assert np.array_equal(out_mlx, out_torch), "MLX-tree HuBERT/RMVPE files differ from the torch files"
