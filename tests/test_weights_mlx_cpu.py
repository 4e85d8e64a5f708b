"""The MLX tree's HuBERT / RMVPE weight files (hubert_mlx.npz, rmvpe_mlx.npz) read back into the reference's torch
names and layouts, bit-exactly (CPU; the device run of the same files is tests/test_gpu_weights_e2e.py)."""
import numpy as np

from mlx_convert import hubert_to_mlx, rmvpe_to_mlx


def _same(a, b):
    assert set(a) == set(b), (sorted(set(a) ^ set(b)))[:8]
    for k in a:
        assert a[k].shape == b[k].shape, (k, a[k].shape, b[k].shape)
        assert np.array_equal(a[k], b[k]), k


def test_mlx_hubert_file_round_trip(tmp_path):
    from rvcx import synthetic
    from rvcx.weights import is_mlx_hubert, load_state_file, normalize_state

    st = synthetic.hubert_state(4)
    mlx = hubert_to_mlx(st)
    assert is_mlx_hubert(mlx) and not is_mlx_hubert(st)
    assert mlx["encoder.pos_conv_embed.weight"].shape == (768, 128, 48)   # (O, K, I/G)
    assert mlx["feature_extractor.conv_layers.0.conv.weight"].shape == (512, 10, 1)
    p = tmp_path / "hubert_mlx.npz"
    np.savez(p, **mlx)
    ref = {k: v for k, v in normalize_state(st).items() if k != "masked_spec_embed"}
    _same(load_state_file(str(p)), ref)


def test_mlx_rmvpe_file_round_trip(tmp_path):
    from rvcx import synthetic
    from rvcx.weights import is_mlx_rmvpe, load_state_file, normalize_state

    st = synthetic.rmvpe_state(5)
    mlx = rmvpe_to_mlx(st)
    assert is_mlx_rmvpe(mlx) and not is_mlx_rmvpe(st)
    # spot-check the converter's names and layouts (tools/convert_rmvpe.py:36-81)
    assert "unet.encoder.layers.0.blocks.0.conv1.weight" in mlx
    assert "unet.decoder.layers.0.blocks.1.bn2.running_var" in mlx
    assert "fc.bigru.backward_grus.0.weight_hh" in mlx and "fc.linear.bias" in mlx
    ct = st["unet.decoder.layers.0.conv1.0.weight"]                       # (In, Out, H, W)
    assert mlx["unet.decoder.layers.0.conv1_trans.weight"].shape == (ct.shape[1], ct.shape[2], ct.shape[3], ct.shape[0])
    p = tmp_path / "rmvpe_mlx.npz"
    np.savez(p, **mlx)
    _same(load_state_file(str(p)), normalize_state(st))


def test_rvc_mlx_searches_the_mlx_tree_first():
    from rvcx.infer.infer import HUBERT_CANDIDATES, RMVPE_CANDIDATES

    # infer_mlx.py:260-264 and rvc_mlx/lib/mlx/rmvpe.py:258
    assert HUBERT_CANDIDATES[:2] == ("rvc_mlx/models/embedders/contentvec/hubert_mlx.npz",
                                     "rvc/models/embedders/contentvec/hubert_mlx.npz")
    assert RMVPE_CANDIDATES[0] == "rvc_mlx/models/predictors/rmvpe_mlx.npz"
