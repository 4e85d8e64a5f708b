"""Test infrastructure: the MLX tree's HuBERT / RMVPE weight converters restated in numpy (mlx is absent here),
so tests can write ``hubert_mlx.npz`` / ``rmvpe_mlx.npz`` exactly as a user of ``rvc_mlx.infer`` holds them.

  * ``hubert_to_mlx`` follows tools/convert_hubert.py:26-67: the positional conv's weight as the weight-norm
    parametrization computes it (torch._weight_norm over dim 2), transposed (O, I/G, K) -> (O, K, I/G) and stored
    as ``encoder.pos_conv_embed.weight``; ``hubert.`` stripped, ``masked_spec_embed`` and the pos-conv weight-norm
    pieces dropped, ``pos_conv_embed.conv.`` -> ``pos_conv_embed.``, feature-encoder Conv1d weights (O, I, K) ->
    (O, K, I), everything else as is.
  * ``rmvpe_to_mlx`` follows tools/convert_rmvpe.py:26-83: the same regex substitutions in the same order
    (``.conv.N.`` -> ``.blocks.N.`` in the encoder / intermediate, ``.conv2.N.`` -> ``.blocks.N.`` in the decoder,
    ConvBlockRes ``conv.0/1/3/4`` -> ``conv1/bn1/conv2/bn2``, decoder ``conv1.0/1`` -> ``conv1_trans/bn1``, the GRU
    to ``fc.bigru.{forward,backward}_grus.0.*``, ``fc.1.`` -> ``fc.linear.``) and the 4-D transposes
    ((O, I, H, W) -> (O, H, W, I); ConvTranspose2d (I, O, H, W) -> (O, H, W, I)).
"""
import re

import numpy as np


def hubert_to_mlx(state):
    import torch

    out = {}
    g = np.asarray(state["encoder.pos_conv_embed.conv.weight_g"], np.float32)
    v = np.asarray(state["encoder.pos_conv_embed.conv.weight_v"], np.float32)
    w = torch._weight_norm(torch.from_numpy(v), torch.from_numpy(g), 2).numpy()
    out["encoder.pos_conv_embed.weight"] = np.ascontiguousarray(w.transpose(0, 2, 1))
    for key, val in state.items():
        k = key[len("hubert."):] if key.startswith("hubert.") else key
        if "masked_spec_embed" in k:
            continue
        if "pos_conv_embed" in k and (".weight" in k or "weight_" in k or "parametrizations" in k):
            continue
        k = k.replace("pos_conv_embed.conv.", "pos_conv_embed.")
        a = np.asarray(val, np.float32)
        if "feature_extractor.conv_layers" in k and "weight" in k and a.ndim == 3:
            a = a.transpose(0, 2, 1)
        out[k] = np.ascontiguousarray(a)
    return out


def rmvpe_to_mlx(state):
    out = {}
    for key, val in state.items():
        if "num_batches_tracked" in key:
            continue
        a = np.asarray(val)
        k = key
        if k.startswith("unet."):
            if "encoder.layers." in k or "intermediate.layers." in k:
                k = re.sub(r"\.conv\.(\d+)\.", r".blocks.\1.", k)
            if "decoder.layers." in k:
                k = re.sub(r"\.conv2\.(\d+)\.", r".blocks.\1.", k)
            if ".blocks." in k and ".conv." in k:
                for src, dst in ((r"\.conv\.0\.", ".conv1."), (r"\.conv\.1\.", ".bn1."),
                                 (r"\.conv\.3\.", ".conv2."), (r"\.conv\.4\.", ".bn2.")):
                    k = re.sub(src, dst, k)
            if "decoder.layers." in k:
                k = re.sub(r"\.conv1\.0\.", ".conv1_trans.", k)
                k = re.sub(r"\.conv1\.1\.", ".bn1.", k)
        if k.startswith("fc.0.gru."):
            d = "backward_grus.0" if "l0_reverse" in k else "forward_grus.0"
            for w in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
                if w in k:
                    k = f"fc.bigru.{d}.{w}"
                    break
        if k.startswith("fc.1."):
            k = k.replace("fc.1.", "fc.linear.")
        if "weight" in key and a.ndim == 4:
            a = a.transpose(1, 2, 3, 0) if "conv1_trans" in k else a.transpose(0, 2, 3, 1)
        out[k] = np.ascontiguousarray(a)
    return out
