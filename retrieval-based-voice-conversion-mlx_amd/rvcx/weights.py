"""Weight ingestion: reference checkpoints -> plain float32 tensors under reference names.

Handles the on-disk formats of the path:
  - RVC ``.pth`` (zip dict with ``weight``/``config``/``f0``/``version``/``sr``),
    fp16 tensors, weight-norm pairs ``*.weight_g``/``*.weight_v``
    (rvc/train/process/extract_model.py:57-109), loaded with
    ``torch.load(weights_only=True)`` only.
  - live torch parametrization names ``*.parametrizations.weight.original0/1``.
  - the MLX tree's own HuBERT and RMVPE files (``hubert_mlx.npz``, tools/convert_hubert.py:36-70;
    ``rmvpe_mlx.npz``, tools/convert_rmvpe.py:26-83): ``load_state_file`` recognises their names and
    layouts and inverts them (``mlx_hubert_to_reference``, ``mlx_rmvpe_to_reference``).
  - MLX voice ``.npz`` / ``.safetensors`` exported by tools/convert_rvc_model.py: already-fused weights
    under remapped keys; ``unmap_mlx_keys`` here, the layouts in rvcx/infer/infer.py
    ``mlx_to_reference_state``.

Weight-norm fusion matches torch exactly (``torch._weight_norm``: w = g * v / ||v||,
norm over every dim except ``dim``, no epsilon). ``dim`` is 0 for every RVC conv
(for ConvTranspose1d that is the input-channel axis) and 2 for the HuBERT
positional conv (modeling_hubert.py HubertPositionalConvEmbedding).
"""
from __future__ import annotations

import re
from typing import Dict, Mapping

import numpy as np

_WN_PAIRS = (
    (".weight_g", ".weight_v"),
    (".parametrizations.weight.original0", ".parametrizations.weight.original1"),
)


def _wn_dim(g_shape) -> int:
    """Infer the weight-norm ``dim`` from the shape of g (all ones except ``dim``)."""
    non1 = [i for i, s in enumerate(g_shape) if s != 1]
    if len(non1) == 1:
        return non1[0]
    if len(non1) == 0:
        return 0
    raise ValueError(f"cannot infer weight_norm dim from g shape {tuple(g_shape)}")


def fuse_weight_norm(v: np.ndarray, g: np.ndarray) -> np.ndarray:
    import torch

    dim = _wn_dim(g.shape)
    tv = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32))
    tg = torch.from_numpy(np.ascontiguousarray(g, dtype=np.float32))
    return torch._weight_norm(tv, tg, dim).numpy().astype(np.float32)


def normalize_state(sd: Mapping[str, object]) -> Dict[str, np.ndarray]:
    """Fuse weight-norm pairs, cast to float32 numpy, drop non-float bookkeeping."""
    arrs: Dict[str, np.ndarray] = {}
    for k, v in sd.items():
        if hasattr(v, "detach"):
            v = v.detach().cpu()
            v = v.float().numpy() if v.is_floating_point() else v.numpy()
        arrs[k] = np.asarray(v)
    out: Dict[str, np.ndarray] = {}
    used = set()
    for k, v in arrs.items():
        for gs, vs in _WN_PAIRS:
            if k.endswith(gs):
                base = k[: -len(gs)]
                vk = base + vs
                if vk not in arrs:
                    raise KeyError(f"weight-norm pair incomplete: {k} without {vk}")
                out[base + ".weight"] = fuse_weight_norm(arrs[vk], v)
                used.update((k, vk))
    for k, v in arrs.items():
        if k in used:
            continue
        if k.endswith("num_batches_tracked"):
            continue
        if not np.issubdtype(v.dtype, np.floating):
            raise TypeError(f"non-float tensor {k} ({v.dtype}) in a weight dict")
        out[k] = np.ascontiguousarray(v, dtype=np.float32)
    return out


def load_rvc_checkpoint(path: str):
    """Load an RVC ``.pth`` with the non-executing loader. Returns (state, cfg_list, meta)."""
    import torch

    cpt = torch.load(path, map_location="cpu", weights_only=True)
    if "weight" not in cpt:
        raise ValueError(f"{path}: not an RVC inference checkpoint (no 'weight' key)")
    state = {k: v for k, v in cpt["weight"].items() if not k.startswith("enc_q.")}
    meta = {k: cpt.get(k) for k in ("f0", "version", "sr", "vocoder")}
    return normalize_state(state), list(cpt.get("config", [])), meta


def load_state_file(path: str) -> Dict[str, np.ndarray]:
    """Load a bare state dict (``rmvpe.pt``, ``pytorch_model.bin``, ``.safetensors``, ``.npz``). MLX-tree
    HuBERT / RMVPE files (``hubert_mlx.npz``, ``rmvpe_mlx.npz``) come back under the reference's torch names
    and layouts."""
    if path.endswith(".safetensors"):
        from safetensors.numpy import load_file

        return normalize_state(to_reference_layout(load_file(path)))
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            return normalize_state(to_reference_layout({k: z[k] for k in z.files}))
    import torch

    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "weight" in sd and isinstance(sd["weight"], dict):
        sd = sd["weight"]
    return normalize_state(sd)


def _np32(v) -> np.ndarray:
    return np.asarray(v.detach().cpu().numpy() if hasattr(v, "detach") else v)


def is_mlx_hubert(keys) -> bool:
    """tools/convert_hubert.py:26-31 stores the fused positional-conv weight as ``encoder.pos_conv_embed.weight``
    (no ``.conv.``); a torch/HF ContentVec state never has that key."""
    return "encoder.pos_conv_embed.weight" in set(keys)


def is_mlx_rmvpe(keys) -> bool:
    """tools/convert_rmvpe.py:56-74 renames the BiGRU to ``fc.bigru.*`` and the classifier to ``fc.linear.*``."""
    return any(k.startswith("fc.bigru.") or k.startswith("fc.linear.") or (k.startswith("unet.") and ".blocks." in k)
               for k in keys)


def mlx_hubert_to_reference(sd: Mapping[str, object]) -> Dict[str, np.ndarray]:
    """Invert tools/convert_hubert.py:26-67: ``encoder.pos_conv_embed.weight`` (O, K, I/G), already fused by
    the weight-norm parametrization) -> ``encoder.pos_conv_embed.conv.weight`` (O, I/G, K);
    ``encoder.pos_conv_embed.bias`` -> ``...conv.bias``; the feature-encoder Conv1d weights (O, K, I) ->
    (O, I, K); linears and norms unchanged (MLX nn.Linear is (O, I) like torch). A stray ``hubert.`` prefix
    (convert_hubert.py:40-41 strips it) is dropped too."""
    out: Dict[str, np.ndarray] = {}
    for k, v in sd.items():
        a = _np32(v)
        n = k[len("hubert."):] if k.startswith("hubert.") else k
        if n == "encoder.pos_conv_embed.weight":
            n, a = "encoder.pos_conv_embed.conv.weight", a.transpose(0, 2, 1)
        elif n == "encoder.pos_conv_embed.bias":
            n = "encoder.pos_conv_embed.conv.bias"
        elif n.startswith("feature_extractor.conv_layers.") and n.endswith(".conv.weight") and a.ndim == 3:
            a = a.transpose(0, 2, 1)
        out[n] = np.ascontiguousarray(a)
    return out


_RMVPE_BLOCK_INNER = {"conv1": "conv.0", "bn1": "conv.1", "conv2": "conv.3", "bn2": "conv.4"}
_RMVPE_BLOCK = re.compile(r"^(unet\.(encoder|intermediate|decoder)\.layers\.\d+)\.blocks\.(\d+)\.([a-z0-9_]+)\.(.*)$")
_RMVPE_DEC_HEAD = re.compile(r"^(unet\.decoder\.layers\.\d+)\.(conv1_trans|bn1)\.(.*)$")
_RMVPE_GRU = re.compile(r"^fc\.bigru\.(forward|backward)_grus\.0\.(weight_ih|weight_hh|bias_ih|bias_hh)$")


def mlx_rmvpe_to_reference(sd: Mapping[str, object]) -> Dict[str, np.ndarray]:
    """Invert tools/convert_rmvpe.py:26-83 (E2E of rvc/lib/predictors/RMVPE.py:289-340):
      * ``unet.{encoder,intermediate}.layers.L.blocks.B.X`` -> ``...layers.L.conv.B.Y`` and
        ``unet.decoder.layers.L.blocks.B.X`` -> ``...layers.L.conv2.B.Y``, with the ConvBlockRes members
        X = conv1 / bn1 / conv2 / bn2 -> Y = conv.0 / conv.1 / conv.3 / conv.4 (``shortcut`` unchanged);
      * ``unet.decoder.layers.L.conv1_trans`` / ``.bn1`` -> ``.conv1.0`` / ``.conv1.1``;
      * ``fc.bigru.{forward,backward}_grus.0.W`` -> ``fc.0.gru.W_l0`` / ``W_l0_reverse``; ``fc.linear`` -> ``fc.1``;
      * Conv2d weights (O, H, W, I) -> (O, I, H, W); the ConvTranspose2d weight (O, H, W, I) -> (I, O, H, W)."""
    out: Dict[str, np.ndarray] = {}
    for k, v in sd.items():
        a = _np32(v)
        n, trans = k, False
        m = _RMVPE_BLOCK.match(k)
        if m:
            head, part, blk, member, rest = m.groups()
            holder = "conv2" if part == "decoder" else "conv"
            n = f"{head}.{holder}.{blk}.{_RMVPE_BLOCK_INNER.get(member, member)}.{rest}"
        else:
            m = _RMVPE_DEC_HEAD.match(k)
            if m:
                head, member, rest = m.groups()
                trans = member == "conv1_trans"
                n = f"{head}.conv1.{0 if trans else 1}.{rest}"
            else:
                m = _RMVPE_GRU.match(k)
                if m:
                    n = f"fc.0.gru.{m.group(2)}_l0{'_reverse' if m.group(1) == 'backward' else ''}"
                elif k.startswith("fc.linear."):
                    n = "fc.1." + k[len("fc.linear."):]
        if a.ndim == 4 and k.endswith("weight"):
            a = a.transpose(3, 0, 1, 2) if trans else a.transpose(0, 3, 1, 2)
        out[n] = np.ascontiguousarray(a)
    return out


def to_reference_layout(sd: Mapping[str, object]) -> Mapping[str, object]:
    """MLX-tree HuBERT / RMVPE states -> reference names and layouts; any other state passes through."""
    if is_mlx_hubert(sd.keys()):
        return mlx_hubert_to_reference(sd)
    if is_mlx_rmvpe(sd.keys()):
        return mlx_rmvpe_to_reference(sd)
    return sd


_MLX_RULES = [
    (re.compile(r"^dec\.resblock_(\d+)\.c([12])_(\d+)\.(.*)$"), r"dec.resblocks.\1.convs\2.\3.\4"),
    (re.compile(r"^dec\.up_(\d+)\.(.*)$"), r"dec.ups.\1.\2"),
    (re.compile(r"^dec\.noise_conv_(\d+)\.(.*)$"), r"dec.noise_convs.\1.\2"),
    (re.compile(r"^enc_p\.encoder\.attn_(\d+)\.(.*)$"), r"enc_p.encoder.attn_layers.\1.\2"),
    (re.compile(r"^enc_p\.encoder\.norm1_(\d+)\.(.*)$"), r"enc_p.encoder.norm_layers_1.\1.\2"),
    (re.compile(r"^enc_p\.encoder\.norm2_(\d+)\.(.*)$"), r"enc_p.encoder.norm_layers_2.\1.\2"),
    (re.compile(r"^enc_p\.encoder\.ffn_(\d+)\.(.*)$"), r"enc_p.encoder.ffn_layers.\1.\2"),
    (re.compile(r"^flow\.flow_(\d+)\.enc\.in_layer_(\d+)\.(.*)$"), r"flow.flows.\1.enc.in_layers.\2.\3"),
    (re.compile(r"^flow\.flow_(\d+)\.enc\.res_skip_layer_(\d+)\.(.*)$"), r"flow.flows.\1.enc.res_skip_layers.\2.\3"),
    (re.compile(r"^flow\.flow_(\d+)\.(.*)$"), r"flow.flows.\1.\2"),
]


def unmap_mlx_keys(keys) -> Dict[str, str]:
    """Inverse of rvc_mlx/infer/infer_mlx.py:17-89 ``remap_keys`` (name mapping only)."""
    out = {}
    for k in keys:
        n = k
        for pat, rep in _MLX_RULES:
            if pat.match(n):
                n = pat.sub(rep, n)
                break
        if n.startswith("enc_p.encoder.norm_layers_"):
            n = n.replace(".weight", ".gamma").replace(".bias", ".beta")
        out[k] = n
    return out


def crepe_torch_layout(sd: Mapping[str, object]) -> Dict[str, np.ndarray]:
    """CREPE weights in torchcrepe's names and layouts (conv{i}.weight [O][I][K][1], classifier.weight
    [360][in]) from either torchcrepe's own state dict or the MLX npz that tools/convert_crepe_weights.py:43-70
    writes (conv weights transposed to (O, K, 1, I), the classifier weight to (in, 360))."""
    out = {}
    for k, v in sd.items():
        a = np.asarray(v.detach().cpu().numpy() if hasattr(v, "detach") else v, dtype=np.float32)
        if k.endswith("num_batches_tracked"):
            continue
        if k.startswith("conv") and k.endswith(".weight") and a.ndim == 4 and "_BN" not in k:
            if a.shape[2] == 1:  # MLX (O, K, 1, I) -> torch (O, I, K, 1) (torch dim 2 is the kernel, 512 or 64)
                a = np.ascontiguousarray(a.transpose(0, 3, 1, 2))
        elif k == "classifier.weight" and a.ndim == 2 and a.shape[1] == 360 and a.shape[0] != 360:
            a = np.ascontiguousarray(a.T)  # MLX converter's (in, 360) -> (360, in)
        out[k] = a
    return out


def load_crepe_weights(path: str) -> Dict[str, np.ndarray]:
    """crepe_full.npz / crepe_tiny.npz (MLX, rvc_mlx/lib/mlx/crepe.py:270-280), .safetensors, or torchcrepe's
    full.pth / tiny.pth (weights_only)."""
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            return crepe_torch_layout({k: z[k] for k in z.files})
    if path.endswith(".safetensors"):
        from safetensors.numpy import load_file

        return crepe_torch_layout(load_file(path))
    import torch

    return crepe_torch_layout(torch.load(path, map_location="cpu", weights_only=True))
