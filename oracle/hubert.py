"""Oracle: HuBERT / ContentVec feature extractor (``last_hidden_state``).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). Restates transformers'
HubertModel.forward (pinned 4.57.3 in the reference's uv.lock:3261-3262; the
container has 5.15.0, whose modeling_hubert.py is the text followed here) for the
contentvec config (rvc_mlx/models/embedders/contentvec/config.json):
feat_extract_norm="group", feat_proj_layer_norm=True, do_stable_layer_norm=False.
Called by the pipeline as ``model(feats)["last_hidden_state"]`` (rvc/infer/pipeline.py:331).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from oracle.synth import _t


def hubert_forward(w, cfg, audio: torch.Tensor, version: str = "v2") -> torch.Tensor:
    """audio [B, N] float32 -> [B, L, 768] (v2) or [B, L, 256] (v1, final_proj; pipeline.py:332-334)."""
    with torch.no_grad():
        x = audio[:, None]
        # HubertFeatureEncoder (modeling_hubert.py HubertGroupNormConvLayer / NoLayerNormConvLayer)
        for i, s in enumerate(cfg.conv_stride):
            x = F.conv1d(x, _t(w, f"feature_extractor.conv_layers.{i}.conv.weight"), None, stride=s)
            if i == 0:
                x = F.group_norm(x, x.shape[1], _t(w, "feature_extractor.conv_layers.0.layer_norm.weight"),
                                 _t(w, "feature_extractor.conv_layers.0.layer_norm.bias"), 1e-5)
            x = F.gelu(x)
        x = x.transpose(1, 2)
        # HubertFeatureProjection
        x = F.layer_norm(x, (x.shape[-1],), _t(w, "feature_projection.layer_norm.weight"),
                         _t(w, "feature_projection.layer_norm.bias"), cfg.layer_norm_eps)
        x = F.linear(x, _t(w, "feature_projection.projection.weight"), _t(w, "feature_projection.projection.bias"))
        # HubertEncoder: positional conv (weight_norm dim=2, same-pad removes the last frame)
        K = cfg.num_conv_pos_embeddings
        pos = F.conv1d(x.transpose(1, 2), _t(w, "encoder.pos_conv_embed.conv.weight"),
                       _t(w, "encoder.pos_conv_embed.conv.bias"), padding=K // 2,
                       groups=cfg.num_conv_pos_embedding_groups)
        if K % 2 == 0:
            pos = pos[:, :, :-1]
        pos = F.gelu(pos).transpose(1, 2)
        x = x + pos
        x = F.layer_norm(x, (x.shape[-1],), _t(w, "encoder.layer_norm.weight"), _t(w, "encoder.layer_norm.bias"),
                         cfg.layer_norm_eps)
        B, L, D = x.shape
        nh = cfg.num_heads
        hd = D // nh
        for i in range(cfg.num_layers):
            p = f"encoder.layers.{i}"
            res = x
            q = F.linear(x, _t(w, p + ".attention.q_proj.weight"), _t(w, p + ".attention.q_proj.bias"))
            k = F.linear(x, _t(w, p + ".attention.k_proj.weight"), _t(w, p + ".attention.k_proj.bias"))
            v = F.linear(x, _t(w, p + ".attention.v_proj.weight"), _t(w, p + ".attention.v_proj.bias"))
            q = q.view(B, L, nh, hd).transpose(1, 2)
            k = k.view(B, L, nh, hd).transpose(1, 2)
            v = v.view(B, L, nh, hd).transpose(1, 2)
            att = torch.matmul(q, k.transpose(2, 3)) * (hd ** -0.5)
            att = torch.softmax(att, dim=-1)
            o = torch.matmul(att, v).transpose(1, 2).reshape(B, L, D)
            o = F.linear(o, _t(w, p + ".attention.out_proj.weight"), _t(w, p + ".attention.out_proj.bias"))
            x = res + o
            x = F.layer_norm(x, (D,), _t(w, p + ".layer_norm.weight"), _t(w, p + ".layer_norm.bias"),
                             cfg.layer_norm_eps)
            h = F.linear(x, _t(w, p + ".feed_forward.intermediate_dense.weight"),
                         _t(w, p + ".feed_forward.intermediate_dense.bias"))
            h = F.gelu(h)
            h = F.linear(h, _t(w, p + ".feed_forward.output_dense.weight"),
                         _t(w, p + ".feed_forward.output_dense.bias"))
            x = x + h
            x = F.layer_norm(x, (D,), _t(w, p + ".final_layer_norm.weight"), _t(w, p + ".final_layer_norm.bias"),
                             cfg.layer_norm_eps)
        if version == "v1":
            x = F.linear(x, _t(w, "final_proj.weight"), _t(w, "final_proj.bias"))
    return x
