"""Model and pipeline constants for the RVC v2 48 kHz inference path.

Values follow the reference configs:
  - synthesizer list layout: rvc/train/process/extract_model.py:62-81 and
    rvc/configs/48000.json (upsample [12,10,2,2], kernels [24,20,4,4], ...)
  - pipeline constants x_pad/x_query/x_center/x_max: rvc_mlx/configs/config.py:9-15
    and rvc/configs/config.py:23-56
  - HuBERT/ContentVec: rvc_mlx/models/embedders/contentvec/config.json
  - RMVPE: rvc/lib/predictors/RMVPE.py:420-443 (E2E(4, 1, (2, 2)), 128 mels,
    hop 160, win 1024, fmin 30, fmax 8000)
"""
from __future__ import annotations

import dataclasses
import json
import math
import os
from typing import List, Sequence


@dataclasses.dataclass(frozen=True)
class SynthConfig:
    """SynthesizerTrnMs768NSFsid hyper-parameters (the .pth ``config`` list)."""

    spec_channels: int = 1025
    segment_size: int = 36
    inter_channels: int = 192
    hidden_channels: int = 192
    filter_channels: int = 768
    n_heads: int = 2
    n_layers: int = 6
    kernel_size: int = 3
    p_dropout: float = 0.0
    resblock: str = "1"
    resblock_kernel_sizes: tuple = (3, 7, 11)
    resblock_dilation_sizes: tuple = ((1, 3, 5), (1, 3, 5), (1, 3, 5))
    upsample_rates: tuple = (12, 10, 2, 2)
    upsample_initial_channel: int = 512
    upsample_kernel_sizes: tuple = (24, 20, 4, 4)
    spk_embed_dim: int = 109
    gin_channels: int = 256
    sr: int = 48000
    text_enc_hidden_dim: int = 768
    window_size: int = 10  # encoders.py:33 (Encoder default window_size=10)
    flow_kernel: int = 5  # synthesizers.py:154-161 (ResidualCouplingBlock(..., 5, 1, 3))
    flow_layers: int = 3
    flow_n: int = 4
    use_f0: bool = True  # cpt["f0"]: pitch-guided (NSF decoders) or the plain HiFiGANGenerator (synthesizers.py:84-139)
    vocoder: str = "HiFi-GAN"  # cpt["vocoder"] (infer.py:478): "HiFi-GAN" | "MRF HiFi-GAN" | "RefineGAN"

    @property
    def upp(self) -> int:
        return int(math.prod(self.upsample_rates))

    def as_list(self) -> list:
        """The 18-element list stored as ``cpt['config']`` (extract_model.py:62-81)."""
        return [
            self.spec_channels, self.segment_size, self.inter_channels,
            self.hidden_channels, self.filter_channels, self.n_heads, self.n_layers,
            self.kernel_size, self.p_dropout, self.resblock,
            [int(k) for k in self.resblock_kernel_sizes],
            [[int(d) for d in ds] for ds in self.resblock_dilation_sizes],
            [int(u) for u in self.upsample_rates], self.upsample_initial_channel,
            [int(k) for k in self.upsample_kernel_sizes], self.spk_embed_dim,
            self.gin_channels, self.sr,
        ]

    @staticmethod
    def from_list(cfg: Sequence) -> "SynthConfig":
        if len(cfg) < 18:
            raise ValueError(f"synthesizer config list needs 18 entries, got {len(cfg)}")
        return SynthConfig(
            spec_channels=int(cfg[0]), segment_size=int(cfg[1]),
            inter_channels=int(cfg[2]), hidden_channels=int(cfg[3]),
            filter_channels=int(cfg[4]), n_heads=int(cfg[5]), n_layers=int(cfg[6]),
            kernel_size=int(cfg[7]), p_dropout=float(cfg[8]), resblock=str(cfg[9]),
            resblock_kernel_sizes=tuple(int(k) for k in cfg[10]),
            resblock_dilation_sizes=tuple(tuple(int(d) for d in ds) for ds in cfg[11]),
            upsample_rates=tuple(int(u) for u in cfg[12]),
            upsample_initial_channel=int(cfg[13]),
            upsample_kernel_sizes=tuple(int(k) for k in cfg[14]),
            spk_embed_dim=int(cfg[15]), gin_channels=int(cfg[16]), sr=int(cfg[17]),
        )

    @staticmethod
    def from_json(path: str) -> "SynthConfig":
        """Read a per-sample-rate JSON (rvc/configs/48000.json layout) or an exported list."""
        with open(path) as f:
            conf = json.load(f)
        if isinstance(conf, list):
            return SynthConfig.from_list(conf)
        m, d = conf.get("model", {}), conf.get("data", {})
        base = SynthConfig()
        return dataclasses.replace(
            base,
            inter_channels=m.get("inter_channels", base.inter_channels),
            hidden_channels=m.get("hidden_channels", base.hidden_channels),
            filter_channels=m.get("filter_channels", base.filter_channels),
            n_heads=m.get("n_heads", base.n_heads), n_layers=m.get("n_layers", base.n_layers),
            kernel_size=m.get("kernel_size", base.kernel_size),
            resblock_kernel_sizes=tuple(m.get("resblock_kernel_sizes", base.resblock_kernel_sizes)),
            resblock_dilation_sizes=tuple(tuple(x) for x in m.get(
                "resblock_dilation_sizes", base.resblock_dilation_sizes)),
            upsample_rates=tuple(m.get("upsample_rates", base.upsample_rates)),
            upsample_initial_channel=m.get("upsample_initial_channel", base.upsample_initial_channel),
            upsample_kernel_sizes=tuple(m.get("upsample_kernel_sizes", base.upsample_kernel_sizes)),
            spk_embed_dim=m.get("spk_embed_dim", base.spk_embed_dim),
            gin_channels=m.get("gin_channels", base.gin_channels),
            text_enc_hidden_dim=m.get("text_enc_hidden_dim", base.text_enc_hidden_dim),
            sr=d.get("sample_rate", base.sr),
        )


@dataclasses.dataclass(frozen=True)
class HubertConfig:
    """ContentVec / HuBERT-base (rvc_mlx/models/embedders/contentvec/config.json)."""

    conv_dim: tuple = (512,) * 7
    conv_kernel: tuple = (10, 3, 3, 3, 3, 2, 2)
    conv_stride: tuple = (5, 2, 2, 2, 2, 2, 2)
    hidden_size: int = 768
    num_heads: int = 12
    num_layers: int = 12
    intermediate_size: int = 3072
    num_conv_pos_embeddings: int = 128
    num_conv_pos_embedding_groups: int = 16
    layer_norm_eps: float = 1e-5
    classifier_proj_size: int = 256  # final_proj (v1 only)

    def frames(self, n_samples: int) -> int:
        t = n_samples
        for k, s in zip(self.conv_kernel, self.conv_stride):
            t = (t - k) // s + 1
        return t


@dataclasses.dataclass(frozen=True)
class RmvpeConfig:
    n_mels: int = 128
    n_class: int = 360
    sample_rate: int = 16000
    win_length: int = 1024
    hop_length: int = 160
    n_fft: int = 1024
    mel_fmin: float = 30.0
    mel_fmax: float = 8000.0
    clamp: float = 1e-5
    en_de_layers: int = 5
    inter_layers: int = 4
    n_blocks: int = 4
    en_out_channels: int = 16
    gru_hidden: int = 256


@dataclasses.dataclass
class PipelineConfig:
    """Pipeline constants (rvc_mlx/configs/config.py:9-15; rvc/configs/config.py:23-56)."""

    x_pad: float = 1
    x_query: float = 6
    x_center: float = 38
    x_max: float = 41
    device: str = "cuda:0"
    is_half: bool = False

    def device_config(self):
        return self.x_pad, self.x_query, self.x_center, self.x_max


SYNTH_48K_V2 = SynthConfig()
HUBERT_BASE = HubertConfig()
RMVPE_CFG = RmvpeConfig()


def config_dir() -> str:
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs")
