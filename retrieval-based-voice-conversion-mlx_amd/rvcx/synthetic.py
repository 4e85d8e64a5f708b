"""Seeded synthetic weights and inputs for the RVC v2 48 kHz path.

The container and the GPU box ship no checkpoints, so every parity test and the
benchmark run on random-initialised weights of the exact reference architecture.
Tensor names and shapes follow the reference state dicts:

  - Synthesizer (.pth ``weight`` dict, weight-norm pairs stored as
    ``*.weight_g`` / ``*.weight_v``): rvc/train/process/extract_model.py:57-109,
    module tree rvc/lib/algorithm/synthesizers.py:12-170 (``enc_q`` deleted as in
    rvc/infer/infer.py:467-488).
  - HuBERT / ContentVec (HF names): transformers modeling_hubert.py
    (HubertModel), config rvc_mlx/models/embedders/contentvec/config.json.
  - RMVPE E2E(4, 1, (2, 2)) state dict: rvc/lib/predictors/RMVPE.py:13-339.

Init scales are chosen so activations stay O(1) through every stack (the
reference's own ``init_weights`` uses N(0, 0.01); any scale is valid for parity).
"""
from __future__ import annotations

from typing import Dict, Iterator, List, Tuple

import numpy as np

from .config import HUBERT_BASE, RMVPE_CFG, SYNTH_48K_V2, HubertConfig, RmvpeConfig, SynthConfig

# (name, shape, kind) ; kind selects the init rule below
Spec = Tuple[str, Tuple[int, ...], str]


# --------------------------------------------------------------------------- specs
def _wn(prefix: str, shape, dim0_len: int) -> List[Spec]:
    """Weight-normed conv: g has shape (dim0,1,...) (torch weight_norm, dim=0)."""
    gshape = (dim0_len,) + (1,) * (len(shape) - 1)
    return [(prefix + ".weight_g", gshape, "wn_g"), (prefix + ".weight_v", tuple(shape), "conv")]


def synth_specs(cfg: SynthConfig = SYNTH_48K_V2) -> List[Spec]:
    H, I, F = cfg.hidden_channels, cfg.inter_channels, cfg.filter_channels
    dk = H // cfg.n_heads
    s: List[Spec] = []
    # TextEncoder (encoders.py:88-144, attentions.py:6-243, normalization.py:4-26)
    s += [("enc_p.emb_phone.weight", (H, cfg.text_enc_hidden_dim), "linear"),
          ("enc_p.emb_phone.bias", (H,), "bias")]
    if cfg.use_f0:
        s += [("enc_p.emb_pitch.weight", (256, H), "embed")]
    for i in range(cfg.n_layers):
        p = f"enc_p.encoder.attn_layers.{i}"
        for c in "qkvo":
            s += [(f"{p}.conv_{c}.weight", (H, H, 1), "conv"), (f"{p}.conv_{c}.bias", (H,), "bias")]
        s += [(f"{p}.emb_rel_k", (1, 2 * cfg.window_size + 1, dk), "relemb"),
              (f"{p}.emb_rel_v", (1, 2 * cfg.window_size + 1, dk), "relemb")]
        s += [(f"enc_p.encoder.norm_layers_1.{i}.gamma", (H,), "ln_g"),
              (f"enc_p.encoder.norm_layers_1.{i}.beta", (H,), "ln_b")]
        s += [(f"enc_p.encoder.ffn_layers.{i}.conv_1.weight", (F, H, cfg.kernel_size), "conv"),
              (f"enc_p.encoder.ffn_layers.{i}.conv_1.bias", (F,), "bias"),
              (f"enc_p.encoder.ffn_layers.{i}.conv_2.weight", (H, F, cfg.kernel_size), "conv"),
              (f"enc_p.encoder.ffn_layers.{i}.conv_2.bias", (H,), "bias")]
        s += [(f"enc_p.encoder.norm_layers_2.{i}.gamma", (H,), "ln_g"),
              (f"enc_p.encoder.norm_layers_2.{i}.beta", (H,), "ln_b")]
    s += [("enc_p.proj.weight", (2 * I, H, 1), "proj"), ("enc_p.proj.bias", (2 * I,), "bias")]
    # HiFiGAN-NSF generator (generators/hifigan_nsf.py:55-171); MRF HiFi-GAN (generators/hifigan_mrf.py:234-330)
    # has the same dataflow under other names, a 9-harmonic source, weight-normed conv_pre and a conv_post bias
    C0 = cfg.upsample_initial_channel
    if cfg.use_f0 and cfg.vocoder == "RefineGAN":
        s += _refinegan_specs(cfg)
        return s + _flow_emb_specs(cfg)
    mrf = cfg.use_f0 and cfg.vocoder == "MRF HiFi-GAN"
    if cfg.use_f0:  # the plain HiFiGANGenerator (no pitch guidance) has no source module (hifigan.py:9-65)
        if mrf:
            s += [("dec.m_source.l_linear.weight", (1, 9), "linear"), ("dec.m_source.l_linear.bias", (1,), "bias")]
        else:
            s += [("dec.m_source.l_linear.weight", (1, 1), "src_lin"),
                  ("dec.m_source.l_linear.bias", (1,), "bias")]
    if mrf:
        s += _wn("dec.conv_pre", (C0, I, 7), C0) + [("dec.conv_pre.bias", (C0,), "bias")]
    else:
        s += [("dec.conv_pre.weight", (C0, I, 7), "conv"), ("dec.conv_pre.bias", (C0,), "bias")]
    chans = [C0 // (2 ** (i + 1)) for i in range(len(cfg.upsample_rates))]
    up_name = "dec.upsamples" if mrf else "dec.ups"
    for i, (u, k) in enumerate(zip(cfg.upsample_rates, cfg.upsample_kernel_sizes)):
        cin = C0 // (2 ** i)
        s += _wn(f"{up_name}.{i}", (cin, chans[i], k), cin)
        s += [(f"{up_name}.{i}.bias", (chans[i],), "bias")]
    ups = list(cfg.upsample_rates)
    for i in range(len(ups) if cfg.use_f0 else 0):
        stride = int(np.prod(ups[i + 1:])) if i + 1 < len(ups) else 1
        kern = 1 if stride == 1 else stride * 2 - stride % 2
        s += [(f"dec.noise_convs.{i}.weight", (chans[i], 1, kern), "noise"),
              (f"dec.noise_convs.{i}.bias", (chans[i],), "bias")]
    j = 0
    for i in range(len(ups)):
        for jj, (k, dil) in enumerate(zip(cfg.resblock_kernel_sizes, cfg.resblock_dilation_sizes)):
            if mrf:
                for m in range(len(dil)):
                    for c in ("conv1", "conv2"):
                        p = f"dec.mrfs.{i}.{jj}.layers.{m}.{c}"
                        s += _wn(p, (chans[i], chans[i], k), chans[i]) + [(f"{p}.bias", (chans[i],), "bias")]
            else:
                for c in ("convs1", "convs2"):
                    for m in range(len(dil)):
                        s += _wn(f"dec.resblocks.{j}.{c}.{m}", (chans[i], chans[i], k), chans[i])
                        s += [(f"dec.resblocks.{j}.{c}.{m}.bias", (chans[i],), "bias")]
            j += 1
    if mrf:
        s += _wn("dec.conv_post", (1, chans[-1], 7), 1) + [("dec.conv_post.bias", (1,), "bias")]
    else:
        s += [("dec.conv_post.weight", (1, chans[-1], 7), "post")]
    s += [("dec.cond.weight", (C0, cfg.gin_channels, 1), "conv"), ("dec.cond.bias", (C0,), "bias")]
    return s + _flow_emb_specs(cfg)


def _refinegan_specs(cfg: SynthConfig) -> List[Spec]:
    """RefineGANGenerator (generators/refinegan.py:258-392), built by Synthesizer with start_channels 16,
    upsample_initial_channel 512 and gin 256 fixed (synthesizers.py:99-107)."""
    s: List[Spec] = [("dec.m_source.merge.0.weight", (1, 1), "src_lin")]
    s += _wn("dec.pre_conv", (16, 1, 7), 16) + [("dec.pre_conv.bias", (16,), "bias")]
    ch = 16
    for i in range(len(cfg.upsample_rates)):
        s += _wn(f"dec.downsample_blocks.{i}", (2 * ch, ch, 7), 2 * ch) + [(f"dec.downsample_blocks.{i}.bias", (2 * ch,),
                                                                             "bias")]
        ch *= 2
    C = 512
    s += _wn("dec.mel_conv", (C // 2, cfg.inter_channels, 7), C // 2) + [("dec.mel_conv.bias", (C // 2,), "bias")]
    s += [("dec.cond.weight", (C // 2, 256, 1), "conv"), ("dec.cond.bias", (C // 2,), "bias")]
    for i in range(len(cfg.upsample_rates)):
        out, cin = C // 2, C + C // 4
        p = f"dec.upsample_conv_blocks.{i}"
        s += [(f"{p}.input_conv.weight", (out, cin, 7), "conv"), (f"{p}.input_conv.bias", (out,), "bias")]
        for j, k in enumerate((3, 7, 11)):
            q = f"{p}.blocks.{j}"
            s += [(f"{q}.0.weight", (out,), "adain")]
            for c in ("convs1", "convs2"):
                for m in range(3):
                    s += _wn(f"{q}.1.{c}.{m}", (out, out, k), out) + [(f"{q}.1.{c}.{m}.bias", (out,), "bias")]
            s += [(f"{q}.2.weight", (out,), "adain")]
        C = out
    s += _wn("dec.conv_post", (1, C, 7), 1)
    return s


def _flow_emb_specs(cfg: SynthConfig) -> List[Spec]:
    H, I = cfg.hidden_channels, cfg.inter_channels
    s: List[Spec] = []
    # flow (residuals.py:103-258, modules.py:5-117); odd indices are Flip
    half = I // 2
    for f in range(cfg.flow_n):
        p = f"flow.flows.{2 * f}"
        s += [(f"{p}.pre.weight", (H, half, 1), "conv"), (f"{p}.pre.bias", (H,), "bias")]
        s += _wn(f"{p}.enc.cond_layer", (2 * H * cfg.flow_layers, cfg.gin_channels, 1), 2 * H * cfg.flow_layers)
        s += [(f"{p}.enc.cond_layer.bias", (2 * H * cfg.flow_layers,), "bias")]
        for L in range(cfg.flow_layers):
            s += _wn(f"{p}.enc.in_layers.{L}", (2 * H, H, cfg.flow_kernel), 2 * H)
            s += [(f"{p}.enc.in_layers.{L}.bias", (2 * H,), "bias")]
            rs = H if L == cfg.flow_layers - 1 else 2 * H
            s += _wn(f"{p}.enc.res_skip_layers.{L}", (rs, H, 1), rs)
            s += [(f"{p}.enc.res_skip_layers.{L}.bias", (rs,), "bias")]
        s += [(f"{p}.post.weight", (half, H, 1), "flowpost"), (f"{p}.post.bias", (half,), "bias")]
    s += [("emb_g.weight", (cfg.spk_embed_dim, cfg.gin_channels), "embed")]
    return s


def hubert_specs(cfg: HubertConfig = HUBERT_BASE, with_final_proj: bool = True) -> List[Spec]:
    s: List[Spec] = []
    cin = 1
    for i, (c, k) in enumerate(zip(cfg.conv_dim, cfg.conv_kernel)):
        s += [(f"feature_extractor.conv_layers.{i}.conv.weight", (c, cin, k), "hconv")]
        cin = c
    s += [("feature_extractor.conv_layers.0.layer_norm.weight", (cfg.conv_dim[0],), "ln_g"),
          ("feature_extractor.conv_layers.0.layer_norm.bias", (cfg.conv_dim[0],), "ln_b")]
    D = cfg.hidden_size
    s += [("feature_projection.layer_norm.weight", (cfg.conv_dim[-1],), "ln_g"),
          ("feature_projection.layer_norm.bias", (cfg.conv_dim[-1],), "ln_b"),
          ("feature_projection.projection.weight", (D, cfg.conv_dim[-1]), "hlinear"),
          ("feature_projection.projection.bias", (D,), "bias")]
    G = cfg.num_conv_pos_embedding_groups
    K = cfg.num_conv_pos_embeddings
    s += [("encoder.pos_conv_embed.conv.weight_g", (1, 1, K), "wn_g"),
          ("encoder.pos_conv_embed.conv.weight_v", (D, D // G, K), "posconv"),
          ("encoder.pos_conv_embed.conv.bias", (D,), "bias"),
          ("encoder.layer_norm.weight", (D,), "ln_g"), ("encoder.layer_norm.bias", (D,), "ln_b")]
    for i in range(cfg.num_layers):
        p = f"encoder.layers.{i}"
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            s += [(f"{p}.attention.{n}.weight", (D, D), "hlinear"), (f"{p}.attention.{n}.bias", (D,), "bias")]
        s += [(f"{p}.layer_norm.weight", (D,), "ln_g"), (f"{p}.layer_norm.bias", (D,), "ln_b"),
              (f"{p}.feed_forward.intermediate_dense.weight", (cfg.intermediate_size, D), "hlinear"),
              (f"{p}.feed_forward.intermediate_dense.bias", (cfg.intermediate_size,), "bias"),
              (f"{p}.feed_forward.output_dense.weight", (D, cfg.intermediate_size), "hlinear"),
              (f"{p}.feed_forward.output_dense.bias", (D,), "bias"),
              (f"{p}.final_layer_norm.weight", (D,), "ln_g"), (f"{p}.final_layer_norm.bias", (D,), "ln_b")]
    if with_final_proj:
        s += [("final_proj.weight", (cfg.classifier_proj_size, D), "hlinear"),
              ("final_proj.bias", (cfg.classifier_proj_size,), "bias")]
    return s


def _conv_block_res(p: str, cin: int, cout: int) -> List[Spec]:
    s = [(f"{p}.conv.0.weight", (cout, cin, 3, 3), "conv2d")]
    s += _bn(f"{p}.conv.1", cout)
    s += [(f"{p}.conv.3.weight", (cout, cout, 3, 3), "conv2d")]
    s += _bn(f"{p}.conv.4", cout)
    if cin != cout:
        s += [(f"{p}.shortcut.weight", (cout, cin, 1, 1), "conv2d"), (f"{p}.shortcut.bias", (cout,), "bias")]
    return s


def _bn(p: str, c: int) -> List[Spec]:
    return [(f"{p}.weight", (c,), "bn_w"), (f"{p}.bias", (c,), "bn_b"),
            (f"{p}.running_mean", (c,), "bn_m"), (f"{p}.running_var", (c,), "bn_v"),
            (f"{p}.num_batches_tracked", (), "bn_n")]


def rmvpe_specs(cfg: RmvpeConfig = RMVPE_CFG) -> List[Spec]:
    s: List[Spec] = []
    s += _bn("unet.encoder.bn", 1)
    cin, cout = 1, cfg.en_out_channels
    for i in range(cfg.en_de_layers):
        for b in range(cfg.n_blocks):
            s += _conv_block_res(f"unet.encoder.layers.{i}.conv.{b}", cin if b == 0 else cout, cout)
        cin, cout = cout, cout * 2
    enc_out = cout  # out_channel of the encoder (= 512 for 16 * 2**5)
    ci = enc_out // 2
    for i in range(cfg.inter_layers):
        for b in range(cfg.n_blocks):
            s += _conv_block_res(f"unet.intermediate.layers.{i}.conv.{b}", ci if b == 0 else enc_out, enc_out)
        ci = enc_out
    c = enc_out
    for i in range(cfg.en_de_layers):
        co = c // 2
        s += [(f"unet.decoder.layers.{i}.conv1.0.weight", (c, co, 3, 3), "conv2d_t")]
        s += _bn(f"unet.decoder.layers.{i}.conv1.1", co)
        for b in range(cfg.n_blocks):
            s += _conv_block_res(f"unet.decoder.layers.{i}.conv2.{b}", co * 2 if b == 0 else co, co)
        c = co
    s += [("cnn.weight", (3, cfg.en_out_channels, 3, 3), "conv2d"), ("cnn.bias", (3,), "bias")]
    Hh = cfg.gru_hidden
    nin = 3 * cfg.n_mels
    for sfx in ("", "_reverse"):
        s += [(f"fc.0.gru.weight_ih_l0{sfx}", (3 * Hh, nin), "gru"),
              (f"fc.0.gru.weight_hh_l0{sfx}", (3 * Hh, Hh), "gru"),
              (f"fc.0.gru.bias_ih_l0{sfx}", (3 * Hh,), "gru"),
              (f"fc.0.gru.bias_hh_l0{sfx}", (3 * Hh,), "gru")]
    s += [("fc.1.weight", (cfg.n_class, 2 * Hh), "fc_out"), ("fc.1.bias", (cfg.n_class,), "fc_bias")]
    return s


# --------------------------------------------------------------------------- init
def _fan_in(shape) -> int:
    if len(shape) <= 1:
        return max(1, shape[0] if shape else 1)
    return int(np.prod(shape[1:]))


def _init(rng: np.random.Generator, shape, kind: str) -> np.ndarray:
    shape = tuple(shape)
    f32 = np.float32
    if kind == "bn_n":
        return np.array(0, dtype=np.int64)
    n = rng.standard_normal(shape)
    u = rng.random(shape)
    fan = _fan_in(shape)
    if kind in ("conv", "linear", "hconv", "conv2d"):
        w = n * (0.9 / np.sqrt(fan))
    elif kind == "hlinear":
        w = n * 0.03
    elif kind == "posconv":
        w = n * (0.5 / np.sqrt(fan))
    elif kind == "conv2d_t":  # ConvTranspose2d weight (C_in, C_out, kh, kw): fan = C_in * 9 / 4
        w = n * (1.2 / np.sqrt(shape[0] * shape[2] * shape[3] / 4.0))
    elif kind == "proj":
        w = n * (0.5 / np.sqrt(fan))
    elif kind == "flowpost":  # reference zero-inits post; random here so the flow is exercised
        w = n * (0.3 / np.sqrt(fan))
    elif kind == "noise":
        w = n * (1.0 / np.sqrt(fan))
    elif kind == "post":
        w = n * (1.5 / np.sqrt(fan))
    elif kind == "src_lin":
        w = 1.0 + 0.5 * n
    elif kind == "adain":  # reference init ones * 1e-4; larger here so the injected noise is exercised
        w = 0.1 + 0.05 * n
    elif kind == "bias":
        w = n * 0.05
    elif kind == "embed":
        w = n * 0.5
    elif kind == "relemb":
        w = n * (shape[-1] ** -0.5)
    elif kind in ("ln_g", "bn_w"):
        w = 1.0 + 0.1 * n
    elif kind in ("ln_b", "bn_b"):
        w = 0.1 * n
    elif kind == "bn_m":
        w = 0.2 * n
    elif kind == "bn_v":
        w = 0.5 + u
    elif kind == "gru":
        w = (2.0 * u - 1.0) / np.sqrt(RMVPE_CFG.gru_hidden)
    elif kind == "fc_out":
        w = n * (2.0 / np.sqrt(fan))
    elif kind == "fc_bias":
        w = -2.0 + 0.5 * n
    elif kind == "wn_g":
        w = None  # filled in by the caller from the matching weight_v norm
    else:
        raise ValueError(kind)
    return None if w is None else w.astype(f32)


def make_state(specs: List[Spec], seed: int) -> Dict[str, np.ndarray]:
    """Draw every tensor of ``specs`` from one PCG64 stream (deterministic order)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out: Dict[str, np.ndarray] = {}
    pending_g: Dict[str, Tuple[Tuple[int, ...], str]] = {}
    for name, shape, kind in specs:
        if kind == "wn_g":
            pending_g[name] = (tuple(shape), name)
            out[name] = np.zeros(shape, np.float32)  # placeholder, keeps key order
            continue
        out[name] = _init(rng, shape, kind)
    # weight_g = ||v|| * (1 + 0.1 * N) so the fused weight differs from v
    for gname, (gshape, _) in pending_g.items():
        v = out[gname[: -len("weight_g")] + "weight_v"].astype(np.float64)
        axes = tuple(i for i in range(v.ndim) if gshape[i] == 1)
        norm = np.sqrt((v * v).sum(axis=axes, keepdims=True))
        jitter = 1.0 + 0.1 * rng.standard_normal(gshape)
        out[gname] = (norm * jitter).astype(np.float32).reshape(gshape)
    return out


def synth_state(seed: int = 2, cfg: SynthConfig = SYNTH_48K_V2) -> Dict[str, np.ndarray]:
    return make_state(synth_specs(cfg), seed)


def hubert_state(seed: int = 4, cfg: HubertConfig = HUBERT_BASE) -> Dict[str, np.ndarray]:
    return make_state(hubert_specs(cfg), seed)


def rmvpe_state(seed: int = 5, cfg: RmvpeConfig = RMVPE_CFG) -> Dict[str, np.ndarray]:
    return make_state(rmvpe_specs(cfg), seed)


def crepe_state(kind: str = "full", seed: int = 11) -> Dict[str, np.ndarray]:
    """Random-init CREPE weights (torchcrepe names and layouts; rvc_mlx/lib/mlx/crepe.py:60-136 shapes). The
    classifier bias sits at -3 so the sigmoid outputs stay off saturation (median top-2 gap ~0.03: clear peaks,
    few near-ties in the argmax)."""
    caps = {"full": [1024, 128, 128, 128, 256, 512], "tiny": [128, 16, 16, 16, 32, 64]}[kind]
    rng = np.random.Generator(np.random.PCG64(seed))
    st: Dict[str, np.ndarray] = {}
    cin = 1
    for i, co in enumerate(caps):
        k = 512 if i == 0 else 64
        p = f"conv{i + 1}"
        st[p + ".weight"] = (rng.standard_normal((co, cin, k, 1)) / np.sqrt(cin * k)).astype(np.float32)
        st[p + ".bias"] = (0.05 * rng.standard_normal(co)).astype(np.float32)
        st[p + "_BN.weight"] = rng.uniform(0.8, 1.2, co).astype(np.float32)
        st[p + "_BN.bias"] = (0.1 * rng.standard_normal(co)).astype(np.float32)
        st[p + "_BN.running_mean"] = rng.uniform(0.2, 0.6, co).astype(np.float32)
        st[p + "_BN.running_var"] = rng.uniform(0.2, 0.6, co).astype(np.float32)
        cin = co
    feat = 4 * caps[-1]
    st["classifier.weight"] = (rng.standard_normal((360, feat)) / np.sqrt(feat)).astype(np.float32)
    st["classifier.bias"] = (rng.standard_normal(360) - 3.0).astype(np.float32)
    return st


# --------------------------------------------------------------------------- inputs
def speech_like(n: int, seed: int = 1, sr: int = 16000) -> np.ndarray:
    """Speech-like 16 kHz signal (SURVEY §8(d) C2 recipe): f0 contour 90-250 Hz with
    5 Hz vibrato, 8 harmonics through 3 formant resonators, ~20% unvoiced noise
    segments, peak 0.7. Returns float64 like soundfile/librosa loaders."""
    rng = np.random.Generator(np.random.PCG64(seed))
    t = np.arange(n) / sr
    seg = max(1, int(0.25 * sr))
    nseg = (n + seg - 1) // seg
    knots = 90.0 + 160.0 * rng.random(nseg + 1)
    f0 = np.interp(np.arange(n) / seg, np.arange(nseg + 1), knots)
    f0 = f0 * (1.0 + 0.02 * np.sin(2 * np.pi * 5.0 * t))
    phase = 2 * np.pi * np.cumsum(f0) / sr
    x = np.zeros(n)
    for h in range(1, 9):
        x += np.sin(h * phase) / h
    # three formant resonators (2-pole IIR)
    from scipy.signal import lfilter
    y = np.zeros(n)
    for fc, bw in ((700.0, 130.0), (1200.0, 70.0), (2600.0, 160.0)):
        r = np.exp(-np.pi * bw / sr)
        a = [1.0, -2.0 * r * np.cos(2 * np.pi * fc / sr), r * r]
        y += lfilter([1.0 - r], a, x)
    unv = rng.random(nseg) < 0.2
    mask = np.repeat(unv, seg)[:n]
    noise = rng.standard_normal(n) * 0.3
    y = np.where(mask, noise, y)
    y = y / (np.abs(y).max() + 1e-9) * 0.7
    return y.astype(np.float64)


def rmvpe_bench_audio(n: int = 80000, seed: int = 0) -> np.ndarray:
    """C1 input (benchmarks/benchmark_rmvpe.py:22-32): 0.3 sin 440 + 0.2 sin 880 + 0.1 N."""
    rng = np.random.Generator(np.random.PCG64(seed))
    t = np.linspace(0, n / 16000.0, n)
    x = 0.3 * np.sin(2 * np.pi * 440 * t) + 0.2 * np.sin(2 * np.pi * 880 * t) + 0.1 * rng.standard_normal(n)
    return x.astype(np.float32)


def f0_walk(B: int, T: int, seed: int = 3, unvoiced: float = 0.2) -> np.ndarray:
    """C3 f0: smooth random walk 100-400 Hz with ~20% unvoiced (zero) frames."""
    rng = np.random.Generator(np.random.PCG64(seed))
    steps = rng.standard_normal((B, T)) * 4.0
    f = 220.0 + np.cumsum(steps, axis=1)
    f = 100.0 + np.abs(((f - 100.0) % 600.0) - 300.0)
    blocks = (rng.random((B, (T + 19) // 20)) < unvoiced)
    mask = np.repeat(blocks, 20, axis=1)[:, :T]
    f[mask] = 0.0
    return f.astype(np.float32)
