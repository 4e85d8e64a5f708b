"""Oracle: SynthesizerTrnMs768NSFsid.infer (TextEncoder -> flow reverse -> HiFiGAN-NSF).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). Functional torch-CPU fp32
restatement over a fused-weight dict ``w`` (reference state-dict names).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

Tensor = torch.Tensor


def _t(w: Dict, k: str) -> Tensor:
    v = w[k]
    return v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))


def sequence_mask(length: Tensor, max_length: int) -> Tensor:
    """rvc/lib/algorithm/commons.py:106-117."""
    x = torch.arange(max_length, dtype=length.dtype)
    return x.unsqueeze(0) < length.unsqueeze(1)


def layer_norm_ct(x: Tensor, gamma: Tensor, beta: Tensor, eps: float = 1e-5) -> Tensor:
    """Channel LayerNorm on [B, C, T] (rvc/lib/algorithm/normalization.py:4-26)."""
    y = F.layer_norm(x.transpose(1, -1), (x.size(1),), gamma, beta, eps)
    return y.transpose(1, -1)


# ----------------------------------------------------------------- relative attention
def rel_attention(w, p: str, x: Tensor, attn_mask: Tensor, n_heads: int, window: int) -> Tensor:
    """MultiHeadAttention.forward with window_size relative keys/values
    (rvc/lib/algorithm/attentions.py:79-185). The pad/reshape skew of
    _relative_position_to_absolute_position (:158-169) and its inverse (:171-180)
    are pure index maps; they are written here as band gathers: the logit for
    key j of query i uses emb_rel_k[j - i + window] when |j - i| <= window, else 0."""
    q = F.conv1d(x, _t(w, p + ".conv_q.weight"), _t(w, p + ".conv_q.bias"))
    k = F.conv1d(x, _t(w, p + ".conv_k.weight"), _t(w, p + ".conv_k.bias"))
    v = F.conv1d(x, _t(w, p + ".conv_v.weight"), _t(w, p + ".conv_v.bias"))
    b, d, t = k.shape
    kc = d // n_heads
    q = q.view(b, n_heads, kc, t).transpose(2, 3)
    k = k.view(b, n_heads, kc, t).transpose(2, 3)
    v = v.view(b, n_heads, kc, t).transpose(2, 3)
    qs = q / math.sqrt(kc)
    scores = torch.matmul(qs, k.transpose(-2, -1))
    ek = _t(w, p + ".emb_rel_k")[0]  # [2w+1, kc]
    ev = _t(w, p + ".emb_rel_v")[0]
    rel = torch.matmul(qs, ek.t())  # [b,h,t,2w+1]; offset o = j - i + window
    nw = 2 * window + 1
    ii = torch.arange(t).view(t, 1)
    jj = torch.arange(t).view(1, t)
    off = jj - ii + window  # [t, t]
    valid = (off >= 0) & (off < nw)
    idx = torch.where(valid, off, torch.full_like(off, nw)).expand(b, n_heads, t, t).contiguous()
    rel_pad = torch.cat([rel, torch.zeros(b, n_heads, t, 1, dtype=rel.dtype)], dim=3)
    scores = scores + torch.gather(rel_pad, 3, idx)
    scores = scores.masked_fill(attn_mask == 0, -1e4)
    p_attn = torch.softmax(scores, dim=-1)
    out = torch.matmul(p_attn, v)
    # band of p_attn: pband[i, o] = p[i, i + o - window] (0 outside [0, t))
    jb = torch.arange(t).view(t, 1) + torch.arange(nw).view(1, nw) - window  # [t, 2w+1]
    vb = (jb >= 0) & (jb < t)
    pband = torch.gather(p_attn, 3, jb.clamp(0, t - 1).expand(b, n_heads, t, nw).contiguous())
    pband = torch.where(vb, pband, torch.zeros((), dtype=pband.dtype))
    out = out + torch.matmul(pband, ev)
    out = out.transpose(2, 3).contiguous().view(b, d, t)
    return F.conv1d(out, _t(w, p + ".conv_o.weight"), _t(w, p + ".conv_o.bias"))


def ffn(w, p: str, x: Tensor, x_mask: Tensor, ksize: int) -> Tensor:
    """FFN.forward, same padding, ReLU (rvc/lib/algorithm/attentions.py:221-243)."""
    pad = (ksize - 1) // 2
    y = F.conv1d(F.pad(x * x_mask, (pad, pad)), _t(w, p + ".conv_1.weight"), _t(w, p + ".conv_1.bias"))
    y = torch.relu(y)
    y = F.conv1d(F.pad(y * x_mask, (pad, pad)), _t(w, p + ".conv_2.weight"), _t(w, p + ".conv_2.bias"))
    return y * x_mask


def text_encoder(w, cfg, phone: Tensor, pitch: Optional[Tensor], lengths: Tensor):
    """TextEncoder.forward + Encoder.forward (rvc/lib/algorithm/encoders.py:11-144)."""
    H = cfg.hidden_channels
    x = F.linear(phone, _t(w, "enc_p.emb_phone.weight"), _t(w, "enc_p.emb_phone.bias"))
    if pitch is not None:
        x = x + F.embedding(pitch, _t(w, "enc_p.emb_pitch.weight"))
    x = x * math.sqrt(H)
    x = F.leaky_relu(x, 0.1)
    x = x.transpose(1, -1)
    x_mask = sequence_mask(lengths, x.size(2)).unsqueeze(1).to(x.dtype)
    attn_mask = x_mask.unsqueeze(2) * x_mask.unsqueeze(-1)
    x = x * x_mask
    for i in range(cfg.n_layers):
        y = rel_attention(w, f"enc_p.encoder.attn_layers.{i}", x, attn_mask, cfg.n_heads, cfg.window_size)
        x = layer_norm_ct(x + y, _t(w, f"enc_p.encoder.norm_layers_1.{i}.gamma"),
                          _t(w, f"enc_p.encoder.norm_layers_1.{i}.beta"))
        y = ffn(w, f"enc_p.encoder.ffn_layers.{i}", x, x_mask, cfg.kernel_size)
        x = layer_norm_ct(x + y, _t(w, f"enc_p.encoder.norm_layers_2.{i}.gamma"),
                          _t(w, f"enc_p.encoder.norm_layers_2.{i}.beta"))
    x = x * x_mask
    stats = F.conv1d(x, _t(w, "enc_p.proj.weight"), _t(w, "enc_p.proj.bias")) * x_mask
    m, logs = torch.split(stats, cfg.inter_channels, dim=1)
    return m, logs, x_mask


# ----------------------------------------------------------------- flow
def wavenet(w, p: str, x: Tensor, x_mask: Tensor, g: Tensor, cfg) -> Tensor:
    """WaveNet.forward (rvc/lib/algorithm/modules.py:78-109) with the
    fused_add_tanh_sigmoid_multiply gate (rvc/lib/algorithm/commons.py:88-103)."""
    H = cfg.hidden_channels
    output = torch.zeros_like(x)
    gc = F.conv1d(g, _t(w, p + ".cond_layer.weight"), _t(w, p + ".cond_layer.bias"))
    pad = (cfg.flow_kernel - 1) // 2
    for i in range(cfg.flow_layers):
        x_in = F.conv1d(x, _t(w, f"{p}.in_layers.{i}.weight"), _t(w, f"{p}.in_layers.{i}.bias"), padding=pad)
        g_l = gc[:, i * 2 * H:(i + 1) * 2 * H, :]
        in_act = x_in + g_l
        acts = torch.tanh(in_act[:, :H, :]) * torch.sigmoid(in_act[:, H:, :])
        rs = F.conv1d(acts, _t(w, f"{p}.res_skip_layers.{i}.weight"), _t(w, f"{p}.res_skip_layers.{i}.bias"))
        if i < cfg.flow_layers - 1:
            x = (x + rs[:, :H, :]) * x_mask
            output = output + rs[:, H:, :]
        else:
            output = output + rs
    return output * x_mask


def flow_reverse(w, cfg, x: Tensor, x_mask: Tensor, g: Tensor) -> Tensor:
    """ResidualCouplingBlock.forward(reverse=True): for flow in reversed(flows), i.e.
    Flip then coupling-layer reverse, n_flows times (rvc/lib/algorithm/residuals.py:151-164,
    Flip :87-100, ResidualCouplingLayer.forward mean_only :233-258)."""
    half = cfg.inter_channels // 2
    for f in reversed(range(cfg.flow_n)):
        x = torch.flip(x, [1])
        p = f"flow.flows.{2 * f}"
        x0, x1 = torch.split(x, [half, half], 1)
        h = F.conv1d(x0, _t(w, p + ".pre.weight"), _t(w, p + ".pre.bias")) * x_mask
        h = wavenet(w, p + ".enc", h, x_mask, g, cfg)
        m = F.conv1d(h, _t(w, p + ".post.weight"), _t(w, p + ".post.bias")) * x_mask
        logs = torch.zeros_like(m)
        x1 = (x1 - m) * torch.exp(-logs) * x_mask
        x = torch.cat([x0, x1], 1)
    return x


# ----------------------------------------------------------------- NSF generator
def sine_source(f0: Tensor, upp: int, sr: int, eps: Tensor, lin_w: Tensor, lin_b: Tensor) -> Tensor:
    """SineGenerator.forward (rvc/lib/algorithm/generators/hifigan.py:156-228) for
    harmonic_num=0, then SourceModuleHnNSF l_linear + tanh (generators/hifigan_nsf.py:48-52).
    ``eps`` is the injected N(0,1) draw of torch.randn_like at hifigan.py:223, shape [B, L*upp].
    Returns har [B, 1, L*upp]."""
    B, L = f0.shape
    f0 = f0.unsqueeze(-1)
    grid = torch.arange(1, upp + 1, dtype=f0.dtype)
    inc = (f0 / sr) * grid
    rem = torch.fmod(inc[:, :-1, -1:] + 0.5, 1.0) - 0.5
    cum = rem.cumsum(dim=1).fmod(1.0).to(f0.dtype)
    inc = inc + F.pad(cum, (0, 0, 1, 0), mode="constant")
    phase = inc.reshape(B, -1, 1)
    sine = torch.sin(2 * np.pi * phase) * 0.1
    uv = (f0 > 0.0).float()
    uv = F.interpolate(uv.transpose(2, 1), scale_factor=float(upp), mode="nearest").transpose(2, 1)
    amp = uv * 0.003 + (1 - uv) * (0.1 / 3)
    noise = amp * eps.reshape(B, -1, 1)
    merged = sine * uv + noise
    har = torch.tanh(F.linear(merged, lin_w, lin_b))
    return har.transpose(1, 2)


def resblock(w, p: str, x: Tensor, ksize: int, dilations) -> Tensor:
    """ResBlock.forward with x_mask=None (rvc/lib/algorithm/residuals.py:71-80)."""
    for m, d in enumerate(dilations):
        xr = x
        y = F.leaky_relu(x, 0.1)
        y = F.conv1d(y, _t(w, f"{p}.convs1.{m}.weight"), _t(w, f"{p}.convs1.{m}.bias"),
                     padding=(ksize * d - d) // 2, dilation=d)
        y = F.leaky_relu(y, 0.1)
        y = F.conv1d(y, _t(w, f"{p}.convs2.{m}.weight"), _t(w, f"{p}.convs2.{m}.bias"),
                     padding=(ksize - 1) // 2)
        x = y + xr
    return x


def nsf_generator(w, cfg, x: Tensor, f0: Tensor, g: Tensor, eps_src: Tensor) -> Tensor:
    """HiFiGANNSFGenerator.forward (rvc/lib/algorithm/generators/hifigan_nsf.py:173-212)."""
    upp = cfg.upp
    har = sine_source(f0, upp, cfg.sr, eps_src, _t(w, "dec.m_source.l_linear.weight"),
                      _t(w, "dec.m_source.l_linear.bias"))
    x = F.conv1d(x, _t(w, "dec.conv_pre.weight"), _t(w, "dec.conv_pre.bias"), padding=3)
    x = x + F.conv1d(g, _t(w, "dec.cond.weight"), _t(w, "dec.cond.bias"))
    ups = list(cfg.upsample_rates)
    nk = len(cfg.resblock_kernel_sizes)
    for i, (u, k) in enumerate(zip(ups, cfg.upsample_kernel_sizes)):
        x = F.leaky_relu(x, 0.1)
        pad = (k - u) // 2 if u % 2 == 0 else u // 2 + u % 2
        x = F.conv_transpose1d(x, _t(w, f"dec.ups.{i}.weight"), _t(w, f"dec.ups.{i}.bias"),
                               stride=u, padding=pad, output_padding=u % 2)
        stride = int(np.prod(ups[i + 1:])) if i + 1 < len(ups) else 1
        kern = 1 if stride == 1 else stride * 2 - stride % 2
        npad = 0 if stride == 1 else (kern - stride) // 2
        x = x + F.conv1d(har, _t(w, f"dec.noise_convs.{i}.weight"), _t(w, f"dec.noise_convs.{i}.bias"),
                         stride=stride, padding=npad)
        xs = 0
        for j in range(nk):
            xs = xs + resblock(w, f"dec.resblocks.{i * nk + j}", x, cfg.resblock_kernel_sizes[j],
                               cfg.resblock_dilation_sizes[j])
        x = xs / nk
    x = F.leaky_relu(x)
    x = torch.tanh(F.conv1d(x, _t(w, "dec.conv_post.weight"), None, padding=3))
    return x


def hifigan_generator(w, cfg, x: Tensor, g: Tensor) -> Tensor:
    """HiFiGANGenerator.forward (rvc/lib/algorithm/generators/hifigan.py:80-104): the decoder of models without
    pitch guidance -- no source module; ups padding (k - u) // 2 without output_padding (:46-58)."""
    x = F.conv1d(x, _t(w, "dec.conv_pre.weight"), _t(w, "dec.conv_pre.bias"), padding=3)
    x = x + F.conv1d(g, _t(w, "dec.cond.weight"), _t(w, "dec.cond.bias"))
    nk = len(cfg.resblock_kernel_sizes)
    for i, (u, k) in enumerate(zip(cfg.upsample_rates, cfg.upsample_kernel_sizes)):
        x = F.leaky_relu(x, 0.1)
        x = F.conv_transpose1d(x, _t(w, f"dec.ups.{i}.weight"), _t(w, f"dec.ups.{i}.bias"), stride=u,
                               padding=(k - u) // 2)
        xs = 0
        for j in range(nk):
            xs = xs + resblock(w, f"dec.resblocks.{i * nk + j}", x, cfg.resblock_kernel_sizes[j],
                               cfg.resblock_dilation_sizes[j])
        x = xs / nk
    x = F.leaky_relu(x)
    return torch.tanh(F.conv1d(x, _t(w, "dec.conv_post.weight"), None, padding=3))


def harmonic_source(f0_up: Tensor, sr: int, harmonics: int, eps: Tensor, rand_ini: Tensor, lin_w: Tensor,
                    lin_b: Optional[Tensor]) -> Tensor:
    """SineGenerator + merge of the MRF / RefineGAN decoders (generators/hifigan_mrf.py:120-230, refinegan.py:158-236)
    on the per-sample f0 [B, N, 1]; eps = randn_like(sine_waves) [B, N, H], rand_ini = torch.rand(B, H).
    torch.cumsum of float32 on CPU accumulates in double: written so here."""
    B, N, _ = f0_up.shape
    f0_buf = torch.zeros(B, N, harmonics, dtype=torch.float32)
    f0_buf[:, :, 0] = f0_up[:, :, 0]
    for idx in range(harmonics - 1):
        f0_buf[:, :, idx + 1] = f0_buf[:, :, 0] * (idx + 2)
    rad = (f0_buf / sr) % 1
    ini = rand_ini.clone()
    ini[:, 0] = 0
    rad[:, 0, :] = rad[:, 0, :] + ini
    tmp = torch.cumsum(rad.double(), 1).float() % 1
    idx = (tmp[:, 1:, :] - tmp[:, :-1, :]) < 0
    shift = torch.zeros_like(rad)
    shift[:, 1:, :] = idx * -1.0
    sines = torch.sin(torch.cumsum((rad + shift).double(), dim=1).float() * 2 * np.pi) * 0.1
    uv = (f0_up > 0).float()
    amp = uv * 0.003 + (1 - uv) * 0.1 / 3
    sw = sines * uv + amp * eps
    return torch.tanh(F.linear(sw, lin_w, lin_b))  # [B, N, 1]


def split_src_noise(eps_src: Tensor, B: int, N: int, harmonics: int):
    """The C-ABI's flat MRF / RefineGAN source noise: [B][N][H] randn then [B][H] initial phases."""
    e = eps_src.reshape(-1)
    return e[: B * N * harmonics].reshape(B, N, harmonics), e[B * N * harmonics:].reshape(B, harmonics)


def mrf_generator(w, cfg, x: Tensor, f0: Tensor, g: Tensor, eps_src: Tensor) -> Tensor:
    """HiFiGANMRFGenerator.forward (generators/hifigan_mrf.py:300-330): nearest f0 upsampling, 9-harmonic source,
    MRF blocks (= the NSF ResBlock dataflow), conv_post with bias."""
    upp = cfg.upp
    B = x.shape[0]
    f0_up = F.interpolate(f0[:, None, :].float(), scale_factor=float(upp), mode="nearest").transpose(-1, -2)
    eps, ini = split_src_noise(eps_src, B, f0_up.shape[1], 9)
    har = harmonic_source(f0_up, cfg.sr, 9, eps, ini, _t(w, "dec.m_source.l_linear.weight"),
                          _t(w, "dec.m_source.l_linear.bias")).transpose(-1, -2)
    x = F.conv1d(x, _t(w, "dec.conv_pre.weight"), _t(w, "dec.conv_pre.bias"), padding=3)
    x = x + F.conv1d(g, _t(w, "dec.cond.weight"), _t(w, "dec.cond.bias"))
    ups = list(cfg.upsample_rates)
    nk = len(cfg.resblock_kernel_sizes)
    for i, (u, k) in enumerate(zip(ups, cfg.upsample_kernel_sizes)):
        x = F.leaky_relu(x, 0.1)
        pad = (k - u) // 2 if u % 2 == 0 else u // 2 + u % 2
        x = F.conv_transpose1d(x, _t(w, f"dec.upsamples.{i}.weight"), _t(w, f"dec.upsamples.{i}.bias"), stride=u,
                               padding=pad, output_padding=u % 2)
        stride = int(np.prod(ups[i + 1:])) if i + 1 < len(ups) else 1
        kern = 1 if stride == 1 else stride * 2 - stride % 2
        npad = 0 if stride == 1 else (kern - stride) // 2
        x = x + F.conv1d(har, _t(w, f"dec.noise_convs.{i}.weight"), _t(w, f"dec.noise_convs.{i}.bias"),
                         stride=stride, padding=npad)
        xs = 0
        for j in range(nk):
            kk, dil = cfg.resblock_kernel_sizes[j], cfg.resblock_dilation_sizes[j]
            y = x
            for m, d in enumerate(dil):  # MRFLayer: x + conv2(lrelu(conv1(lrelu(x))))  (:35-56)
                p = f"dec.mrfs.{i}.{j}.layers.{m}"
                t = F.conv1d(F.leaky_relu(y, 0.1), _t(w, p + ".conv1.weight"), _t(w, p + ".conv1.bias"),
                             padding=(kk * d - d) // 2, dilation=d)
                t = F.conv1d(F.leaky_relu(t, 0.1), _t(w, p + ".conv2.weight"), _t(w, p + ".conv2.bias"),
                             padding=kk // 2)
                y = y + t
            xs = xs + y
        x = xs / nk
    x = F.leaky_relu(x)
    return torch.tanh(F.conv1d(x, _t(w, "dec.conv_post.weight"), _t(w, "dec.conv_post.bias"), padding=3))


REFINEGAN_C0 = 512  # RefineGANGenerator(upsample_initial_channel=512, start_channels=16): not from the config


def refinegan_noise_sizes(cfg, B: int, T: int):
    """Sizes of the RefineGAN decoder's RNG draws in call order (refinegan.py): the source's randn_like [B, N, 1],
    its torch.rand [B, 1], then per upsampling stage and ParallelResBlock branch the two AdaIN randn_like
    [B, C, T_stage] (in, out)."""
    N = T * cfg.upp
    sizes = [B * N, B]
    ch, t = REFINEGAN_C0, T
    for r in cfg.upsample_rates:
        ch, t = ch // 2, t * r
        sizes += [B * ch * t] * 6
    return sizes


def refinegan_generator(w, cfg, mel: Tensor, f0: Tensor, g: Tensor, eps_src: Tensor) -> Tensor:
    """RefineGANGenerator.forward (rvc/lib/algorithm/generators/refinegan.py:394-436): linear f0 upsampling,
    1-harmonic source, pre_conv, leaky(0.2) + torchaudio kaiser-sinc resampling + conv per downsampling stage,
    mel_conv + cond, then per upsampling stage leaky -> linear x rate -> concat the matching down branch ->
    ParallelResBlock (input_conv, 3 x [AdaIN -> ResBlock(slope 0.2) -> AdaIN], mean) -> leaky -> conv_post -> tanh.
    eps_src: the flat C-ABI layout of every draw (refinegan_noise_sizes)."""
    from oracle.realtime import functional_resample

    B, _, T = mel.shape
    upp = cfg.upp
    ups = list(cfg.upsample_rates)
    sizes = refinegan_noise_sizes(cfg, B, T)
    parts = list(torch.split(eps_src.reshape(-1), sizes))
    N = T * upp
    f0u = F.interpolate(f0.float().unsqueeze(1), size=N, mode="linear")  # [B, 1, N]
    eps, ini = parts[0].reshape(B, N, 1), parts[1].reshape(B, 1)
    har = harmonic_source(f0u.transpose(1, 2), cfg.sr, 1, eps, ini, _t(w, "dec.m_source.merge.0.weight"),
                          None).transpose(1, 2)
    x = F.conv1d(har, _t(w, "dec.pre_conv.weight"), _t(w, "dec.pre_conv.bias"), padding=3)
    downs = []
    size = upp
    for i in range(len(ups)):
        new_size = int(size / ups[-i - 1])
        x = F.leaky_relu(x, 0.2)
        downs.append(x)
        x = functional_resample(x.contiguous(), int(T * size), int(T * new_size), lowpass_filter_width=64,
                                rolloff=0.9475937167399596, resampling_method="sinc_interp_kaiser",
                                beta=14.769656459379492)
        x = F.conv1d(x, _t(w, f"dec.downsample_blocks.{i}.weight"), _t(w, f"dec.downsample_blocks.{i}.bias"),
                     padding=3)
        size = new_size
    m = F.conv1d(mel, _t(w, "dec.mel_conv.weight"), _t(w, "dec.mel_conv.bias"), padding=3)
    m = m + F.conv1d(g, _t(w, "dec.cond.weight"), _t(w, "dec.cond.bias"))
    x = torch.cat([m, x], dim=1)
    k = 2
    for i, (r, down) in enumerate(zip(ups, reversed(downs))):
        x = F.leaky_relu(x, 0.2)
        x = F.interpolate(x, scale_factor=float(r), mode="linear")
        x = torch.cat([x, down], dim=1)
        p = f"dec.upsample_conv_blocks.{i}"
        x = F.conv1d(x, _t(w, p + ".input_conv.weight"), _t(w, p + ".input_conv.bias"), padding=3)
        outs = []
        for j, (ks, dil) in enumerate(zip((3, 7, 11), (1, 3, 5))):
            q = f"{p}.blocks.{j}"
            y = F.leaky_relu(x + parts[k].reshape(x.shape) * _t(w, q + ".0.weight")[None, :, None], 0.2)
            k += 1
            for mm, d in enumerate((1, 3, 5)):  # refinegan.py ResBlock (:49-61)
                t = F.conv1d(F.leaky_relu(y, 0.2), _t(w, f"{q}.1.convs1.{mm}.weight"), _t(w, f"{q}.1.convs1.{mm}.bias"),
                             padding=(ks * d - d) // 2, dilation=d)
                t = F.conv1d(F.leaky_relu(t, 0.2), _t(w, f"{q}.1.convs2.{mm}.weight"),
                             _t(w, f"{q}.1.convs2.{mm}.bias"), padding=(ks - 1) // 2)
                y = t + y
            y = F.leaky_relu(y + parts[k].reshape(y.shape) * _t(w, q + ".2.weight")[None, :, None], 0.2)
            k += 1
            outs.append(y)
        x = torch.stack(outs, dim=0).mean(dim=0)
    x = F.leaky_relu(x, 0.2)
    return torch.tanh(F.conv1d(x, _t(w, "dec.conv_post.weight"), None, padding=3))


def decoder(w, cfg, x: Tensor, f0, g: Tensor, eps_src) -> Tensor:
    """The decoder Synthesizer selects (synthesizers.py:84-139)."""
    if not getattr(cfg, "use_f0", True):
        return hifigan_generator(w, cfg, x, g)
    voc = getattr(cfg, "vocoder", "HiFi-GAN")
    if voc == "MRF HiFi-GAN":
        return mrf_generator(w, cfg, x, f0, g, eps_src)
    if voc == "HiFi-GAN":
        return nsf_generator(w, cfg, x, f0, g, eps_src)
    if voc == "RefineGAN":
        return refinegan_generator(w, cfg, x, f0, g, eps_src)
    raise ValueError(voc)


def synth_infer(w, cfg, phone: Tensor, lengths: Tensor, pitch: Tensor, nsff0: Tensor, sid: Tensor,
                eps_z: Tensor, eps_src: Tensor, rate=None):
    """Synthesizer.infer (rvc/lib/algorithm/synthesizers.py:206-243) with the two RNG draws
    injected: eps_z for randn_like at :228, eps_src for hifigan.py:223 (over the frames the decoder runs on).
    rate (:230-234): z_p, x_mask and nsff0 from frame int(T * (1 - rate)) on.
    Returns (o [B,1,T'*upp], x_mask, (z, z_p, m_p, logs_p))."""
    with torch.no_grad():
        g = F.embedding(sid, _t(w, "emb_g.weight")).unsqueeze(-1)
        m_p, logs_p, x_mask = text_encoder(w, cfg, phone, pitch if getattr(cfg, "use_f0", True) else None, lengths)
        z_p = (m_p + torch.exp(logs_p) * eps_z * 0.66666) * x_mask
        if rate is not None:
            head = int(z_p.shape[2] * (1.0 - float(rate)))
            z_p, x_mask = z_p[:, :, head:], x_mask[:, :, head:]
            if getattr(cfg, "use_f0", True) and nsff0 is not None:
                nsff0 = nsff0[:, head:]
        z = flow_reverse(w, cfg, z_p, x_mask, g)
        o = decoder(w, cfg, z * x_mask, nsff0, g, eps_src)  # synthesizers.py:233-239
    return o, x_mask, (z, z_p, m_p, logs_p)


def dec_only(w, cfg, z: Tensor, nsff0: Tensor, sid: Tensor, eps_src: Tensor) -> Tensor:
    """Generator alone (config C3): HiFiGAN-NSF on latent z with speaker conditioning."""
    with torch.no_grad():
        g = F.embedding(sid, _t(w, "emb_g.weight")).unsqueeze(-1)
        return decoder(w, cfg, z, nsff0, g, eps_src)
