"""The fused attention kernel (csrc/flash_attn.hip) against fp64, through rvcx_flash_attention.

Both uses of the path: HuBERT's plain attention (modeling_hubert.py HubertAttention, dk 64) and the TextEncoder's
windowed relative-position attention with a key mask (rvc/lib/algorithm/attentions.py:79-185, dk 96, window 10).
The kernel runs the products in the two-plane fp16 split with q, k, v and the relative tables at a fixed 2^-4 scale
(K / V from fragment images, k_kv_split16). The bar is the one the contraction kernels meet
(tests/test_gpu_conv_math.py): every output element within fp32 rounding of its own magnitude sum_j p_ij |v_jd|
(+ the relative band's): at most 4x the error of torch's own fp32 evaluation of the same inputs, and below 1e-5 for
unit-scale operands. Covered: unit-scale operands, operands spread element-wise over 2^+-4 (larger logits, sharper
softmax), and V head dimensions spread over 2^+-12 with one at 2^-20 of the largest (the K / V
images' dynamic range).
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(qkv, nh, qscale, rel_k, rel_v, window, mask, dtype):
    x = torch.from_numpy(qkv).to(dtype)
    B, T, H3 = x.shape
    H = H3 // 3
    dk = H // nh
    q, k, v = (x[..., i * H:(i + 1) * H].reshape(B, T, nh, dk).transpose(1, 2) for i in range(3))
    qs = q * qscale
    s = qs @ k.transpose(-1, -2)
    nw = 2 * window + 1
    if rel_k is not None:
        rk = torch.from_numpy(rel_k).to(dtype)
        rel = qs @ rk.T  # [B, nh, T, nw], offset o = j - i + window
        ii, jj = torch.arange(T).view(T, 1), torch.arange(T).view(1, T)
        off = jj - ii + window
        valid = (off >= 0) & (off < nw)
        idx = torch.where(valid, off, torch.full_like(off, nw)).expand(B, nh, T, T).contiguous()
        s = s + torch.gather(torch.cat([rel, torch.zeros(B, nh, T, 1, dtype=dtype)], dim=3), 3, idx)
    if mask is not None:
        m = torch.from_numpy(mask).to(dtype)
        am = m[:, None, :, None] * m[:, None, None, :]
        s = s.masked_fill(am == 0, -1e4)
    p = torch.softmax(s, dim=-1)
    out = p @ v
    mag = p.abs() @ v.abs()
    if rel_v is not None:
        rv = torch.from_numpy(rel_v).to(dtype)
        jb = torch.arange(T).view(T, 1) + torch.arange(nw).view(1, nw) - window
        vb = (jb >= 0) & (jb < T)
        pb = torch.gather(p, 3, jb.clamp(0, T - 1).expand(B, nh, T, nw).contiguous())
        pb = torch.where(vb, pb, torch.zeros((), dtype=dtype))
        out = out + pb @ rv
        mag = mag + pb.abs() @ rv.abs()
    return (out.transpose(1, 2).reshape(B, T, H).numpy(), mag.transpose(1, 2).reshape(B, T, H).numpy())


CASES = [  # name, B, T, n_heads, dk, window, lengths (None: no mask), operand spread, V column spread
    ("hubert", 1, 775, 12, 64, 0, None, 0, 0),
    ("hubert spread", 1, 775, 12, 64, 0, None, 4, 0),
    ("hubert vcols", 1, 775, 12, 64, 0, None, 0, 12),
    ("hubert C4", 1, 1599, 12, 64, 0, None, 0, 0),
    ("te", 2, 300, 2, 96, 10, (300, 211), 0, 0),
    ("te spread", 2, 300, 2, 96, 10, (300, 211), 4, 0),
    ("te vcols", 1, 1550, 2, 96, 10, (1550,), 0, 12),
]


@pytest.mark.parametrize("name,B,T,nh,dk,window,lengths,spread,vcols", CASES)
def test_flash_attention_is_fp32_accurate(engine, name, B, T, nh, dk, window, lengths, spread, vcols):
    rng = np.random.Generator(np.random.PCG64(T * 13 + nh * 7 + dk + spread + vcols))
    H = nh * dk
    qkv = rng.standard_normal((B, T, 3 * H)).astype(np.float32)
    if spread:
        qkv *= np.exp2(rng.integers(-spread, spread + 1, size=qkv.shape)).astype(np.float32)
    if vcols:
        cs = np.exp2(rng.integers(-vcols, vcols + 1, size=H)).astype(np.float32)
        cs[0], cs[dk + 3] = 2.0 ** 12, 2.0 ** -8  # one head dimension at 2^-20 of the largest
        qkv[..., 2 * H:] *= cs
    rel_k = rel_v = mask = None
    if window:
        rel_k = (rng.standard_normal((2 * window + 1, dk)) / math.sqrt(dk)).astype(np.float32)
        rel_v = (rng.standard_normal((2 * window + 1, dk)) / math.sqrt(dk)).astype(np.float32)
    if lengths is not None:
        mask = (np.arange(T)[None, :] < np.array(lengths)[:, None]).astype(np.float32)
    qscale = dk ** -0.5
    y = engine.flash_attention(qkv, nh, qscale, rel_k, rel_v, window, mask).cpu().numpy()
    r64, mag = _ref(qkv, nh, qscale, rel_k, rel_v, window, mask, torch.float64)
    r32, _ = _ref(qkv, nh, qscale, rel_k, rel_v, window, mask, torch.float32)
    rows = np.ones((B, T), bool) if mask is None else mask > 0  # padded query rows are discarded downstream
    den = mag + 1e-300
    err = float(np.max((np.abs(y - r64) / den)[rows]))
    err32 = float(np.max((np.abs(r32 - r64) / den)[rows]))
    print(f"\nattention {name}: device {err:.2e}, torch fp32 {err32:.2e}")
    assert np.isfinite(y[rows]).all()
    # spread operands give logits of hundreds, where the softmax amplifies fp32's own rounding of the logits (torch's
    # fp32 evaluation errs ~1e-4 there): the bar is then relative to it alone
    assert err <= 4.0 * err32 + 1e-7, (err, err32)
    if not spread:
        assert err < 1e-5, (err, err32)
