"""Numerics of the fused ResBlock pair kernel (csrc/resblock_fused.hip, rvcx_resblock_pair) against an fp64
evaluation of the reference's ResBlock iteration (rvc/lib/algorithm/residuals.py:71-80):

    out = conv2(lrelu(conv1_d(lrelu(x)) + b1)) + b2 + x,   y = out | acc + out | (acc + out) / div

The fused kernel keeps the conv1 output in LDS and uses the exact 3-plane bf16 split arithmetic; the claim tested:
its error against fp64 stays at fp32 rounding level (< 2e-6 of max |out|), at both channel counts (32, 64), kernel size
and dilation the generators use, on ragged lengths, batches, tiny inputs (T below the halo) and each tile
configuration, and it agrees with the two-launch path (two rvcx_conv1d calls) to the same level.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

F = torch.nn.functional


def _ref(x, w1, b1, w2, b2, d):
    """fp64 ResBlock pair on [B][T][C] inputs (torch layout weights [C][C][k])."""
    k = w1.shape[2]
    xd = torch.from_numpy(x.astype(np.float64)).permute(0, 2, 1)
    t = F.conv1d(F.leaky_relu(xd, 0.1), torch.from_numpy(w1.astype(np.float64)),
                 torch.from_numpy(b1.astype(np.float64)), padding=d * (k - 1) // 2, dilation=d)
    t = F.leaky_relu(t, 0.1)
    o = F.conv1d(t, torch.from_numpy(w2.astype(np.float64)), torch.from_numpy(b2.astype(np.float64)),
                 padding=(k - 1) // 2) + xd
    return o.permute(0, 2, 1).numpy()


def _weights(rng, C, k):
    w1 = (rng.standard_normal((C, C, k)) / np.sqrt(C * k)).astype(np.float32)
    w2 = (rng.standard_normal((C, C, k)) / np.sqrt(C * k)).astype(np.float32)
    b1 = (0.1 * rng.standard_normal(C)).astype(np.float32)
    b2 = (0.1 * rng.standard_normal(C)).astype(np.float32)
    return w1, b1, w2, b2


CASES = [  # B, T, C, k, d, cfg
    (1, 5000, 32, 3, 1, 0),
    (1, 5003, 32, 7, 3, 0),
    (2, 4111, 32, 11, 5, 0),
    (1, 4000, 32, 11, 5, 0),
    (1, 3001, 64, 3, 1, 0),
    (2, 2999, 64, 11, 5, 0),
    (1, 3000, 64, 7, 3, 0),
    (1, 3000, 64, 11, 1, 0),
    (1, 17, 32, 11, 5, 0),    # T shorter than the halo: every tap row outside [0, T) is padding
    (3, 40, 64, 7, 3, 0),
]


@pytest.mark.parametrize("B,T,C,k,d,cfg", CASES)
def test_fused_pair_matches_fp64(engine, B, T, C, k, d, cfg):
    rng = np.random.Generator(np.random.PCG64(1000 * C + 10 * k + d + T))
    x = rng.standard_normal((B, T, C)).astype(np.float32)
    w1, b1, w2, b2 = _weights(rng, C, k)
    ref = _ref(x, w1, b1, w2, b2, d)
    y = engine.resblock_pair(x, w1, b1, w2, b2, d, cfg=cfg).cpu().numpy()
    assert y.shape == ref.shape
    err = float(np.abs(y - ref).max() / np.abs(ref).max())
    assert err < 2e-6, err


@pytest.mark.parametrize("mode", [1, 2])
def test_fused_pair_accumulate_modes(engine, mode):
    rng = np.random.Generator(np.random.PCG64(77 + mode))
    B, T, C, k, d = 2, 3000, 64, 7, 3
    x = rng.standard_normal((B, T, C)).astype(np.float32)
    acc = rng.standard_normal((B, T, C)).astype(np.float32)
    w1, b1, w2, b2 = _weights(rng, C, k)
    out = _ref(x, w1, b1, w2, b2, d)
    ref = acc.astype(np.float64) + out
    if mode == 2:
        ref = ref / 3.0
    y = engine.resblock_pair(x, w1, b1, w2, b2, d, acc=acc, acc_mode=mode, acc_div=3.0).cpu().numpy()
    err = float(np.abs(y - ref).max() / np.abs(ref).max())
    assert err < 2e-6, err


def test_fused_pair_matches_two_launch_path(engine):
    """The fused kernel against the unfused path's two contractions (rvcx_conv1d, split arithmetic) with the
    activations applied in between: same arithmetic, different summation order -> fp32-rounding agreement."""
    rng = np.random.Generator(np.random.PCG64(9))
    T, C, k, d = 6000, 32, 11, 5
    x = rng.standard_normal((1, T, C)).astype(np.float32)
    w1, b1, w2, b2 = _weights(rng, C, k)
    y = engine.resblock_pair(x, w1, b1, w2, b2, d).cpu().numpy()[0]
    xt = torch.nn.functional.leaky_relu(torch.from_numpy(x[0]), 0.1).numpy()
    t = engine.conv1d(xt, w1, b1, dilation=d, padding=d * (k - 1) // 2, math="split")
    t = torch.nn.functional.leaky_relu(t, 0.1)
    o = engine.conv1d(t, w2, b2, padding=(k - 1) // 2, math="split").cpu().numpy() + x[0]
    assert float(np.abs(y - o).max() / np.abs(o).max()) < 2e-6


@pytest.mark.parametrize("B,T,C,k,d,cfg", [c for c in CASES if c[5] == 0])
def test_fused_pair_fp16_arithmetic(engine, B, T, C, k, d, cfg):
    """cfg bits 4-5: the two-plane fp16 split (fp32-class: within 3x the exact split's bound) and the fp16 hi planes
    alone (the realtime reduced-precision mode: fp16 rounding)."""
    rng = np.random.Generator(np.random.PCG64(1000 * C + 10 * k + d + T))
    x = rng.standard_normal((B, T, C)).astype(np.float32)
    w1, b1, w2, b2 = _weights(rng, C, k)
    ref = _ref(x, w1, b1, w2, b2, d)
    e = {}
    for fmt in (1, 2):
        y = engine.resblock_pair(x, w1, b1, w2, b2, d, cfg=cfg | (fmt << 4)).cpu().numpy()
        e[fmt] = float(np.abs(y - ref).max() / np.abs(ref).max())
    assert e[1] < 6e-6, e
    assert e[2] < 3e-3, e
    print(f"\nfused pair B{B} T{T} C{C} k{k} d{d}: h16x2 {e[1]:.2e} f16 {e[2]:.2e}")


def test_fused_pair_rejects_unsupported(engine):
    from rvcx._lib import RvcxError

    rng = np.random.Generator(np.random.PCG64(3))
    x = rng.standard_normal((1, 100, 128)).astype(np.float32)
    w1, b1, w2, b2 = _weights(rng, 128, 3)
    with pytest.raises(RvcxError):
        engine.resblock_pair(x, w1, b1, w2, b2, 1)


@pytest.mark.parametrize("C,k,d", [(32, 11, 5), (64, 7, 3), (32, 3, 1)])
def test_fused_pair_fp16_per_channel_weight_spread(engine, C, k, d):
    """per-output-channel weight scales over 2^-24..1 (and one channel at 2^-20 of the tensor's
    largest) in both convs, the residual x and b2 scaled with conv2's channel so every output channel lives at its
    own magnitude. Each channel is held to the fp32-class bar relative to ITS OWN peak (the fp16 images carry one
    power-of-two scale per output channel, resblock_fused.hip k_rb_wsplit_h16)."""
    rng = np.random.Generator(np.random.PCG64(4242 + C + k))
    T = 3000
    x = rng.standard_normal((1, T, C)).astype(np.float32)
    w1, b1, w2, b2 = _weights(rng, C, k)
    # scales at or below 1 so the activations stay in the generator's range (the fp16 activation planes hold values
    # up to 2^20, split_bf16.h H16_XS); only the spread between channels matters to the per-channel weight scales
    s1 = np.exp2(rng.integers(-24, 1, size=C)).astype(np.float64)
    s2 = np.exp2(rng.integers(-24, 1, size=C)).astype(np.float64)
    s1[0], s2[0], s2[7] = 1.0, 1.0, 2.0 ** -20   # channel 7 at 2^-20 of the largest
    w1 = (w1 * s1[:, None, None]).astype(np.float32)
    b1 = (b1 * s1).astype(np.float32)
    w2 = (w2 * s2[:, None, None]).astype(np.float32)
    b2 = (b2 * s2).astype(np.float32)
    x = (x * s2[None, None, :]).astype(np.float32)
    ref = _ref(x, w1, b1, w2, b2, d)[0]
    peak = np.abs(ref).max(axis=0)
    for cfg, bar in ((0, 2e-6), (1 << 4, 6e-6)):
        y = engine.resblock_pair(x, w1, b1, w2, b2, d, cfg=cfg).cpu().numpy()[0]
        err = np.abs(y - ref).max(axis=0) / peak
        print(f"\nfused pair C{C} k{k} spread, cfg {cfg}: worst channel {err.max():.2e} (ch {int(err.argmax())}), "
              f"2^-20 channel {err[7]:.2e}")
        assert err.max() < bar, (cfg, float(err.max()), int(err.argmax()))


@pytest.mark.parametrize("B,T,d,mode", [(1, 5000, 1, 0), (2, 4111, 3, 1), (1, 3001, 5, 2), (1, 17, 5, 0), (3, 127, 1, 2),
                                        (1, 252, 3, 0), (1, 200003, 5, 1)])
def test_k3_pair_matches_streamed_form(engine, B, T, d, mode):
    """The k = 3, 32-channel fp16 pairs run on the weight-resident kernel (resblock_fused.hip k_rb_pair3: both convs'
    images in registers, the next tile's rows prefetched across the convs). Same tile, MFMA sequence and epilogue
    order as the streamed-weight kernel (cfg 1 forces it): bit-identical, on ragged lengths, batches, T below the halo,
    exact multiples of the 126-row tile, a long run of tiles per workgroup, every dilation and accumulate mode; and
    within the fp16 split's fp64 bar."""
    rng = np.random.Generator(np.random.PCG64(31 * T + d + mode))
    C, k = 32, 3
    x = rng.standard_normal((B, T, C)).astype(np.float32)
    acc = rng.standard_normal((B, T, C)).astype(np.float32) if mode else None
    w1, b1, w2, b2 = _weights(rng, C, k)
    y_res = engine.resblock_pair(x, w1, b1, w2, b2, d, acc=acc, acc_mode=mode, acc_div=3.0, cfg=1 << 4).cpu().numpy()
    y_str = engine.resblock_pair(x, w1, b1, w2, b2, d, acc=acc, acc_mode=mode, acc_div=3.0,
                                 cfg=(1 << 4) | 1).cpu().numpy()
    assert np.array_equal(y_res, y_str), float(np.abs(y_res - y_str).max())
    if T > 10000:
        return
    ref = _ref(x, w1, b1, w2, b2, d)
    if mode:
        ref = acc.astype(np.float64) + ref
        if mode == 2:
            ref = ref / 3.0
    err = float(np.abs(y_res - ref).max() / np.abs(ref).max())
    assert err < 6e-6, err
