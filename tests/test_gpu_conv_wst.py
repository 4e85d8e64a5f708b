"""The weight-stationary conv kernel (csrc/conv_wst.hip) through rvcx_conv1d_gen.

It takes the generator's short convs (k = 3 ResBlock convs at 64 / 128 channels, residuals.py:71-80; the two-tap
ConvTranspose phases of the last upsample stages, hifigan_nsf.py:184-199). Its claim is bit-identity with the
weight-streamed kernel (same split image, same MFMA products in the same order, same epilogue order), so the test
compares the two element for element, on ragged lengths (one partial tile, tile boundaries, many tiles per
persistent workgroup), every epilogue form the generator uses (convs1: leaky ReLU; convs2: residual, stored /
accumulated / accumulated and divided by the ResBlock count), the dilations 1 / 3 / 5 and per-column weight spread
(the split image's per-column scales). It also holds both to fp64 at the fp32 bar the other contraction kernels meet
(tests/test_gpu_conv_math.py: every element within 1e-6 of its own magnitude sum).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [  # T, C (= N), taps, dil, epilogue, weight spread ("conv2" / "acc" / "accdiv": no pre-activation, as convs2
    # reads convs1's activated output; "conv1" / "up": the leaky-ReLU pre-activation)
    (1000, 128, 3, 1, "conv1", 0),
    (1000, 128, 3, 3, "conv2", 0),
    (20011, 128, 3, 5, "acc", 0),
    (20011, 128, 3, 1, "accdiv", "ch12"),
    (65, 128, 3, 3, "conv1", "dead20"),
    (37, 64, 3, 5, "conv2", 0),
    (64, 64, 3, 1, "conv1", 0),
    (20011, 64, 3, 3, "conv1", "ch12"),
    (20011, 64, 3, 5, "accdiv", 0),
    (4097, 64, 3, 1, "acc", "dead20"),
    (20011, 128, 2, 1, "up", 0),
    (1, 128, 2, 1, "up", 0),
    (20011, 64, 2, 1, "up", "ch12"),
    (150001, 128, 3, 3, "conv2", 0),   # ~9 tiles per persistent workgroup (exactness only)
    (300007, 64, 3, 5, "acc", 0),
    (5003, 128, 3, 1, "prer", "ch12"),  # pre-activation + residual + accumulate (every epilogue bit at once)
    (5003, 64, 3, 1, "prer", 0),
]


def _wspread(rng, N, kind):
    if kind == "ch12":
        s = np.exp2(rng.integers(-12, 13, size=N)).astype(np.float64)
        s[0] = 2.0 ** 12
        s[5] = 2.0 ** -8
    else:
        s = np.ones(N)
        s[3] = 2.0 ** -20
    return s


def _lrelu(v, s):
    return np.where(v > 0, v, v * s)


@pytest.mark.parametrize("T,C,K,dil,epi,wsp", CASES)
def test_wst_matches_wsb_and_fp64(engine, T, C, K, dil, epi, wsp):
    rng = np.random.Generator(np.random.PCG64(T * 3 + C + K * 11 + dil))
    x = rng.standard_normal((T, C)).astype(np.float32)
    w = (rng.standard_normal((C, C, K)) / np.sqrt(C * K)).astype(np.float32)
    b = rng.standard_normal(C).astype(np.float32) * 0.1
    if wsp:
        cs = _wspread(rng, C, wsp)
        w = (w * cs[:, None, None]).astype(np.float32)
        b = (b * cs).astype(np.float32)
    pad = dil * (K - 1) // 2 if K == 3 else 1
    T_out = T + 2 * pad - dil * (K - 1)
    slope = 0.1 if epi == "conv1" else None
    res = rng.standard_normal((T_out, C)).astype(np.float32) if epi in ("conv2", "acc", "accdiv", "prer") else None
    acc = rng.standard_normal((T_out, C)).astype(np.float32) if epi in ("acc", "accdiv", "prer") else None
    mode = {"acc": 1, "accdiv": 2, "prer": 2}.get(epi, 0)
    div = 3.0 if epi in ("accdiv", "prer") else 1.0
    pre = 0.1 if epi in ("conv1", "up", "prer") else None
    kw = dict(bias=b, dilation=dil, padding=pad, pre_slope=pre, slope=slope, res=res, acc=acc, acc_mode=mode,
              acc_div=div)
    y_wst = engine.conv1d_gen(x, w, kernel="wst", **kw).cpu().numpy()
    y_wsb = engine.conv1d_gen(x, w, kernel="wsb", **kw).cpu().numpy()
    y_pol = engine.conv1d_gen(x, w, kernel="policy", **kw).cpu().numpy()
    assert y_wst.shape == (T_out, C)
    assert np.array_equal(y_wst, y_wsb), float(np.max(np.abs(y_wst - y_wsb)))
    assert np.array_equal(y_pol, y_wst)
    if T > 25000:
        return
    xd = torch.from_numpy(_lrelu(x.astype(np.float64), pre) if pre is not None else x.astype(np.float64)).T[None]
    wd = torch.from_numpy(w.astype(np.float64))
    v = torch.nn.functional.conv1d(xd, wd, None, padding=pad, dilation=dil)[0].T.numpy()
    mag = torch.nn.functional.conv1d(xd.abs(), wd.abs(), None, padding=pad, dilation=dil)[0].T.numpy()
    v = v + b.astype(np.float64)
    mag = mag + np.abs(b.astype(np.float64))
    if slope is not None:
        v = _lrelu(v, slope)
    if res is not None:
        v = v + res
        mag = mag + np.abs(res)
    if acc is not None:
        v = (acc + v) / div
        mag = (np.abs(acc) + mag) / div
    err = float(np.max(np.abs(y_wst - v) / (mag + 1e-300)))
    print(f"\nwst T{T} C{C} k{K} d{dil} {epi} {wsp}: fp64 err {err:.2e}")
    assert err < 1e-6, err


def test_wst_rejects_other_shapes(engine):
    """Shapes outside the kernel's instantiations are refused with RVCX_E_SHAPE, not run on another kernel."""
    x = np.zeros((100, 32), np.float32)
    w = np.zeros((32, 32, 3), np.float32)
    with pytest.raises(RuntimeError):
        engine.conv1d_gen(x, w, padding=1, kernel="wst")
    x = np.zeros((100, 128), np.float32)
    w = np.zeros((128, 128, 7), np.float32)
    with pytest.raises(RuntimeError):
        engine.conv1d_gen(x, w, padding=3, kernel="wst")
