"""Numerics of the contraction kernels against fp64 (rvcx_conv1d, both arithmetic modes).

The default "split" mode computes every fp32 contraction on bf16 MFMA through an exact 3-way split of both
operands (csrc/conv_emu.hip); "f32" is the fp32-input MFMA, an exact fp32 fma chain. The claim tested here: the
split mode is fp32 accurate -- its error against an fp64 evaluation of the same fp32 inputs is at most the native
fp32 path's error (both well under 1e-6 of sum |x w|), on every shape class the path runs (halo convs with
dilation, strided convs, plain GEMMs, ragged channel counts, split-K), including inputs spanning many binades.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [  # T, C_in, N, taps, dil, stride, scale_spread (activations), weight spread (see _wspread)
    (3000, 128, 128, 11, 5, 1, 0, 0),
    (2000, 64, 64, 3, 1, 1, 0, 0),
    (4000, 32, 32, 7, 3, 1, 0, 0),
    (1550, 192, 768, 3, 1, 1, 0, 0),
    (775, 768, 2304, 1, 1, 1, 0, 0),       # HuBERT qkv (GEMM pipeline)
    (150, 3072, 768, 1, 1, 1, 0, 0),       # long contraction: split-K
    (5000, 512, 512, 3, 1, 2, 0, 0),       # HuBERT strided feature conv
    (1000, 37, 45, 5, 2, 1, 0, 0),         # ragged channels (scalar paths)
    (3000, 256, 200, 7, 3, 1, 0, 0),       # N not a multiple of the tile (weight-streamed: padded columns)
    (2500, 64, 32, 11, 5, 1, 4, 0),        # narrow N (weight-streamed 256 x 32 tile), spread operands
    (2000, 128, 64, 7, 1, 1, 12, 0),       # operands spread over 2^+-12
    (196, 512, 512, 9, 1, 1, 0, 0),        # the U-Net's deepest 1-D analogue: 9 taps, few rows, long K (split-K)
    (1599, 768, 3072, 1, 1, 1, 0, 0),      # HuBERT FFN at the 30 s (C4) length
    # weight spread (trained weight-norm checkpoints fuse a per-output-channel g, so a dead or
    # near-dead channel sits orders of magnitude below the tensor's largest): per-column scales over 2^+-12 and one
    # column at 2^-20 of the tensor max, on the weight-streamed, gather-streamed and split-K shapes
    (3000, 128, 128, 11, 5, 1, 0, "ch12"),
    (3000, 128, 128, 7, 1, 1, 4, "dead20"),
    (2000, 64, 64, 3, 1, 1, 0, "ch12"),
    (3000, 256, 200, 7, 3, 1, 0, "ch12"),
    (775, 768, 2304, 1, 1, 1, 0, "ch12"),
    (196, 512, 512, 9, 1, 1, 0, "dead20"),
    (1550, 192, 768, 3, 1, 1, 0, "ch12"),
]


def _ref(x, w, bias, dil, pad, stride):
    xd = torch.from_numpy(x.astype(np.float64)).T[None]
    wd = torch.from_numpy(w.astype(np.float64))
    y = torch.nn.functional.conv1d(xd, wd, torch.from_numpy(bias.astype(np.float64)), stride=stride, padding=pad,
                                   dilation=dil)[0].T
    ya = torch.nn.functional.conv1d(xd.abs(), wd.abs(), None, stride=stride, padding=pad, dilation=dil)[0].T
    return y.numpy(), ya.numpy()


def _wspread(rng, N, kind):
    """Per-output-column weight scales (powers of two, so the fp64 reference sees exactly the scaled weights): "ch12"
    spreads the columns over 2^+-12 and puts one at 2^-20 of the largest; "dead20" leaves every column at 1 but
    one at 2^-20."""
    if kind == "ch12":
        s = np.exp2(rng.integers(-12, 13, size=N)).astype(np.float64)
        s[0] = 2.0 ** 12
        s[min(5, N - 1)] = 2.0 ** -8  # 2^-20 of the max
    else:
        s = np.ones(N)
        s[min(3, N - 1)] = 2.0 ** -20
    return s


@pytest.mark.parametrize("T,C,N,K,dil,stride,spread,wsp", CASES)
def test_split_math_is_fp32_accurate(engine, T, C, N, K, dil, stride, spread, wsp):
    """Every arithmetic against fp64, per output element relative to its own sum |x w| (+ |bias|): a column whose
    weights are 2^-20 of the tensor's largest is held to the same bar as the largest one."""
    rng = np.random.Generator(np.random.PCG64(T * 7 + C))
    x = rng.standard_normal((T, C)).astype(np.float32)
    w = (rng.standard_normal((N, C, K)) / np.sqrt(C * K)).astype(np.float32)
    if spread:
        x *= np.exp2(rng.integers(-spread, spread + 1, size=x.shape)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    if wsp:
        cs = _wspread(rng, N, wsp)
        w = (w * cs[:, None, None]).astype(np.float32)
        bias = (bias * cs).astype(np.float32)
    pad = dil * (K - 1) // 2
    ref, mag = _ref(x, w, bias, dil, pad, stride)
    errs = {}
    # "wsb": the same split arithmetic on the weight-streamed kernel (conv_wsb.hip), where the shape allows it
    wsb = stride == 1 and C % 32 == 0 and (K - 1) * dil <= 64
    gs = C % 32 == 0  # "gs": the gather-streamed kernel (conv_gs.hip: per-step A gather, split-K by the size policy)
    for mode in ("f32", "split") + (("wsb", "h16", "f16") if wsb else ()) + (("gs", "gs_h16") if gs else ()):
        y = engine.conv1d(x, w, bias, dilation=dil, padding=pad, stride=stride, math=mode).cpu().numpy()
        assert y.shape == ref.shape
        errs[mode] = float(np.max(np.abs(y - ref) / (mag + np.abs(bias) + 1e-300)))
    # both within fp32 rounding of the contraction; the split mode no worse than native fp32 (+ slack for the
    # different summation order of equally accurate evaluations)
    assert errs["f32"] < 1e-6, errs
    assert errs["split"] < 1e-6, errs
    assert errs["split"] <= 1.5 * errs["f32"] + 1e-8, errs
    if wsb:  # one unsplit accumulation chain per output (no split-K partial sums): the fp32 bound only
        assert errs["wsb"] < 1e-6, errs
        # the two-plane fp16 split (22-bit operands, rvcx_set_conv_math mode 3): within the same fp32 bound and at
        # most 4x the native fp32 path's error; the reduced-precision hi planes alone: fp16 rounding (2^-11)
        assert errs["h16"] < 1e-6 and errs["h16"] <= 4.0 * errs["f32"] + 1e-8, errs
        assert errs["f16"] < 2e-3, errs
    print(f"\n{T}x{C}->{N} k{K}: " + " ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    if gs:
        assert errs["gs"] < 1e-6, errs
        assert errs["gs_h16"] < 1e-6 and errs["gs_h16"] <= 4.0 * errs["f32"] + 1e-8, errs


def test_context_math_mode_switch(engine):
    rng = np.random.Generator(np.random.PCG64(5))
    x = rng.standard_normal((512, 64)).astype(np.float32)
    w = rng.standard_normal((64, 64, 3)).astype(np.float32)
    a = engine.conv1d(x, w, None, padding=1, math="f32").cpu().numpy()
    b = engine.conv1d(x, w, None, padding=1, math="split").cpu().numpy()
    engine.set_conv_math("f32")
    try:
        c = engine.conv1d(x, w, None, padding=1).cpu().numpy()
    finally:
        engine.set_conv_math("default")
    assert np.array_equal(a, c)  # the context mode reaches the kernel
    assert not np.array_equal(a, b) and np.allclose(a, b, rtol=1e-5, atol=1e-4)


SMALL2D = [  # H, W, C_in, N, spread, weight spread: the RMVPE U-Net's few-channel 3x3 convs (csrc/conv2d_small.hip)
    (64, 128, 16, 16, 0, 0),   # level 0
    (48, 128, 16, 32, 0, 0),   # level 0 -> 1 channels
    (40, 64, 32, 32, 0, 0),    # level 1
    (40, 64, 32, 16, 0, 0),    # decoder 32 -> 16
    (33, 128, 16, 3, 0, 0),    # the 16 -> 3 output conv, ragged rows
    (36, 64, 32, 32, 10, 0),   # operands spread over 2^+-10
    (40, 64, 32, 32, 0, "ch12"),   # per-column weight scales over 2^+-12, one column at 2^-20 of the max
    (64, 128, 16, 16, 0, "dead20"),
]


@pytest.mark.parametrize("H,W,C,N,spread,wsp", SMALL2D)
def test_unet_small_2d_convs_are_fp32_accurate(engine, H, W, C, N, spread, wsp):
    """The default arithmetic (two-plane fp16 split, k_conv2d_h16) and the exact-f32 form against fp64: both within
    1e-6 of each output's sum |x w|, the split at most 4x the f32 form's error."""
    rng = np.random.Generator(np.random.PCG64(H * 131 + C + N))
    x = rng.standard_normal((H, W, C)).astype(np.float32)
    w = (rng.standard_normal((N, C, 3, 3)) / np.sqrt(9 * C)).astype(np.float32)
    if spread:
        x *= np.exp2(rng.integers(-spread, spread + 1, size=x.shape)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    if wsp:
        cs = _wspread(rng, N, wsp)
        w = (w * cs[:, None, None, None]).astype(np.float32)
        bias = (bias * cs).astype(np.float32)
    xd = torch.from_numpy(x.astype(np.float64)).permute(2, 0, 1)[None]
    wd = torch.from_numpy(w.astype(np.float64))
    ref = torch.relu(torch.nn.functional.conv2d(xd, wd, torch.from_numpy(bias.astype(np.float64)), padding=1))
    mag = torch.nn.functional.conv2d(xd.abs(), wd.abs(), None, padding=1) + np.abs(bias)[None, :, None, None]
    ref = ref[0].permute(1, 2, 0).numpy()
    mag = mag[0].permute(1, 2, 0).numpy() + 1e-300
    errs = {}
    for mode in ("f32", "default"):
        y = engine.conv2d3x3(x, w, bias, relu=True, math=mode).cpu().numpy()
        assert y.shape == ref.shape
        errs[mode] = float(np.max(np.abs(y - ref) / mag))
    print(f"\n2-D {H}x{W} {C}->{N}: " + " ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    assert errs["f32"] < 1e-6, errs
    assert errs["default"] < 1e-6 and errs["default"] <= 4.0 * errs["f32"] + 1e-8, errs


DEEP2D = [  # H, W, C_in, N, weight spread: the RMVPE U-Net's deep levels (windowed gather-streamed kernel, conv_gs.hip)
    (49, 4, 512, 512, 0),    # intermediate (196 px)
    (98, 8, 256, 256, 0),    # level 3 (784 px)
    (196, 16, 128, 128, 0),  # level 2 (3136 px)
    (33, 8, 256, 80, 0),     # ragged rows and a partial 32-column tile
    (20, 32, 128, 64, 0),
    # per-column weight scales (the windowed kernel shares h16_finish's per-column inverse scales)
    (49, 4, 512, 512, "ch12"),
    (98, 8, 256, 256, "dead20"),
    (196, 16, 128, 128, "ch12"),
    (33, 8, 256, 80, "dead20"),
]


@pytest.mark.parametrize("H,W,C,N,wsp", DEEP2D)
def test_unet_deep_level_windowed_kernels(engine, H, W, C, N, wsp):
    """The windowed gather-streamed kernel (64 x 64 tiles, K split over workgroups by the size policy) against fp64,
    per output element relative to its own sum |x w|: within 1e-6 and at most 4x the exact-f32 kernel's error, also
    with per-column weight scales over 2^+-12 and a column at 2^-20 of the tensor max."""
    rng = np.random.Generator(np.random.PCG64(H * 7 + W + C + N))
    x = rng.standard_normal((H, W, C)).astype(np.float32)
    w = (rng.standard_normal((N, C, 3, 3)) / np.sqrt(9 * C)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    if wsp:
        cs = _wspread(rng, N, wsp)
        w = (w * cs[:, None, None, None]).astype(np.float32)
        bias = (bias * cs).astype(np.float32)
    xd = torch.from_numpy(x.astype(np.float64)).permute(2, 0, 1)[None]
    wd = torch.from_numpy(w.astype(np.float64))
    ref = torch.relu(torch.nn.functional.conv2d(xd, wd, torch.from_numpy(bias.astype(np.float64)), padding=1))
    mag = torch.nn.functional.conv2d(xd.abs(), wd.abs(), None, padding=1) + np.abs(bias)[None, :, None, None]
    ref = ref[0].permute(1, 2, 0).numpy()
    mag = mag[0].permute(1, 2, 0).numpy() + 1e-300
    errs = {}
    for mode in ("f32", "gsw"):
        y = engine.conv2d3x3(x, w, bias, relu=True, math=mode).cpu().numpy()
        assert y.shape == ref.shape
        errs[mode] = float(np.max(np.abs(y - ref) / mag))
    print(f"\n2-D deep {H}x{W} {C}->{N} {wsp or ''}: " + " ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    assert errs["f32"] < 1e-6, errs
    assert errs["gsw"] < 1e-6 and errs["gsw"] <= 4.0 * errs["f32"] + 1e-8, errs


UPCONV = [  # H, W, C_in, N, weight spread: the U-Net decoder's ConvTranspose2d (3x3, stride 2, pad 1, output pad 1)
    (49, 4, 512, 256, 0),     # decoder level 0 (the intermediate's output)
    (98, 8, 256, 128, 0),
    (196, 16, 128, 64, 0),
    (392, 32, 64, 32, 0),
    (33, 8, 256, 40, 0),      # ragged rows, 4 x 40 virtual columns (a partial tile)
    (98, 8, 256, 128, "ch12"),
    (196, 16, 128, 64, "dead20"),
    (49, 4, 512, 256, "ch12"),
]


@pytest.mark.parametrize("H,W,C,N,wsp", UPCONV)
def test_unet_upconv_phase_gather_kernel(engine, H, W, C, N, wsp):
    """the decoder's up-convs run as a 2x2-tap phase conv with 4 N virtual columns on the
    fp16-split gather kernel, whose epilogue maps the phase layout (store_tile16 OUT_UPSAMPLE2D). Against fp64
    torch.nn.functional.conv_transpose2d (RMVPE.py ResDecoderBlock conv1: stride 2, padding 1, output_padding 1),
    per output element relative to its own sum |x w|: within 1e-6 and at most 4x the exact-f32 kernel's error, also
    with per-output-channel weight scales over 2^+-12 and a channel at 2^-20 of the tensor max."""
    rng = np.random.Generator(np.random.PCG64(H * 11 + W + C + N))
    x = rng.standard_normal((H, W, C)).astype(np.float32)
    w = (rng.standard_normal((C, N, 3, 3)) / np.sqrt(9 * C)).astype(np.float32)  # torch layout [C_in][N][kh][kw]
    bias = rng.standard_normal(N).astype(np.float32)
    if wsp:
        cs = _wspread(rng, N, wsp)
        w = (w * cs[None, :, None, None]).astype(np.float32)
        bias = (bias * cs).astype(np.float32)
    xd = torch.from_numpy(x.astype(np.float64)).permute(2, 0, 1)[None]
    wd = torch.from_numpy(w.astype(np.float64))
    ct = torch.nn.functional.conv_transpose2d
    ref = torch.relu(ct(xd, wd, torch.from_numpy(bias.astype(np.float64)), stride=2, padding=1, output_padding=1))
    mag = ct(xd.abs(), wd.abs(), None, stride=2, padding=1, output_padding=1) + np.abs(bias)[None, :, None, None]
    ref = ref[0].permute(1, 2, 0).numpy()
    mag = mag[0].permute(1, 2, 0).numpy() + 1e-300
    errs = {}
    for mode in ("f32", "default"):
        y = engine.convtranspose2d_s2(x, w, bias, relu=True, math=mode).cpu().numpy()
        assert y.shape == ref.shape, (y.shape, ref.shape)
        errs[mode] = float(np.max(np.abs(y - ref) / mag))
    print(f"\nup-conv {H}x{W} {C}->{N} {wsp or ''}: " + " ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    assert errs["f32"] < 1e-6, errs
    assert errs["default"] < 1e-6 and errs["default"] <= 4.0 * errs["f32"] + 1e-8, errs
