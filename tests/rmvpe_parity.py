"""RMVPE / pipeline parity against a reference run whose salience is known (test helper, no GPU needed).

The RMVPE decode (rvc/lib/predictors/RMVPE.py:484-540) is discontinuous: an argmax flip between two near-tied
bins moves f0 by >= 20 cents, and the NSF source integrates f0 into its phase (generators/hifigan.py:156-228), so
from the first flipped frame on the waveform legitimately drifts from the reference. With random-init weights
such near ties exist (tests/golden/*: top-1 vs top-2 margins down to 2e-5). The checks here separate that from a
real error:

  1. salience error  err = max |device - reference| over the exact fp32 values the reference decoded (argmax
     +- 4 bins and the runner-up), raised to the lower bound the fp16 copy of the whole matrix implies; it must
     itself be within what fp32 arithmetic explains: 3x the reference's own fp32-vs-fp64 salience gap on the clip
     (8.7e-5 .. 1.5e-4, tests/golden/add_salience_noise.py);
  2. near-tied frames  top-1 - top-2 <= 2 err (the argmax may flip) or |top-1 - 0.03| <= err (voicing may flip);
  3. every frame whose device argmax differs from the reference's must be near-tied;
  4. every other frame's f0 must agree within the bound the salience error implies for decode's weighted
     average (sum_j |c_j - avg| err / (sum_j s_j - 9 err), x1.5), and its voicing must agree.

The waveform is compared sample by sample where f0 cannot move it: the synthesis path fed the reference's own
pitch track (the strict gate), and the pipeline's output against that path fed the device's own f0 (consistency);
the end-to-end output against the reference by spectrogram correlation.
"""
from __future__ import annotations

import numpy as np

CENTS = np.pad(20.0 * np.arange(360) + 1997.3794084376191, (4, 4))  # RMVPE.py:442-443
THRED = 0.03


def margins(hidden, thred=THRED):
    """The decision margins make_golden_sizes.salience_margins stores, for an fp32 salience [F, 360]."""
    h = np.asarray(hidden, np.float32)
    order = np.argsort(-h, axis=1, kind="stable")
    i1, i2 = order[:, 0], order[:, 1]
    rows = np.arange(h.shape[0])
    hp = np.pad(h, ((0, 0), (4, 4)))
    return {"sal_margin": h[rows, i1] - h[rows, i2], "sal_thr_margin": h[rows, i1] - np.float32(thred),
            "sal_argmax": i1, "sal_second": i2, "sal_top2": h[rows, i2],
            "sal_win": np.stack([hp[rows, i1 + j] for j in range(9)], axis=1)}


def _cents(f):
    f = np.asarray(f, np.float64)
    out = np.zeros_like(f)
    v = f > 0
    out[v] = 1200.0 * np.log2(f[v] / 10.0)
    return out


def check_rmvpe(dev_f0, dev_hidden, ref, ref_f0, thred=THRED, max_err=None):
    """Principled f0 parity (module docstring). ref: mapping with sal_* (and optionally hidden16). The salience
    error itself must stay <= max_err (absolute, salience in [0, 1]); default 3 x the fixture's sal_fp32_noise
    (how far the reference's own fp32 salience sits from fp64 on this clip, tests/golden/add_salience_noise.py):
    beyond that it is a real error, and the near-tie set it would open up is meaningless.
    Returns dict(err, n_near, flips (frame indices), first_flip (or None))."""
    F = len(ref_f0)
    h = np.asarray(dev_hidden, np.float32)[:F]
    assert h.shape == (F, 360), h.shape
    rows = np.arange(F)
    i1 = np.asarray(ref["sal_argmax"]).astype(np.int64)
    i2 = np.asarray(ref["sal_second"]).astype(np.int64)
    hp = np.pad(h, ((0, 0), (4, 4)))
    win = np.stack([hp[rows, i1 + j] for j in range(9)], axis=1)
    err = max(float(np.abs(win - ref["sal_win"]).max()), float(np.abs(h[rows, i2] - ref["sal_top2"]).max()))
    if "hidden16" in ref:
        h16 = np.asarray(ref["hidden16"])
        # the whole matrix against its fp16 copy: rel <= 1e-3 of the peak, and no bin off by more than err +
        # the fp16 half-spacing (else err is raised to the bound the copy implies)
        d = np.abs(h - h16.astype(np.float32))
        assert float(d.max()) <= 1e-3 * float(np.abs(h16).max()), float(d.max())
        err = max(err, float((d - np.spacing(h16).astype(np.float32) / 2).max()))
    if max_err is None:
        max_err = 3.0 * float(ref["sal_fp32_noise"])
    if err > max_err:
        ew = np.abs(win - ref["sal_win"]).max(1)
        blk = [float(ew[i:i + 256].max()) for i in range(0, F, 256)]
        raise AssertionError(f"salience error {err:.3e} > {max_err:.1e}: window err max {ew.max():.3e} at frame "
                             f"{int(ew.argmax())}, p50 {np.median(ew):.2e}, p99 {np.percentile(ew, 99):.2e}; per 256 "
                             f"frames {['%.1e' % v for v in blk]}")
    near_arg = np.asarray(ref["sal_margin"]) <= 2 * err + 1e-7
    near_thr = np.abs(np.asarray(ref["sal_thr_margin"])) <= err + 1e-7
    dev_arg = np.argmax(h, axis=1)
    flips = dev_arg != i1
    bad = flips & ~near_arg
    assert not bad.any(), (f"argmax differs on frames that are not near-tied: {np.where(bad)[0][:10]} "
                           f"(err {err:.3e}, margins {np.asarray(ref['sal_margin'])[bad][:5]})")
    ok = ~flips & ~near_thr
    vd, vr = np.asarray(dev_f0) > 0, np.asarray(ref_f0) > 0
    assert np.array_equal(vd[ok], vr[ok]), f"voicing differs on {np.where(ok & (vd != vr))[0][:10]}"
    both = ok & vd & vr
    s = np.asarray(ref["sal_win"], np.float64)
    cm = np.stack([CENTS[i1 + j] for j in range(9)], axis=1)
    avg = (s * cm).sum(1) / s.sum(1)
    bound = 1.5 * err * np.abs(cm - avg[:, None]).sum(1) / np.maximum(s.sum(1) - 9 * err, 1e-12) + 1e-6
    dc = np.abs(_cents(dev_f0) - _cents(ref_f0))
    over = both & (dc > bound)
    assert not over.any(), (f"f0 off by more than the salience error allows on {np.where(over)[0][:10]}: "
                            f"{dc[over][:5]} cents vs bound {bound[over][:5]}")
    fl = np.where(flips | (near_thr & (vd != vr)))[0]
    return {"err": err, "n_near": int((near_arg | near_thr).sum()), "flips": fl,
            "first_flip": int(fl[0]) if len(fl) else None}


def rel_err(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))


def trim_normalize(vc, t_pad_tgt=48000):
    """voice_conversion output -> Pipeline.pipeline's: trim t_pad_tgt per side, peak-normalise (pipeline.py:494,
    :550-552)."""
    y = np.asarray(vc, np.float32)[t_pad_tgt:-t_pad_tgt]
    mx = np.abs(y).max() / 0.99
    return y / mx if mx > 1 else y
