"""The two RMVPE regimes the C2 / C4 fixtures do not reach, on the HIP path against the REFERENCE itself
(tests/golden/make_golden_sizes.py c1 / long ran rvc/lib/predictors/RMVPE.py RMVPE0Predictor.infer_from_audio,
RMVPE.py:497-513, with the seeded weights):

  * C1 (BASELINE configs[0], benchmarks/benchmark_rmvpe.py:22-32): 5 s of 0.3 sin 440 + 0.2 sin 880 + 0.1 N(0,1),
    the strong-salience, always-voiced regime of the reference's own parity tests (tests/pitch/test_parity.py:368);
  * more than mel2hidden's 32000-frame chunk (RMVPE.py:459-481): 340 s of speech-like audio, 34001 mel frames, two
    chunks run as independent E2E passes; the seam (frames 31488 .. 32511) is held to the principled salience bar of
    tests/rmvpe_parity.py, every frame to the reference's f0 within 50 cents / the same voicing.

Tolerances as test_gpu_c2_parity.py: device salience vs the reference's within 3x the reference's own fp32-vs-fp64
gap on the clip (sal_fp32_noise); argmax flips only on near-tied frames; every other frame's f0 within the cents
bound that error implies.
"""
import numpy as np
import pytest

from conftest import golden
from rmvpe_parity import check_rmvpe

pytestmark = pytest.mark.gpu


def test_rmvpe_c1_clip_vs_reference(engine):
    from rvcx import synthetic

    g = golden("rmvpe_c1.npz")
    audio = synthetic.rmvpe_bench_audio(80000, seed=int(g["audio_seed"]))
    assert abs(float(audio.astype(np.float64).sum()) - float(g["audio_sum"])) < 1e-6
    f0, hid = engine.rmvpe(audio, thred=0.03, want_hidden=True)
    engine.check_device_status()
    f0, hid = f0.cpu().numpy(), hid.cpu().numpy()
    assert f0.shape == g["f0"].shape == (501,)
    r = check_rmvpe(f0, hid, g, g["f0"])
    vd, vr = f0 > 0, g["f0"] > 0
    assert np.array_equal(vd, vr) and vr.all()
    cents = 1200 * np.abs(np.log2(f0[vr] / g["f0"][vr]))
    assert np.mean(cents <= 50) >= 0.99
    print(f"\nC1: salience err {r['err']:.2e} (bound {3 * float(g['sal_fp32_noise']):.2e}), {r['n_near']} near-tied, "
          f"flips {list(r['flips'])}, max {cents.max():.3f} cents, mean f0 {f0.mean():.2f} Hz")


def test_rmvpe_beyond_one_chunk_vs_reference(engine):
    """> 32000 mel frames: the chunked mel2hidden branch (runtime_fe.cpp, batched full chunks + the tail chunk)."""
    from rvcx import synthetic

    g = golden("rmvpe_long.npz")
    n = int(g["n"])
    audio = synthetic.speech_like(n, seed=int(g["audio_seed"])).astype(np.float32)
    assert abs(float(audio.astype(np.float64).sum()) - float(g["audio_sum"])) < 1e-6 * max(1.0, abs(float(g["audio_sum"])))
    f0, hid = engine.rmvpe(audio, thred=0.03, want_hidden=True)
    engine.check_device_status()
    f0 = f0.cpu().numpy()
    F = 1 + n // 160
    assert F > 32000 and f0.shape == g["f0"].shape == (F,)
    lo, hi = (int(v) for v in g["win"])
    r = check_rmvpe(f0[lo:hi], hid[lo:hi].cpu().numpy(), g, g["f0_win"])
    # every frame: the reference's voicing and f0 within 50 cents (SURVEY §8(d) gate iii)
    ref = g["f0"].astype(np.float64)
    vd, vr = f0 > 0, ref > 0
    agree = float(np.mean(vd == vr))
    both = vd & vr
    cents = 1200 * np.abs(np.log2(f0[both] / ref[both]))
    assert agree >= 0.995, agree
    assert float(np.mean(cents <= 50)) >= 0.99
    print(f"\nlong ({F} frames): seam salience err {r['err']:.2e}, flips {list(r['flips'])}, voicing agree {agree:.5f}, "
          f"within 50 cents {float(np.mean(cents <= 50)):.5f}")
