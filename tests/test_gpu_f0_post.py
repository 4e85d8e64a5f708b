"""rvcx_f0_post (Pipeline.get_f0's pitch shift + coarse quantisation, rvc/infer/pipeline.py:278-291) is
INTEGER output: it must be bit-exact, not "98 % of frames".

1. Real f0 tracks (the reference's ios_test_data RMVPE f0 of real speech, the reference-run RMVPE f0 of the
   golden fixtures) x pitch shifts: coarse == the reference formula evaluated by numpy, exactly; pitchf and
   the shifted f0 exactly equal.
2. A sweep that puts the scaled mel value within a few ulps of every half-integer k + 0.5 (where rint can go
   either way): the device must equal the reference chain with a correctly rounded log (Decimal), which is
   the machine-independent value of the reference formula. numpy's own log differs from the correctly
   rounded one by an ulp on a few inputs (it is a SIMD approximation that also differs from glibc); on every
   point where numpy's log is correctly rounded the device must also equal numpy.
"""
from decimal import Decimal, getcontext

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

MEL_MIN = 1127 * np.log(1 + 50 / 700)
MEL_MAX = 1127 * np.log(1 + 1100 / 700)


def ref_coarse(f0, pitch, log=np.log):
    """pipeline.py:280-289 verbatim (f0 float64 numpy array, pitch int semitones)."""
    f0 = np.array(f0, dtype=np.float64)
    f0 *= pow(2, pitch / 12)
    f0bak = f0.copy()
    f0_mel = 1127 * log(1 + f0 / 700)
    f0_mel[f0_mel > 0] = (f0_mel[f0_mel > 0] - MEL_MIN) * 254 / (MEL_MAX - MEL_MIN) + 1
    f0_mel[f0_mel <= 1] = 1
    f0_mel[f0_mel > 255] = 255
    return np.rint(f0_mel).astype(int), f0bak


def log_cr(x):
    getcontext().prec = 60
    return np.array([float(Decimal(float(v)).ln()) for v in np.asarray(x, np.float64).reshape(-1)])


def device(engine, f0, pitch):
    coarse, pitchf, fs = engine.f0_post(np.asarray(f0, np.float64), float(pitch))
    return coarse.cpu().numpy(), pitchf.cpu().numpy(), fs.cpu().numpy()


@pytest.mark.parametrize("pitch", [-12, -5, 0, 3, 7, 12])
def test_f0_post_bit_exact_on_reference_f0(engine, pitch):
    tracks = [golden("ios_kat.npz")["rmvpe_f0"], golden("rmvpe_1s.npz")["f0"]]
    for name in ("pipeline_c2_ios.npz", "pipeline_c2_synth.npz"):
        try:
            tracks.append(golden(name)["f0_raw"])
        except FileNotFoundError:
            pass
    for f0 in tracks:
        f0 = np.asarray(f0, np.float64)
        c, pf, fs = device(engine, f0, pitch)
        rc, rf = ref_coarse(f0, pitch)
        assert np.array_equal(c, rc), np.flatnonzero(c != rc)[:10]
        assert np.array_equal(fs, rf)
        assert np.array_equal(pf, rf.astype(np.float32))


def _half_integer_sweep(ulps=6):
    """f0 values whose scaled mel lands within a few ulps of k + 0.5, k = 1..254, plus the clamp edges."""
    ks = np.arange(1, 255, dtype=np.float64)
    m = (ks + 0.5 - 1) * (MEL_MAX - MEL_MIN) / 254 + MEL_MIN
    f = 700 * (np.exp(m / 1127) - 1)
    pts = [f]
    up, dn = f.copy(), f.copy()
    for _ in range(ulps):
        up = np.nextafter(up, np.inf)
        dn = np.nextafter(dn, -np.inf)
        pts += [up.copy(), dn.copy()]
    edges = np.array([0.0, 1e-300, 50.0, 1100.0, 49.999999, 1100.000001, 5000.0, 20000.0])
    return np.concatenate(pts + [edges])


def test_f0_post_half_integer_sweep_correctly_rounded(engine):
    f0 = _half_integer_sweep()
    c, _, _ = device(engine, f0, 0)
    cr, _ = ref_coarse(f0, 0, log=log_cr)
    assert np.array_equal(c, cr), np.flatnonzero(c != cr)[:10]
    # near-ties really are exercised: the sweep crosses the rounding boundary of most half-integers
    v = (1127 * log_cr(1 + f0 / 700) - MEL_MIN) * 254 / (MEL_MAX - MEL_MIN) + 1
    frac = v - np.floor(v)
    assert np.mean(np.abs(frac - 0.5) < 1e-12) > 0.9
    # numpy's log: where it is correctly rounded, numpy's coarse equals the device's
    y = 1 + f0 / 700
    np_ok = np.log(y) == log_cr(y)
    nc, _ = ref_coarse(f0, 0)
    assert np.array_equal(c[np_ok], nc[np_ok])
    assert np_ok.mean() > 0.95, np_ok.mean()
