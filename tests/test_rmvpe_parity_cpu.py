"""The salience-aware parity check (tests/rmvpe_parity.py) on the reference's own C2 salience, no GPU: it accepts
a perturbation at the measured error level that flips only near-tied frames and rejects a flip elsewhere, a
voicing change, and an f0 shift larger than the salience error allows."""
import numpy as np
import pytest

from conftest import golden
from rmvpe_parity import check_rmvpe, margins


def decode(h, thred=0.03):
    """RMVPE0Predictor.decode (RMVPE.py:484-540), numpy."""
    from oracle import rmvpe as ormvpe

    return ormvpe.decode(h, thred)


@pytest.fixture(scope="module")
def case():
    g = golden("pipeline_c2_synth.npz")
    h = g["hidden16"].astype(np.float32)
    ref = margins(h)  # exact margins of this (fp16-valued) salience
    return h, ref, decode(h)


def test_identity_passes(case):
    h, ref, f0 = case
    r = check_rmvpe(f0, h, ref, f0, max_err=1e-4)
    assert r["err"] == 0.0 and r["first_flip"] is None


def test_near_tie_flip_is_accepted(case):
    h, ref, f0 = case
    m = np.where(ref["sal_margin"] > 0, ref["sal_margin"], np.inf)  # (the fp16 copy holds exact ties)
    k = int(np.argmin(m))
    d = h.copy()
    eps = float(ref["sal_margin"][k])
    d[k, ref["sal_second"][k]] += np.float32(1.5 * eps)  # the runner-up overtakes: error 1.5 eps >= margin / 2
    r = check_rmvpe(decode(d), d, ref, f0, max_err=1e-2)  # (fp16-valued salience: margins >= 4.9e-4)
    assert k in r["flips"] and r["first_flip"] == k


def test_flip_outside_near_ties_fails(case):
    h, ref, f0 = case
    k = int(np.argmax(ref["sal_margin"]))
    d = h.copy() + np.float32(1e-6)
    d[k, ref["sal_second"][k]] = h[k, ref["sal_argmax"][k]] + 0.01
    with pytest.raises(AssertionError):
        check_rmvpe(decode(d), d, ref, f0, max_err=1e-4)  # the salience error itself is too large


def test_f0_shift_beyond_bound_fails(case):
    h, ref, f0 = case
    d = h + np.float32(1e-6)
    f = decode(d)
    v = np.where(f > 0)[0][5]
    f[v] *= 2 ** (5 / 1200)  # 5 cents: far above what a 1e-6 salience error allows
    with pytest.raises(AssertionError):
        check_rmvpe(f, d, ref, f0, max_err=1e-4)
