"""CREPE host side and oracle (no GPU): weight-layout mapping of the MLX npz (tools/convert_crepe_weights.py),
framing / decode semantics of rvc_mlx/lib/mlx/crepe.py on known answers."""
import numpy as np

from oracle import crepe as oc


def test_mlx_npz_layout_maps_to_torch(tmp_path):
    from rvcx import synthetic
    from rvcx.weights import load_crepe_weights

    w = synthetic.crepe_state("tiny", seed=3)
    mlx = {}
    for k, v in w.items():  # convert_crepe_weights.py:52-61
        if k.startswith("conv") and k.endswith(".weight") and "_BN" not in k:
            v = np.transpose(v, (0, 2, 3, 1))
        elif k == "classifier.weight":
            v = v.T
        mlx[k] = v
    mlx["conv1_BN.num_batches_tracked"] = np.zeros((), np.float32)
    p = tmp_path / "crepe_tiny.npz"
    np.savez(p, **mlx)
    got = load_crepe_weights(str(p))
    assert set(got) == set(w)
    for k in w:
        np.testing.assert_array_equal(got[k], w[k])


def test_frames_normalised():
    x = (np.sin(np.arange(4000) * 0.05) * 3 + 1).astype(np.float32)
    fr = oc.frame_audio(x)
    assert fr.shape == (1 + 4000 // 160, 1024)
    np.testing.assert_allclose(fr.mean(1), 0, atol=1e-5)
    np.testing.assert_allclose(fr.std(1), 1, atol=1e-4)
    silent = oc.frame_audio(np.zeros(2000, np.float32))
    assert not silent.any()  # std 0 <= 1e-10: no division (crepe.py:352-354)


def test_decode_known_answers():
    F = 4
    p = np.zeros((F, 360), np.float32)
    p[0, 100] = 0.9  # lone peak: cents = CENTS[100] exactly
    p[1, 200], p[1, 201] = 0.5, 0.5  # two equal bins: first argmax, mean of the two bins
    p[2, 5] = 0.99  # below f0_min 50 Hz (bin 5 ~ 33 Hz) -> masked
    p[2, 150] = 0.3
    f0, per = oc.decode(p, 50.0, 1100.0)
    assert per[0] == np.float32(0.9) and per[1] == np.float32(0.5) and per[2] == np.float32(0.3)
    c0 = np.float32(oc.CENTS[100])
    assert f0[0] == np.float32(10.0) * np.float32(2) ** (c0 / np.float32(1200.0))
    c1 = np.float32((oc.CENTS[200] + oc.CENTS[201]) / 2)
    np.testing.assert_allclose(f0[1], 10 * 2 ** (c1 / 1200), rtol=1e-6)
    assert f0[3] == np.float32(10.0) and per[3] == 0  # nothing in range: cents 0 -> 10 Hz, periodicity 0


def test_rvc_semantics_oracle_framing_and_viterbi():
    """oracle.crepe's restatement of rvc/'s CREPE (torchcrepe.predict): zero-padded frames with unit unbiased std
    (the edge frames see the zeros), and a viterbi path that follows a clean track moving <= 1 bin per frame, masks
    the bins outside [f0_min, f0_max) and keeps the track through a short low-probability gap."""
    from oracle import crepe as oc

    n = 16000
    a = np.sin(2 * np.pi * 200.0 * np.arange(n) / 16000.0).astype(np.float32)
    fr = oc.frame_audio_torch(a)
    assert fr.shape == (1 + n // 160, 1024)
    np.testing.assert_allclose(fr[50].std(ddof=1), 1.0, rtol=1e-5)
    assert np.all(fr[0][:512] == fr[0][0])  # zero padding: the first half of frame 0 is one constant
    F = 120
    track = (120 + np.round(10 * np.sin(np.arange(F) / 8.0))).astype(int)
    probs = np.full((F, 360), 0.05, dtype=np.float32)
    probs[np.arange(F), track] = 0.99
    probs[60:64] = 0.05  # a gap: the path stays near the track
    bins = oc.viterbi_bins(probs, 50.0, 1100.0)
    keep = np.r_[0:60, 64:F]
    np.testing.assert_array_equal(bins[keep], track[keep])
    assert np.all(np.abs(bins[60:64] - track[59]) <= 11)
    lo, hi = oc.torchcrepe_bin_range(50.0, 1100.0)
    assert (lo, hi) == (39, 308)
    probs2 = probs.copy()
    probs2[:, 20] = 1.0  # below f0_min: masked, never chosen
    assert np.all(oc.viterbi_bins(probs2, 50.0, 1100.0) >= lo)
