"""Parity at the full workload sizes of C3 and C4 (BASELINE configs[2] / configs[3]) against reference runs.

C3  rvcx_dec_only at B = 32 x 400 frames on bench.py's own C3 input (z ~ PCG64(3), f0 = f0_walk(32, 400, 3),
    sid 0). Rows 0, 13 and 31 against the reference HiFiGANNSFGenerator (generators/hifigan_nsf.py:173-212) run
    on those rows with recorded noise (tests/golden/dec_c3_rows.npz, make_golden_sizes.py c3); the generator
    is unmasked so a row does not depend on its batch. Bar: rel <= 2e-3 of the row's peak (the fixture is
    stored in fp16: <= 2.5e-4 of that is storage rounding), spectrogram correlation >= 0.999; all 32 rows
    finite and inside tanh's range.
C4  rvcx_pipeline_batch at B = 8 x 30 s (480000 samples: HuBERT L = 1599 and synthesizer T = 3198 frames, the
    key-split sizes of the fused attention; RMVPE over 3201 mel frames, U-Net and BiGRU batched 8 wide).
    Row 0 against the reference Pipeline.pipeline on that utterance (tests/golden/pipeline_c4_30s.npz), rows 1
    and 2 against the CPU oracle pipeline (oracle/pipeline.py) with their own noise; all three through the
    salience-aware f0 check and the waveform check of tests/rmvpe_parity.py (2e-3 before the first flipped
    frame, spectrogram correlation >= 0.999); rows 3-7 finite and peak-normalised.
"""
import numpy as np
import pytest

from conftest import fixture_noise, golden
from rmvpe_parity import check_rmvpe, check_waveform, margins, rel_err

pytestmark = pytest.mark.gpu


def c3_inputs(B=32, T=400):
    """bench.py bench_c3's input (and make_golden_sizes.c3_inputs), bit for bit."""
    from rvcx import synthetic

    rng = np.random.Generator(np.random.PCG64(3))
    z = rng.standard_normal((B, 192, T)).astype(np.float32)
    f0 = synthetic.f0_walk(B, T, seed=3).astype(np.float32)
    return z, f0


def test_c3_generator_b32_vs_reference(engine):
    from oracle.metrics import spectrogram_correlation

    g = golden("dec_c3_rows.npz")
    z, f0 = c3_inputs()
    assert float(z.astype(np.float64).sum()) == float(g["z_sum"]) and float(f0.astype(np.float64).sum()) == float(g["f0_sum"])
    B, T = z.shape[0], z.shape[2]
    upp = engine.upp
    rows = [int(r) for r in g["rows"]]
    es = np.random.default_rng(77).standard_normal((B, T * upp)).astype(np.float32)
    er = np.random.Generator(np.random.PCG64(int(g["noise_seed"]))).standard_normal(tuple(g["eps_src_shape"]))
    er = er.astype(np.float32)
    assert abs(float(er.astype(np.float64).sum()) - float(g["eps_sum"])) < 1e-6 * abs(float(g["eps_sum"])) + 1e-6
    es[rows] = er.reshape(len(rows), -1)
    out = engine.dec_only(z, f0, np.zeros(B, np.int32), eps_src=es)
    engine.check_device_status()
    out = out.cpu().numpy()
    assert out.shape == (B, T * upp)
    assert np.isfinite(out).all() and float(np.abs(out).max()) <= 1.0
    assert (np.abs(out).max(1) > 0).all()
    for k, r in enumerate(rows):
        ref = g["out16"][k].astype(np.float32)
        assert spectrogram_correlation(out[r], ref) >= 0.999
        assert rel_err(out[r], ref) <= 2e-3, (r, rel_err(out[r], ref))


@pytest.mark.timeout(420)
def test_c4_batch8_30s_vs_reference_and_oracle(engine, synth_w, hubert_w, rmvpe_w):
    from rvcx import synthetic
    from test_gpu_pipeline_api import NoiseRecorder, oracle_pipeline

    g = golden("pipeline_c4_30s.npz")
    n, B = 480000, 8
    clips = [synthetic.speech_like(n, seed=1000 + k).astype(np.float32).astype(np.float64) for k in range(B)]
    assert float(clips[0].sum()) == float(g["audio_sum"])
    engine.set_pipeline_highpass()
    T = (n + 2 * 16000) // 160 - 2  # p_len = min(m // 160, 2 L) = 3198
    upp = engine.upp
    rng = np.random.default_rng(5)
    ez = rng.standard_normal((B, 192 * T)).astype(np.float32)
    es = rng.standard_normal((B, T * upp)).astype(np.float32)
    z0, s0 = fixture_noise(g)
    assert z0.size == 192 * T and s0.size == T * upp
    ez[0], es[0] = z0, s0
    refs, ref_sal = [g["out16"].astype(np.float32)], [dict(g)]
    ref_f0 = [g["f0_raw"]]
    for b in (1, 2):
        noise = NoiseRecorder(60 + b)
        orc = oracle_pipeline(synth_w, hubert_w, rmvpe_w, noise)
        refs.append(orc.pipeline(0, clips[b].copy(), protect=0.33))
        ref_f0.append(orc.last["f0_raw"])
        ref_sal.append(margins(orc.last["hidden"]))
        ref_sal[-1]["hidden_exact"] = np.asarray(orc.last["hidden"], np.float32)
        ez[b], es[b] = noise.cat()
    opts = engine.pipeline_opts(protect=0.33)
    y, f0, hid = engine.pipeline_batch(np.stack(clips), opts, sids=0, eps_z=ez, eps_src=es, want_f0=True,
                                       want_hidden=True)
    engine.check_device_status()
    y, f0, hid = y.cpu().numpy(), f0.cpu().numpy(), hid.cpu().numpy()
    assert y.shape == (B, 1439040) and f0.shape == (B, 3201)
    for b in range(3):
        if "hidden_exact" in ref_sal[b]:
            he = ref_sal[b]["hidden_exact"]
            assert rel_err(hid[b][: he.shape[0]], he) <= 1e-3
        r = check_rmvpe(f0[b], hid[b], ref_sal[b], ref_f0[b])
        w = check_waveform(y[b], refs[b], r["first_flip"])
        print(f"\nC4 row {b}: salience err {r['err']:.2e}, {r['n_near']} near-tied, flips {list(r['flips'])[:8]}, "
              f"spec corr {w['spec_corr']:.6f}, prefix {w['prefix']} rel {w['rel']}")
    assert np.isfinite(y).all()
    peaks = np.abs(y).max(1)
    assert (peaks > 0).all() and (peaks <= 0.99 + 1e-6).all()
