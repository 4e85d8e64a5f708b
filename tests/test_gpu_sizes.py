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
    and 2 against the CPU oracle pipeline (oracle/pipeline.py) with their own noise. Per row: the salience-aware
    f0 check of tests/rmvpe_parity.py; spectrogram correlation >= 0.999 end to end; the 30 s synthesis path fed
    the reference's pitch track within 1e-4 of the peak (1e-3 against the fp16 fixture); the batched output within
    1e-4 of the single-utterance path fed the batch's own f0. Rows 3-7 finite and peak-normalised.
"""
import numpy as np
import pytest

from conftest import fixture_noise, golden
from rmvpe_parity import check_rmvpe, margins, rel_err, trim_normalize

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
    from oracle.metrics import spectrogram_correlation
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
    # row 0: the reference run; rows 1-2: the oracle pipeline (exact fp32 salience, own noise)
    refs = [{"out": g["out16"].astype(np.float32), "f0": g["f0_raw"], "pitch": g["pitch"].astype(np.int64), "sal": dict(g),
             "tol": 1e-3}]  # (the fixture output is fp16: <= 2.5e-4 of the peak is storage rounding)
    for b in (1, 2):
        noise = NoiseRecorder(60 + b)
        orc = oracle_pipeline(synth_w, hubert_w, rmvpe_w, noise)
        out = orc.pipeline(0, clips[b].copy(), protect=0.33)
        sal = margins(orc.last["hidden"])
        sal["sal_fp32_noise"] = g["sal_fp32_noise"]  # same clip length and kind
        sal["exact"] = np.asarray(orc.last["hidden"], np.float32)
        refs.append({"out": out, "f0": orc.last["f0_raw"], "pitch": np.asarray(orc.last["pitch"], np.int64),
                     "sal": sal, "tol": 1e-4})
        ez[b], es[b] = noise.cat()
    opts = engine.pipeline_opts(protect=0.33)
    y, f0, hid = engine.pipeline_batch(np.stack(clips), opts, sids=0, eps_z=ez, eps_src=es, want_f0=True,
                                       want_hidden=True)
    engine.check_device_status()
    y, f0, hid = y.cpu().numpy(), f0.cpu().numpy(), hid.cpu().numpy()
    assert y.shape == (B, 1439040) and f0.shape == (B, 3201)
    for b, ref in enumerate(refs):
        if "exact" in ref["sal"]:
            assert rel_err(hid[b], ref["sal"]["exact"]) <= 1e-3
        r = check_rmvpe(f0[b], hid[b], ref["sal"], ref["f0"])
        c = spectrogram_correlation(y[b], ref["out"])
        assert c >= 0.999, (b, c)
        # the 30 s synthesis path (HuBERT L = 1599, TextEncoder / flow / generator T = 3198) fed the reference's
        # own pitch: the sample-level gate
        _, p32 = engine.highpass_pad(clips[b], 16000)
        P = p32.shape[0] // 160  # voice_conversion takes >= n/160 pitch frames and uses p_len = min(n/160, 2L)
        vc = trim_normalize(engine.voice_conversion(p32, ref["pitch"][:P], ref["f0"][:P].astype(np.float32), 0, 0.33,
                                                    eps_z=ez[b], eps_src=es[b]).cpu().numpy())
        e_ref = rel_err(vc, ref["out"])
        assert e_ref <= ref["tol"], (b, e_ref)
        # the batched pass equals the single-utterance path fed the batch's own f0 (B = 8 vs B = 1 GEMM orders)
        coarse, pitchf, _ = engine.f0_post(f0[b], 0.0)
        vcd = trim_normalize(engine.voice_conversion(p32, coarse[:P], pitchf[:P], 0, 0.33, eps_z=ez[b],
                                                     eps_src=es[b]).cpu().numpy())
        cons = rel_err(y[b], vcd)
        assert cons <= 1e-4, (b, cons)
        print(f"\nC4 row {b}: salience err {r['err']:.2e}, {r['n_near']} near-tied, flips {list(r['flips'])[:8]}, "
              f"spec corr {c:.6f}, vc on reference pitch {e_ref:.2e}, batch vs single {cons:.2e}")
    assert np.isfinite(y).all()
    peaks = np.abs(y).max(1)
    assert (peaks > 0).all() and (peaks <= 0.99 + 1e-6).all()
