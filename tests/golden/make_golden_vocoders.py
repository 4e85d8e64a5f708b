"""Golden vectors for the synthesizer variants beside the default pitch-guided HiFi-GAN (NSF), by running the
REFERENCE's own modules (survey container only; never on the GPU box).

Run:  python tests/golden/make_golden_vocoders.py [nof0] [mrf] [refinegan]

  nof0       Synthesizer(use_f0=False): TextEncoder without emb_pitch + HiFiGANGenerator
             (rvc/lib/algorithm/synthesizers.py:84, :119-139, :233-239; generators/hifigan.py:9-104)
  mrf        Synthesizer(vocoder="MRF HiFi-GAN"): HiFiGANMRFGenerator with the 9-harmonic source
             (synthesizers.py:86-98; generators/hifigan_mrf.py); torch.rand (initial phases) recorded too
  refinegan  Synthesizer(vocoder="RefineGAN"): RefineGANGenerator (synthesizers.py:99-107; generators/refinegan.py).
             torchaudio is absent here: torchaudio.functional.resample is replaced by oracle.realtime's restatement
             of torchaudio 2.x (kaiser window), so that one piece is pinned to the restatement. Its noise (the AdaIN
             draws are ~1.8 M floats) is not stored: the seeds and draw shapes are, and tests regenerate it.
Each fixture holds the inputs, the recorded RNG draws and the reference outputs; weights are regenerated from the
seeds (rvcx.synthetic) by the tests. Harness as in make_golden.py (stubs, seeded noise streams).
"""
from __future__ import annotations

import dataclasses
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402  (sets sys.path, imports torch + transformers first)
import torch  # noqa: E402

from rvcx import synthetic  # noqa: E402
from rvcx.config import SYNTH_48K_V2  # noqa: E402

SEED_W = 21  # synthesizer weights of the variant fixtures
SEED_IN = 23


def build(cfg, vocoder: str):
    from rvc.lib.algorithm.synthesizers import Synthesizer

    net = Synthesizer(*cfg.as_list(), use_f0=cfg.use_f0, text_enc_hidden_dim=768, vocoder=vocoder)
    del net.enc_q
    net.eval()
    sd = mg.to_torch_state(synthetic.synth_state(SEED_W, cfg))
    ref = net.state_dict()
    assert set(sd) == set(ref), (sorted(set(ref) - set(sd))[:8], sorted(set(sd) - set(ref))[:8])
    for k, v in ref.items():
        assert tuple(v.shape) == tuple(sd[k].shape), (k, v.shape, sd[k].shape)
    net.load_state_dict(sd, strict=True)
    return net


def nof0():
    cfg = dataclasses.replace(SYNTH_48K_V2, use_f0=False)
    net = build(cfg, "HiFi-GAN")
    rng = np.random.Generator(np.random.PCG64(SEED_IN))
    B, T = 2, 40
    phone = rng.standard_normal((B, T, 768)).astype(np.float32)
    lengths = np.array([40, 33], np.int64)
    sid = np.array([5, 100], np.int64)
    ns = mg.NoiseStream(SEED_IN + 1)
    orig = torch.randn_like
    torch.randn_like = ns
    try:
        with torch.no_grad():
            o, x_mask, (z, z_p, m_p, logs_p) = net.infer(torch.from_numpy(phone), torch.from_numpy(lengths), None,
                                                         None, torch.from_numpy(sid))
    finally:
        torch.randn_like = orig
    assert len(ns.draws) == 1, len(ns.draws)  # only z_p's randn_like: the HiFiGANGenerator draws nothing
    np.savez_compressed(os.path.join(mg.OUT, "synth_nof0_b2.npz"), phone=phone, lengths=lengths, sid=sid,
                        eps_z=ns.draws[0], o=o.numpy(), z=z.numpy(), z_p=z_p.numpy(), seed_w=SEED_W)
    print("synth_nof0_b2: o", o.shape, float(o.abs().max()), float(o.std()))


class UniformStream:
    """Replaces torch.rand: seeded PCG64 uniforms in [0, 1), recorded in call order."""

    def __init__(self, seed):
        self.rng = np.random.Generator(np.random.PCG64(seed))
        self.draws = []

    def __call__(self, *size, **kw):
        if len(size) == 1 and isinstance(size[0], (tuple, list)):
            size = tuple(size[0])
        x = self.rng.random(size).astype(np.float32)
        self.draws.append(x)
        return torch.from_numpy(x.copy())


def mrf():
    cfg = dataclasses.replace(SYNTH_48K_V2, vocoder="MRF HiFi-GAN")
    net = build(cfg, "MRF HiFi-GAN")
    rng = np.random.Generator(np.random.PCG64(SEED_IN + 10))
    B, T = 2, 24
    phone = rng.standard_normal((B, T, 768)).astype(np.float32)
    f0 = synthetic.f0_walk(B, T, seed=SEED_IN + 11)
    pitch = rng.integers(1, 256, size=(B, T)).astype(np.int64)
    lengths = np.array([24, 19], np.int64)
    sid = np.array([1, 7], np.int64)
    ns, us = mg.NoiseStream(SEED_IN + 12), UniformStream(SEED_IN + 13)
    orig_n, orig_u = torch.randn_like, torch.rand
    torch.randn_like, torch.rand = ns, us
    try:
        with torch.no_grad():
            o, x_mask, (z, z_p, m_p, logs_p) = net.infer(torch.from_numpy(phone), torch.from_numpy(lengths),
                                                         torch.from_numpy(pitch), torch.from_numpy(f0),
                                                         torch.from_numpy(sid))
    finally:
        torch.randn_like, torch.rand = orig_n, orig_u
    assert len(ns.draws) == 2 and len(us.draws) == 1, (len(ns.draws), len(us.draws))
    eps_src = np.concatenate([ns.draws[1].reshape(-1), us.draws[0].reshape(-1)])  # C-ABI layout (include/rvcx.h)
    np.savez_compressed(os.path.join(mg.OUT, "synth_mrf_b2.npz"), phone=phone, f0=f0, pitch=pitch, lengths=lengths,
                        sid=sid, eps_z=ns.draws[0], eps_src=eps_src, o=o.numpy(), z=z.numpy(), z_p=z_p.numpy(),
                        seed_w=SEED_W)
    print("synth_mrf_b2: o", o.shape, float(o.abs().max()), float(o.std()))


def refinegan():
    import types

    from oracle.realtime import functional_resample

    ta = sys.modules.setdefault("torchaudio", types.ModuleType("torchaudio"))
    fn = types.ModuleType("torchaudio.functional")
    fn.resample = functional_resample
    ta.functional = fn
    sys.modules["torchaudio.functional"] = fn
    cfg = dataclasses.replace(SYNTH_48K_V2, vocoder="RefineGAN")
    net = build(cfg, "RefineGAN")
    rng = np.random.Generator(np.random.PCG64(SEED_IN + 20))
    B, T = 1, 6
    phone = rng.standard_normal((B, T, 768)).astype(np.float32)
    f0 = synthetic.f0_walk(B, T, seed=SEED_IN + 21)
    pitch = rng.integers(1, 256, size=(B, T)).astype(np.int64)
    lengths = np.array([T], np.int64)
    sid = np.array([2], np.int64)
    ns, us = mg.NoiseStream(SEED_IN + 22), UniformStream(SEED_IN + 23)
    orig_n, orig_u = torch.randn_like, torch.rand
    torch.randn_like, torch.rand = ns, us
    try:
        with torch.no_grad():
            o, x_mask, (z, z_p, m_p, logs_p) = net.infer(torch.from_numpy(phone), torch.from_numpy(lengths),
                                                         torch.from_numpy(pitch), torch.from_numpy(f0),
                                                         torch.from_numpy(sid))
    finally:
        torch.randn_like, torch.rand = orig_n, orig_u
    shapes = np.array([d.size for d in ns.draws], np.int64)
    assert len(ns.draws) == 2 + 24 and len(us.draws) == 1, (len(ns.draws), len(us.draws))
    np.savez_compressed(os.path.join(mg.OUT, "synth_refinegan_b1.npz"), phone=phone, f0=f0, pitch=pitch,
                        lengths=lengths, sid=sid, noise_seed=SEED_IN + 22, uniform_seed=SEED_IN + 23,
                        draw_sizes=shapes, o=o.numpy(), z=z.numpy(), seed_w=SEED_W)
    print("synth_refinegan_b1: o", o.shape, float(o.abs().max()), float(o.std()))


def main():
    mg.install_stubs()
    sys.path.insert(0, mg.REF)
    os.chdir(tempfile.mkdtemp(prefix="rvc_golden_voc_"))
    torch.manual_seed(0)
    torch.set_num_threads(8)
    which = set(sys.argv[1:]) or {"nof0"}
    if "nof0" in which:
        nof0()
    if "mrf" in which:
        mrf()
    if "refinegan" in which:
        refinegan()


if __name__ == "__main__":
    main()
