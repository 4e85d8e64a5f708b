"""Generate golden vectors by running the REFERENCE implementation (survey container only).

Run:  python tests/golden/make_golden.py        (needs /root/reference; never on the GPU box)
      python tests/golden/make_golden.py --only-c2   (only the full-size C2 pipeline fixtures)

What it does (SURVEY.md Appendix C recipe):
  1. import transformers first, then stub the modules the reference imports but the
     container lacks (torchaudio, torchcrepe, torchfcpe, faiss, librosa with
     ``filters.mel`` restated in numpy);
  2. build the reference modules (rvc/lib/algorithm/synthesizers.py Synthesizer,
     rvc/lib/predictors/RMVPE.py, transformers.HubertModel from the local contentvec
     config) and load the seeded synthetic weights of rvcx.synthetic;
  3. patch torch.randn_like so the reference's RNG draws come from a seeded numpy
     stream and save those draws next to the outputs;
  4. write small .npz fixtures under tests/golden/.

Weights are NOT stored: tests regenerate them from the seeds recorded here.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import types

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(REPO, "retrieval-based-voice-conversion-mlx_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import transformers  # noqa: E402,F401  (must precede the librosa stub)

from oracle.rmvpe import mel_filterbank  # noqa: E402
from rvcx import synthetic  # noqa: E402
from rvcx.config import HUBERT_BASE, SYNTH_48K_V2  # noqa: E402

SEEDS = {"synth": 2, "hubert": 4, "rmvpe": 5, "noise": 7, "inputs": 11}


def install_stubs():
    for name in ("torchaudio", "torchcrepe", "faiss"):
        sys.modules.setdefault(name, types.ModuleType(name))
    fcpe = types.ModuleType("torchfcpe")
    fcpe.spawn_infer_model_from_pt = None
    sys.modules["torchfcpe"] = fcpe
    lib = types.ModuleType("librosa")
    filters = types.ModuleType("librosa.filters")

    def mel(sr, n_fft, n_mels=128, fmin=0.0, fmax=None, htk=False, **kw):
        return mel_filterbank(sr, n_fft, n_mels, fmin, fmax if fmax is not None else sr / 2.0, htk)

    filters.mel = mel
    lib.filters = filters
    sys.modules["librosa"] = lib
    sys.modules["librosa.filters"] = filters


class NoiseStream:
    """Replaces torch.randn_like: seeded PCG64 normal draws, recorded in call order."""

    def __init__(self, seed):
        self.rng = np.random.Generator(np.random.PCG64(seed))
        self.draws = []

    def __call__(self, t, *a, **k):
        x = self.rng.standard_normal(tuple(t.shape)).astype(np.float32)
        self.draws.append(x)
        return torch.from_numpy(x).to(t.dtype)


def to_torch_state(d):
    out = {}
    for k, v in d.items():
        if k.endswith(".weight_g"):
            k = k[: -len(".weight_g")] + ".parametrizations.weight.original0"
        elif k.endswith(".weight_v"):
            k = k[: -len(".weight_v")] + ".parametrizations.weight.original1"
        out[k] = torch.from_numpy(np.asarray(v))
    return out


def build_synth():
    from rvc.lib.algorithm.synthesizers import Synthesizer

    net = Synthesizer(*SYNTH_48K_V2.as_list(), use_f0=True, text_enc_hidden_dim=768, vocoder="HiFi-GAN")
    del net.enc_q
    net.eval()
    sd = to_torch_state(synthetic.synth_state(SEEDS["synth"]))
    ref_keys = set(net.state_dict().keys())
    assert set(sd.keys()) == ref_keys, (sorted(ref_keys - set(sd)), sorted(set(sd) - ref_keys))
    for k, v in net.state_dict().items():
        assert tuple(v.shape) == tuple(sd[k].shape), (k, v.shape, sd[k].shape)
    net.load_state_dict(sd, strict=True)
    return net


def build_hubert():
    from transformers import HubertConfig, HubertModel

    with open(os.path.join(REF, "rvc_mlx/models/embedders/contentvec/config.json")) as f:
        conf = json.load(f)
    conf.pop("architectures", None)
    model = HubertModel(HubertConfig(**conf)).eval()
    st = synthetic.hubert_state(SEEDS["hubert"])
    st = {k: v for k, v in st.items() if not k.startswith("final_proj")}
    sd = to_torch_state(st)
    ref = model.state_dict()
    missing = set(ref) - set(sd)
    assert missing <= {"masked_spec_embed"}, missing
    extra = set(sd) - set(ref)
    assert not extra, extra
    for k in sd:
        assert tuple(ref[k].shape) == tuple(sd[k].shape), (k, ref[k].shape, sd[k].shape)
    model.load_state_dict(sd, strict=False)
    return model


def build_rmvpe_state():
    from rvc.lib.predictors.RMVPE import E2E

    model = E2E(4, 1, (2, 2))
    st = synthetic.rmvpe_state(SEEDS["rmvpe"])
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in st.items()}
    ref = model.state_dict()
    assert set(ref) == set(sd), (set(ref) ^ set(sd))
    for k in sd:
        assert tuple(ref[k].shape) == tuple(sd[k].shape), (k, ref[k].shape, sd[k].shape)
    model.load_state_dict(sd, strict=True)
    return model.eval(), sd


class Recorder(torch.nn.Module):
    """HuBERT wrapper for the reference pipeline that keeps last_hidden_state of every call."""

    def __init__(self, m):
        super().__init__()
        self.m = m
        self.out = []

    def forward(self, x):
        r = self.m(x)
        self.out.append(r["last_hidden_state"].detach().numpy().copy())
        return r


def c2_fixtures(hub, net, scratch):
    """The headline config C2 at full size: the reference Pipeline.pipeline
    (rvc/infer/pipeline.py:390-558, x_pad=1, one chunk) on the 13.5 s clips
      * ios: the reference's own real-speech clip ios_test_data/input_audio.npy (216100 samples), and
      * synth: the bench's C2 clip (rvcx.synthetic.speech_like(216100, seed=1000), rounded to float32
        values so the fixture is exact and small),
    with seeded noise. Saved per clip: the final output, the RMVPE f0 and get_f0's (pitch, pitchf), the
    HuBERT features (fp16, for the staged test) and the noise seed; the noise itself is regenerated from
    the seed (NoiseStream: PCG64 standard normals, eps_z [1,192,T] then eps_src [1,T*480,1])."""
    import rvc.infer.pipeline as rpipe
    from rvc.infer.pipeline import Pipeline

    class Cfg:
        x_pad, x_query, x_center, x_max, device = 1, 6, 38, 41, "cpu"

    clips = {
        "ios": np.load(os.path.join(REF, "ios_test_data", "input_audio.npy")).astype(np.float64),
        "synth": synthetic.speech_like(216100, seed=1000).astype(np.float32).astype(np.float64),
    }
    for k, (name, audio) in enumerate(clips.items()):
        pipe = Pipeline(48000, Cfg())
        rec = Recorder(hub)
        got = {}
        orig_get_f0 = rpipe.Pipeline.get_f0

        def get_f0(self, *a, **kw):
            c, f = orig_get_f0(self, *a, **kw)
            got["pitch"], got["pitchf"] = np.array(c), np.array(f)
            return c, f

        seed = SEEDS["noise"] + 100 + k
        ns = NoiseStream(seed)
        orig = torch.randn_like
        torch.randn_like = ns
        rpipe.Pipeline.get_f0 = get_f0
        try:
            outp = pipe.pipeline(rec, net, 0, audio.copy(), 0, "rmvpe", "", 0.0, True, 1.0, "v2", 0.33,
                                 False, 1.0, False, 155.0)
        finally:
            torch.randn_like = orig
            rpipe.Pipeline.get_f0 = orig_get_f0
        assert len(rec.out) == 1 and len(ns.draws) == 2, "expected one chunk"
        extra = {"audio32": audio.astype(np.float32)} if name == "synth" else {}
        np.savez_compressed(
            os.path.join(OUT, f"pipeline_c2_{name}.npz"), out=np.asarray(outp, np.float32),
            f0_raw=got["pitchf"].astype(np.float64), pitch=got["pitch"].astype(np.int64),
            feats16=rec.out[0][0].astype(np.float16), noise_seed=np.int64(seed),
            eps_z_shape=np.array(ns.draws[0].shape), eps_src_shape=np.array(ns.draws[1].shape),
            eps_sum=np.array([float(ns.draws[0].astype(np.float64).sum()), float(ns.draws[1].astype(np.float64).sum())]),
            **extra)
        print(f"pipeline_c2_{name}:", np.shape(outp), "voiced", int((got["pitchf"] > 0).sum()),
              "feats", rec.out[0].shape)


def main():
    install_stubs()
    sys.path.insert(0, REF)
    scratch = tempfile.mkdtemp(prefix="rvc_golden_")
    os.makedirs(os.path.join(scratch, "rvc", "models", "predictors"))
    os.chdir(scratch)
    torch.manual_seed(0)
    torch.set_num_threads(8)
    rng = np.random.Generator(np.random.PCG64(SEEDS["inputs"]))
    meta = {"seeds": SEEDS, "torch": torch.__version__, "transformers": transformers.__version__}

    only_c2 = "--only-c2" in sys.argv
    net = build_synth()
    if only_c2:
        hub = build_hubert()
        e2e, rsd = build_rmvpe_state()
        torch.save(rsd, os.path.join(scratch, "rvc", "models", "predictors", "rmvpe.pt"))
        c2_fixtures(hub, net, scratch)
        return

    # ---------------- synthesizer at T=64 frames (module outputs) ----------------
    T = 64
    phone = rng.standard_normal((1, T, 768)).astype(np.float32)
    f0 = synthetic.f0_walk(1, T, seed=SEEDS["inputs"])
    pitch = rng.integers(1, 256, size=(1, T)).astype(np.int64)
    lengths = np.array([T], np.int64)
    sid = np.array([3], np.int64)
    import rvc.lib.algorithm.synthesizers as rsyn
    import rvc.lib.algorithm.generators.hifigan as rhg

    ns = NoiseStream(SEEDS["noise"])
    orig = torch.randn_like
    torch.randn_like = ns
    try:
        with torch.no_grad():
            o, x_mask, (z, z_p, m_p, logs_p) = net.infer(
                torch.from_numpy(phone), torch.from_numpy(lengths), torch.from_numpy(pitch),
                torch.from_numpy(f0), torch.from_numpy(sid))
    finally:
        torch.randn_like = orig
    eps_z, eps_src = ns.draws[0], ns.draws[1]
    np.savez_compressed(os.path.join(OUT, "synth_t64.npz"), phone=phone, f0=f0, pitch=pitch, lengths=lengths,
                        sid=sid, eps_z=eps_z, eps_src=eps_src.reshape(1, -1), o=o.numpy(), z=z.numpy(),
                        z_p=z_p.numpy(), m_p=m_p.numpy(), logs_p=logs_p.numpy())
    print("synth_t64: o", o.shape, float(o.abs().max()), float(o.std()))

    # ---------------- ragged batch (B=2, lengths 48/40) ----------------
    T2 = 48
    phone2 = rng.standard_normal((2, T2, 768)).astype(np.float32)
    f02 = synthetic.f0_walk(2, T2, seed=SEEDS["inputs"] + 1)
    pitch2 = rng.integers(1, 256, size=(2, T2)).astype(np.int64)
    lengths2 = np.array([48, 40], np.int64)
    sid2 = np.array([0, 108], np.int64)
    ns = NoiseStream(SEEDS["noise"] + 1)
    torch.randn_like = ns
    try:
        with torch.no_grad():
            o2, m2, (z2, zp2, mp2, lp2) = net.infer(
                torch.from_numpy(phone2), torch.from_numpy(lengths2), torch.from_numpy(pitch2),
                torch.from_numpy(f02), torch.from_numpy(sid2))
    finally:
        torch.randn_like = orig
    np.savez_compressed(os.path.join(OUT, "synth_b2_ragged.npz"), phone=phone2, f0=f02, pitch=pitch2,
                        lengths=lengths2, sid=sid2, eps_z=ns.draws[0], eps_src=ns.draws[1].reshape(2, -1),
                        o=o2.numpy(), z=z2.numpy(), z_p=zp2.numpy(), m_p=mp2.numpy(), logs_p=lp2.numpy())
    print("synth_b2_ragged: o", o2.shape)

    # ---------------- generator alone (C3 shape scaled: B=2, T=24) ----------------
    zg = rng.standard_normal((2, 192, 24)).astype(np.float32)
    f0g = synthetic.f0_walk(2, 24, seed=SEEDS["inputs"] + 2)
    ns = NoiseStream(SEEDS["noise"] + 2)
    torch.randn_like = ns
    try:
        with torch.no_grad():
            g = net.emb_g(torch.tensor([0, 0])).unsqueeze(-1)
            og = net.dec(torch.from_numpy(zg), torch.from_numpy(f0g), g=g)
    finally:
        torch.randn_like = orig
    np.savez_compressed(os.path.join(OUT, "dec_b2_t24.npz"), z=zg, f0=f0g, sid=np.array([0, 0]),
                        eps_src=ns.draws[0].reshape(2, -1), o=og.numpy())
    print("dec: o", og.shape)

    # ---------------- HuBERT on 1 s ----------------
    hub = build_hubert()
    aud = synthetic.speech_like(16000, seed=SEEDS["inputs"]).astype(np.float32)
    with torch.no_grad():
        hf = hub(torch.from_numpy(aud)[None])["last_hidden_state"]
    np.savez_compressed(os.path.join(OUT, "hubert_1s.npz"), audio=aud, feats=hf.numpy())
    print("hubert:", hf.shape, float(hf.std()))

    # ---------------- RMVPE on 1 s ----------------
    from rvc.lib.predictors.RMVPE import RMVPE0Predictor

    e2e, rsd = build_rmvpe_state()
    rpath = os.path.join(scratch, "rvc", "models", "predictors", "rmvpe.pt")
    torch.save(rsd, rpath)
    pred = RMVPE0Predictor(rpath, device="cpu")
    ar = synthetic.speech_like(16000, seed=SEEDS["inputs"] + 3).astype(np.float32)
    with torch.no_grad():
        mel = pred.mel_extractor(torch.from_numpy(ar)[None], center=True)
        hidden = pred.mel2hidden(mel).squeeze(0).numpy()
    f0r = pred.decode(hidden, thred=0.03)
    np.savez_compressed(os.path.join(OUT, "rmvpe_1s.npz"), audio=ar, mel=mel.numpy(), hidden=hidden, f0=f0r)
    print("rmvpe: mel", mel.shape, "hidden", hidden.shape, "voiced", int((f0r > 0).sum()))

    # ---------------- full pipeline on 2.5 s (x_pad=1, one chunk) ----------------
    from rvc.infer.pipeline import Pipeline

    class Cfg:
        x_pad, x_query, x_center, x_max, device = 1, 6, 38, 41, "cpu"

    class HubWrap(torch.nn.Module):
        def __init__(self, m):
            super().__init__()
            self.m = m

        def forward(self, x):
            return self.m(x)

    pipe = Pipeline(48000, Cfg())
    ap = synthetic.speech_like(40000, seed=SEEDS["inputs"] + 4)
    ns = NoiseStream(SEEDS["noise"] + 3)
    torch.randn_like = ns
    try:
        outp = pipe.pipeline(HubWrap(hub), net, 0, ap.copy(), 0, "rmvpe", "", 0.0, True, 1.0, "v2", 0.33,
                             False, 1.0, False, 155.0)
    finally:
        torch.randn_like = orig
    np.savez_compressed(os.path.join(OUT, "pipeline_2p5s.npz"), audio=ap, eps_z=ns.draws[0],
                        eps_src=ns.draws[1].reshape(1, -1), out=np.asarray(outp, np.float32))
    print("pipeline:", np.shape(outp), float(np.abs(outp).max()))

    with open(os.path.join(OUT, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
