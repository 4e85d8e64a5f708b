"""Streaming (config C5) fixture from the REFERENCE's own realtime code (survey container only).

Run:  python tests/golden/make_golden_stream.py      (needs /root/reference; never on the GPU box)

Runs rvc/realtime/core.py ``VoiceChanger`` -> ``Realtime`` -> rvc/realtime/pipeline.py
``Realtime_Pipeline`` (create_pipeline, realloc, inference, voice_conversion, process_audio/SOLA) for 16
independent streams at the C5 geometry (read_chunk_size 96 = 256 ms hops @48 kHz, crossfade 0.1 s, extra
0.5 s), hop by hop, with the seeded synthetic weights.

Imports the container lacks are stubbed:
  * torchaudio.transforms.Resample -> oracle/realtime.py's restatement of torchaudio's sinc_interp_hann
    resampler (torchaudio is not installed: this one piece stays a restatement, "parity unpinned" against
    torchaudio itself);
  * noisereduce.torchgate, pedalboard, webrtcvad, soxr, soundfile, wget, faiss, torchcrepe, torchfcpe: never
    called on this path (clean_audio / post_process / vad off, no index);
  * rvc.lib.utils.load_embedding (which would download ContentVec): returns transformers.HubertModel built
    from the reference's local contentvec config with the seeded weights.
Everything else -- buffer geometry, circular writes, RMS gate, realtime f0 quantisation, HuBERT + repeated
last frame, x2 upsample, protect, Synthesizer.infer, clip, * sqrt(vol), output resample, SOLA search and
crossfade -- is the reference's code.

Saved (tests/golden/stream_c5_16.npz): per stream and hop the output block (fp16), vol, SOLA offset; the
inputs are regenerated from their seeds (rvcx.synthetic.speech_like at 48 kHz, float32; a SHA-256 of the
float32 bytes is stored to prove the regeneration exact) and so is the noise (PCG64 per stream, eps_z then
eps_src per hop).
"""
from __future__ import annotations

import hashlib
import os
import shutil
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (paths, stubs, weight builders)

import torch  # noqa: E402

N_STREAMS, HOPS, BLOCK = 16, 6, 96 * 128
INPUT_SEED0, NOISE_SEED0 = 300, 700
OPTS = dict(f0_up_key=2, index_rate=0.0, protect=0.33, volume_envelope=1, f0_autotune=False,
            f0_autotune_strength=1, proposed_pitch=False, proposed_pitch_threshold=155.0)
SILENT_STREAM = 15  # its hops 2-3 are digital silence: the gated path (core.py:274-298)


def stream_inputs():
    from rvcx import synthetic

    x = np.stack([synthetic.speech_like(BLOCK * HOPS, seed=INPUT_SEED0 + s, sr=48000).astype(np.float32)
                  for s in range(N_STREAMS)])
    x[SILENT_STREAM, 2 * BLOCK:4 * BLOCK] = 0.0
    return x


def inputs_digest(x: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(x, dtype=np.float32).tobytes()).hexdigest()


def install_realtime_stubs():
    from oracle.realtime import resample

    mg.install_stubs()
    ta = types.ModuleType("torchaudio")
    tat = types.ModuleType("torchaudio.transforms")

    class Resample(torch.nn.Module):
        def __init__(self, orig_freq, new_freq, dtype=torch.float32, **kw):
            super().__init__()
            assert dtype == torch.float32 and not kw
            self.o, self.n = int(orig_freq), int(new_freq)

        def forward(self, x):
            return resample(x, self.o, self.n)

    tat.Resample = Resample
    ta.transforms = tat
    sys.modules["torchaudio"] = ta
    sys.modules["torchaudio.transforms"] = tat
    nr = types.ModuleType("noisereduce")
    nrt = types.ModuleType("noisereduce.torchgate")
    nrt.TorchGate = None
    nr.torchgate = nrt
    sys.modules["noisereduce"] = nr
    sys.modules["noisereduce.torchgate"] = nrt
    pb = types.ModuleType("pedalboard")
    for n in ("Pedalboard", "Chorus", "Distortion", "Reverb", "PitchShift", "Limiter", "Gain", "Bitcrush",
              "Clipping", "Compressor", "Delay"):
        setattr(pb, n, None)
    sys.modules["pedalboard"] = pb
    for n in ("webrtcvad", "soxr", "soundfile", "wget"):
        sys.modules.setdefault(n, types.ModuleType(n))


def main():
    from transformers import HubertConfig, HubertModel  # noqa: F401  (resolve before the module stubs exist)

    install_realtime_stubs()
    sys.path.insert(0, mg.REF)
    scratch = tempfile.mkdtemp(prefix="rvc_stream_golden_")
    os.makedirs(os.path.join(scratch, "rvc", "models", "predictors"))
    shutil.copytree(os.path.join(mg.REF, "rvc", "configs"), os.path.join(scratch, "rvc", "configs"),
                    ignore=shutil.ignore_patterns("*.py", "__pycache__"))
    os.chdir(scratch)
    torch.manual_seed(0)
    torch.set_num_threads(8)

    from rvcx import synthetic
    from rvcx.config import SYNTH_48K_V2

    # the model file the reference loads with torch.load(weights_only=True) (pipeline.py:41-52)
    sd = mg.to_torch_state(synthetic.synth_state(mg.SEEDS["synth"]))
    model_path = os.path.join(scratch, "model.pth")
    torch.save({"config": SYNTH_48K_V2.as_list(), "weight": sd, "f0": 1, "version": "v2", "vocoder": "HiFi-GAN",
                "sr": 48000}, model_path)
    _, rsd = mg.build_rmvpe_state()
    torch.save(rsd, os.path.join(scratch, "rvc", "models", "predictors", "rmvpe.pt"))
    hub = mg.build_hubert()

    import rvc.realtime.pipeline as rtp
    from rvc.realtime import core

    rtp.load_embedding = lambda *a, **k: hub  # never download
    x = stream_inputs()
    outs = np.zeros((N_STREAMS, HOPS, BLOCK), np.float32)
    vols = np.zeros((N_STREAMS, HOPS), np.float64)
    offs = np.full((N_STREAMS, HOPS), -1, np.int64)
    orig_randn, orig_argmax = torch.randn_like, torch.argmax
    for s in range(N_STREAMS):
        vc = core.VoiceChanger(96, 0.1, 0.5, model_path=model_path, index_path="", f0_method="rmvpe",
                               silent_threshold=-90, sid=s % 4)
        if s == 0:
            net = vc.vc_model.pipeline.vc.net_g
            refm = mg.build_synth()
            rtp.strip_parametrizations(refm)
            ref = refm.state_dict()
            got = {k: v for k, v in net.state_dict().items() if not k.startswith("enc_q.")}  # unused posterior enc
            assert set(ref) == set(got), (sorted(set(ref) - set(got))[:5], sorted(set(got) - set(ref))[:5])
            for k, v in got.items():  # strict=False in the reference load: prove nothing was skipped
                assert torch.equal(v, ref[k]), k
            rt = vc.vc_model
            geom = (rt.convert_feature_size_16k, rt.skip_head, rt.return_length, rt.convert_buffer.shape[0])
            assert geom == (87, 50, 37, 13920), geom
        ns = mg.NoiseStream(NOISE_SEED0 + s)
        seen = []

        def argmax(t, *a, **k):
            r = orig_argmax(t, *a, **k)
            if t.dim() == 1 and t.shape[0] == vc.sola_search_frame + 1:
                seen.append(int(r))
            return r

        torch.randn_like, torch.argmax = ns, argmax
        try:
            for h in range(HOPS):
                res, vol, _ = vc.on_request(x[s, h * BLOCK:(h + 1) * BLOCK].copy(), **OPTS)
                outs[s, h] = res
                vols[s, h] = vol
                offs[s, h] = seen[-1]
        finally:
            torch.randn_like, torch.argmax = orig_randn, orig_argmax
        assert len(ns.draws) == 2 * HOPS and len(seen) == HOPS
        print(f"stream {s}: offs {offs[s].tolist()} vol {np.round(vols[s], 4).tolist()}", flush=True)
    np.savez_compressed(os.path.join(mg.OUT, "stream_c5_16.npz"), out16=outs.astype(np.float16), vol=vols,
                        sola_offset=offs, n_streams=N_STREAMS, hops=HOPS, block=BLOCK, input_seed0=INPUT_SEED0,
                        noise_seed0=NOISE_SEED0, silent_stream=SILENT_STREAM, sids=np.arange(N_STREAMS) % 4,
                        f0_up_key=OPTS["f0_up_key"], protect=OPTS["protect"], input_sha256=inputs_digest(x),
                        out_peak=np.abs(outs).max(axis=2))


if __name__ == "__main__":
    main()
