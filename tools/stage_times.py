"""Unprofiled per-stage wall times of the C2 step (diagnostic, not product code).

Times each device stage of bench.py's C2 step on its own, with no profiler attached and no per-launch events:
the whole pipeline, RMVPE (U-Net + BiGRU + decode), HuBERT, Synthesizer.infer (TextEncoder + flow + generator) and
the generator alone (dec_only), all at C2's padded length (216100 + 2 x 16000 samples -> 1550 frames). Each figure
is the mean over R back-to-back calls bracketed by a device synchronise, so host issue overlaps the GPU as it does
in the bench. TE + flow = synth_infer - dec_only; the U-Net front = rmvpe - the BiGRU's own time (bench_gru).

    python tools/stage_times.py [--reps 20]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "retrieval-based-voice-conversion-mlx_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="", help="comma-separated stage names (default: all)")
    args = ap.parse_args()
    from rvcx import synthetic
    from rvcx.config import SYNTH_48K_V2
    from rvcx.engine import Engine
    from rvcx.weights import normalize_state

    dev = torch.device("cuda:0")
    eng = Engine(0)
    eng.load_synth(normalize_state(synthetic.synth_state(2)), SYNTH_48K_V2)
    eng.load_hubert(normalize_state(synthetic.hubert_state(4)))
    eng.load_rmvpe(normalize_state(synthetic.rmvpe_state(5)))
    eng.set_pipeline_highpass(16000)
    n = 216100
    audio = torch.as_tensor(synthetic.speech_like(n, seed=1000), dtype=torch.float64).to(dev)
    pad = torch.as_tensor(synthetic.speech_like(n + 32000, seed=1001), dtype=torch.float32).to(dev)
    T = (n + 32000) // 160
    rng = np.random.Generator(np.random.PCG64(7))
    phone = torch.as_tensor(rng.standard_normal((1, T, 768)).astype(np.float32), device=dev)
    lengths = torch.tensor([T], dtype=torch.int32, device=dev)
    f0 = torch.as_tensor(synthetic.f0_walk(1, T, seed=3), dtype=torch.float32, device=dev)
    coarse = torch.clamp((f0 / 4).round().to(torch.int32), 1, 255)
    sid = torch.zeros((1,), dtype=torch.int32, device=dev)
    z = torch.as_tensor(rng.standard_normal((1, 192, T)).astype(np.float32), device=dev)
    cap = (n + 32000) // 160 * eng.upp
    out = torch.empty((cap,), dtype=torch.float32, device=dev)

    stages = {
        "pipeline": lambda i: eng.pipeline(audio, sid=0, semitones=0.0, protect=0.33, t_pad=16000, t_pad_tgt=48000,
                                           seed=1234 + i, out=out),
        "rmvpe": lambda i: eng.rmvpe(pad),
        "hubert": lambda i: eng.hubert(pad),
        "synth_infer": lambda i: eng.synth_infer(phone, lengths, coarse, f0, sid, seed=i),
        "dec_only": lambda i: eng.dec_only(z, f0, sid, seed=i),
    }
    if args.only:
        stages = {k: v for k, v in stages.items() if k in args.only.split(",")}
    res = {}
    for name, fn in stages.items():
        for i in range(3):
            fn(i)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(args.reps):
            fn(i)
        torch.cuda.synchronize(dev)
        res[name] = round((time.perf_counter() - t0) / args.reps * 1000.0, 3)
        print(f"{name:12s} {res[name]:8.3f} ms", flush=True)
    if "synth_infer" in res and "dec_only" in res:
        res["te_flow"] = round(res["synth_infer"] - res["dec_only"], 3)
    print(json.dumps({"frames": T, "reps": args.reps, "ms": res}))
    eng.close()


if __name__ == "__main__":
    main()
