"""Benchmark: RVC v2 48 kHz full pipeline (BASELINE.json configs[1], C2) on MI355X.

One step = one 13.5 s utterance (216100 samples @16 kHz, speech-like synthetic audio already
resident in HBM) through the whole device pipeline: filtfilt -> reflect pad (x_pad = 1 s) ->
RMVPE f0 -> f0 shift/quantise -> HuBERT -> x2 upsample/protect -> TextEncoder -> flow reverse ->
HiFiGAN-NSF -> trim -> peak-normalise, output left in HBM. Random-init weights of the exact
architectures (no checkpoints offline). Multi-GPU: one process per GPU, each rank converts its
own utterances (weak scaling, no data-path collective); only the timing max uses RCCL.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "retrieval-based-voice-conversion-mlx_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense FP32 (vector = f32-in MFMA)
SR_IN = 16000
C2_SAMPLES = 216100  # 13.50625 s (the reference's 13.5 s benchmark clip length)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--samples", type=int, default=C2_SAMPLES)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-sec", type=float, default=2.0)
    ap.add_argument("--roofline-pass", choices=["inline", "after"], default="after",
                    help="inline: HIP events around every conv launch of the timed steps; after: the timed steps "
                         "run without events and an identical K-step pass right after carries them")
    return ap.parse_args()


def cpu_baseline(sample_sec: float):
    """Time the CPU oracle (test infrastructure: oracle/) on a bounded sample of the same workload."""
    from oracle.pipeline import OraclePipeline
    from rvcx import synthetic
    from rvcx.config import HUBERT_BASE, RMVPE_CFG, SYNTH_48K_V2
    from rvcx.weights import normalize_state

    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    sw = normalize_state(synthetic.synth_state(2))
    hw = normalize_state(synthetic.hubert_state(4))
    rw = normalize_state(synthetic.rmvpe_state(5))
    p = OraclePipeline(48000, synth_w=sw, synth_cfg=SYNTH_48K_V2, hubert_w=hw, hubert_cfg=HUBERT_BASE, rmvpe_w=rw,
                       rmvpe_cfg=RMVPE_CFG)
    n = int(sample_sec * SR_IN)
    audio = synthetic.speech_like(n, seed=1)
    p.pipeline(0, audio.copy(), protect=0.33)  # warm-up
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        p.pipeline(0, audio.copy(), protect=0.33)
        ts.append(time.perf_counter() - t0)
    med = statistics.median(ts)
    return {"value": round(sample_sec / med, 4), "unit": "audio-sec/sec", "cores": threads, "kind": "port",
            "sample": f"oracle Pipeline.pipeline (torch-CPU fp32, {threads} threads) on a {sample_sec:.1f} s "
                      f"speech-like clip, x_pad=1, median of 3 after 1 warm-up ({med:.2f} s/run)"}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)

    from scipy import signal

    from rvcx import synthetic
    from rvcx.config import SYNTH_48K_V2
    from rvcx.engine import Engine
    from rvcx.weights import normalize_state

    eng = Engine(local)
    eng.load_synth(normalize_state(synthetic.synth_state(2)), SYNTH_48K_V2)
    eng.load_hubert(normalize_state(synthetic.hubert_state(4)))
    eng.load_rmvpe(normalize_state(synthetic.rmvpe_state(5)))
    b, a = signal.butter(N=5, Wn=48, btype="high", fs=SR_IN)
    eng.set_highpass(b, a, signal.lfilter_zi(b, a))

    n = args.samples
    audio = torch.as_tensor(synthetic.speech_like(n, seed=1000 + rank), dtype=torch.float64, device=dev)
    t_pad, t_pad_tgt = SR_IN * 1, 48000 * 1
    cap = ((n + 2 * t_pad) // 160) * eng.upp
    out = torch.empty((cap,), dtype=torch.float32, device=dev)

    def step(i):
        return eng.pipeline(audio, sid=0, semitones=0.0, protect=0.33, t_pad=t_pad, t_pad_tgt=t_pad_tgt,
                            seed=1234 + i, out=out)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize(dev)
    eng.profile_read()  # drop anything recorded so far
    eng.profile(args.roofline_pass == "inline")
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        y = step(args.warmup + i)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    eng.profile(False)
    if args.roofline_pass == "after":
        eng.profile(True)
        for i in range(args.steps):
            step(args.warmup + i)
        eng.profile(False)
    k_ms, k_flops, k_launches = eng.profile_read()
    from rvcx.sharding import reduce_throughput

    audio_sec = n / SR_IN
    # whole job: audio-seconds summed over ranks / wall time maxed over ranks
    tot = reduce_throughput(dist, args.steps * audio_sec, t1 - t0, device=dev)
    elapsed = tot["elapsed"]
    ms_per_step = elapsed / args.steps * 1000.0
    value = tot["value"]
    assert y.numel() > 0 and bool(torch.isfinite(y).all())

    achieved_tflops = k_flops / (k_ms / 1000.0) / 1e12 if k_ms > 0 else 0.0
    roofline = {"bound": "mfma", "achieved": round(achieved_tflops, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved_tflops / FP32_PEAK_TFLOPS, 4), "traffic": None,
                "kernel": "conv_gemm_kernel (fp32 MFMA implicit-GEMM; all launches of the step)",
                "launches_per_step": k_launches // max(1, args.steps),
                "kernel_ms_per_step": round(k_ms / args.steps, 3),
                "alg_gflop_per_step": round(k_flops / args.steps / 1e9, 2)}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args.cpu_sample_sec)
        except Exception as e:  # reported, never fatal
            cpu = {"error": repr(e)}
    if rank == 0:
        rec = {
            "metric": "audio-sec/sec (realtime factor) RVCv2 48kHz pipeline",
            "value": round(value, 3), "unit": "audio-sec/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic (speech-like, seeded); "
            "random-init weights of the RVCv2-48k / ContentVec / RMVPE architectures",
            "config": {"workload": "C2: full RVCv2 48kHz pipeline, one 13.5 s utterance per step per GPU",
                       "samples_16k": n, "audio_sec_per_step_per_gpu": round(audio_sec, 5), "x_pad": 1,
                       "f0_method": "rmvpe", "index_rate": 0, "protect": 0.33, "parallelism": f"dp{world}"},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        print(json.dumps(rec))
    if dist:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
