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
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "retrieval-based-voice-conversion-mlx_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense FP32 (vector = f32-in MFMA)
BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense BF16 / FP16 MFMA (no sparsity)
# The convs run fp32-accurate contractions as several half-width MFMA plane products: six bf16 products (the exact
# 3-plane split: ceiling 2500 / 6 = 416.7 TF of algorithmic fp32) or, in the generator's weight-streamed convs and
# fused ResBlock pairs, three fp16 products (the two-plane split: 2500 / 3 = 833.3 TF). Each launch is priced at its
# own arithmetic's ceiling (rvcx_profile_read_ex); the few launches on the native f32 MFMA (157.3) are priced at the
# split's, which keeps frac a lower bound.
SPLIT_PEAK_TFLOPS = round(BF16_PEAK_TFLOPS / 6.0, 1)
H16_PEAK_TFLOPS = round(BF16_PEAK_TFLOPS / 3.0, 1)
CONV_KERNEL = ("conv_wsb16_kernel / conv_gs16_kernel / conv_gsw16_kernel / k_rb_pair / conv_emu_kernel / conv_gemm_kernel / "
               "conv_tiny_kernel / conv_tiny_rows_kernel / k_conv2d_small / k_conv2d_h16 "
               "(+ splitk_reduce): every conv, linear and matmul launch of the step, Σ algorithmic fp32 FLOPs / Σ "
               "HIP-event kernel time")
SR_IN = 16000
C2_SAMPLES = 216100  # 13.50625 s (the reference's 13.5 s benchmark clip length)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--samples", type=int, default=C2_SAMPLES)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5"], default="c2",
                    help="c2 (default, the headline line): full pipeline, 13.5 s utterance per step; c3: HiFiGAN-NSF "
                         "generator alone, B=32 x 400 frames per step; c5: 16 realtime streams, one 256 ms hop per step")
    ap.add_argument("--streams", type=int, default=16, help="c5: concurrent streams")
    ap.add_argument("--gen-precision", choices=["fp32", "fp16"], default="fp32",
                    help="c5: each hop's generator on fp16 operands (rvcx_rt_opts.gen_precision, BASELINE C5's fp16; "
                         "gated by tests/test_gpu_stream_ref.py at spectrogram corr >= 0.986)")
    ap.add_argument("--batch", type=int, default=8, help="c4: 30 s utterances per batched pipeline pass")
    ap.add_argument("--c4-utterances", type=int, default=512, help="c4: job size (BASELINE configs[3]: 512)")
    ap.add_argument("--selftest-launch", action="store_true",
                    help="exercise the --gpus N self-launch and the collectives on the CPU (RVCX_DIST_BACKEND=gloo): "
                         "every rank runs a tiny host loop instead of the device pipeline; no GPU is touched")
    ap.add_argument("--roofline-pass", choices=["inline", "after"], default="after",
                    help="inline: HIP events around every conv launch of the timed steps; after: the timed steps "
                         "run without events and an identical K-step pass right after carries them")
    a = ap.parse_args()
    a.steps_given = a.steps is not None
    if a.steps is None:
        a.steps = 10
    return a


def _host_cpu():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return model, os.cpu_count() or 1, avail


def cpu_baseline(n_samples: int, reps: int = 3):
    """Time the CPU oracle (test infrastructure: oracle/) on the SAME C2 workload: the 13.5 s clip through
    Pipeline.pipeline (x_pad = 1), median of 3 after a 2 s warm-up call; plus C1 (RMVPE f0 of the
    5 s benchmark_rmvpe.py clip, BASELINE configs[0]). torch-CPU fp32 on every CPU this process may run on
    (sched_getaffinity), capped at the GPU box's per-GPU CPU share (OMP_NUM_THREADS: 16 there; the box's rules
    forbid sizing a pool by os.cpu_count(), which counts the whole 256-CPU host that every GPU slot shares)."""
    from oracle import rmvpe as ormvpe
    from oracle.pipeline import OraclePipeline
    from rvcx import synthetic
    from rvcx.config import HUBERT_BASE, RMVPE_CFG, SYNTH_48K_V2
    from rvcx.weights import normalize_state

    model, ncpu, avail = _host_cpu()
    # one GPU's share of the host: the GPU box gives each 1-GPU job 16 CPUs (OMP_NUM_THREADS=16 there); the host's
    # 256 logical CPUs serve every GPU slot, so os.cpu_count() would oversubscribe them
    try:
        share = int(os.environ.get("OMP_NUM_THREADS", "16"))
    except ValueError:
        share = 16
    threads = max(1, min(share if share > 0 else 16, avail))
    torch.set_num_threads(threads)
    sw = normalize_state(synthetic.synth_state(2))
    hw = normalize_state(synthetic.hubert_state(4))
    rw = normalize_state(synthetic.rmvpe_state(5))
    p = OraclePipeline(48000, synth_w=sw, synth_cfg=SYNTH_48K_V2, hubert_w=hw, hubert_cfg=HUBERT_BASE, rmvpe_w=rw,
                       rmvpe_cfg=RMVPE_CFG)
    p.pipeline(0, synthetic.speech_like(2 * SR_IN, seed=1).copy(), protect=0.33)  # warm-up
    audio = synthetic.speech_like(n_samples, seed=1000)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        p.pipeline(0, audio.copy(), protect=0.33)
        ts.append(time.perf_counter() - t0)
    med = statistics.median(ts)
    sec = n_samples / SR_IN
    # C1: RMVPE0Predictor.infer_from_audio on the 5 s clip (0.3 sin 440 + 0.2 sin 880 + 0.1 N, seed 0)
    c1_audio = synthetic.rmvpe_bench_audio(80000, seed=0)
    ormvpe.infer_from_audio(p.rw, p.rc, c1_audio, thred=0.03)
    c1 = []
    for _ in range(5):
        t0 = time.perf_counter()
        ormvpe.infer_from_audio(p.rw, p.rc, c1_audio, thred=0.03)
        c1.append(time.perf_counter() - t0)
    c1m = statistics.median(c1)
    return {"value": round(sec / med, 4), "unit": "audio-sec/sec", "cores": threads, "kind": "port",
            "sample": f"oracle Pipeline.pipeline (torch-CPU fp32, {threads} threads) on the C2 clip itself "
                      f"({sec:.2f} s, x_pad=1), median of {reps} after a 2 s warm-up ({med:.2f} s/run)",
            "host_cpu": model, "host_logical_cpus": ncpu, "host_cpus_available": avail,
            "threads_basis": "OMP_NUM_THREADS (16 on the GPU box: one GPU's CPU share), capped by the CPUs available",
            "c1": {"value": round(5.0 / c1m, 3), "unit": "audio-sec/sec", "sec_per_clip": round(c1m, 4),
                   "sample": "C1: oracle RMVPE0Predictor.infer_from_audio on the 5 s benchmark_rmvpe.py clip, "
                             "median of 5"}}


def _pmc_family_traffic(name):
    """HBM bytes per launch of one kernel family from profiles/pmc_traffic.json (its "families" table, the same PMC
    passes as _pmc_traffic), only when measured on this exact source tree; else None."""
    from rvcx.provenance import source_tree_hash

    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    if rec.get("tree") != source_tree_hash():
        return None
    fam = (rec.get("families") or {}).get(name)
    return round(fam["hbm_bytes_per_launch"]) if fam else None


def _dominant(fams, steps):
    """The kernel family with the most event time per step, priced at its own arithmetic's ceiling."""
    name, f = max(fams.items(), key=lambda kv: kv[1]["ms"])
    ms = f["ms"] / steps
    tf = f["flops"] / (f["ms"] / 1e3) / 1e12 if f["ms"] > 0 else 0.0
    ceil = f["flops"] / (f["ceiling_ms"] / 1e3) / 1e12 if f["ceiling_ms"] > 0 else SPLIT_PEAK_TFLOPS
    per_launch_ms = f["ms"] / max(1, f["launches"])
    return {"kernel": name, "gflop_per_step": round(f["flops"] / steps / 1e9, 2), "ms_per_step": round(ms, 3),
            "tflops": round(tf, 3), "ceiling_tflops": round(ceil, 1), "frac": round(tf / ceil, 4) if ceil else None,
            "launches_per_step": f["launches"] // max(1, steps), "avg_launch_us": round(per_launch_ms * 1e3, 2),
            "alg_bytes_per_launch": round(f["bytes"] / max(1, f["launches"])),
            "traffic_bytes_per_launch": _pmc_family_traffic(name)}


def _pmc_traffic():
    """HBM bytes per conv-GEMM launch from the committed PMC passes (tools/pmc_traffic.sh + pmc_traffic.py:
    FETCH_SIZE and WRITE_SIZE in separate rocprofv3 runs of this bench, FETCH_SIZE doubled per
    MI355X_MICROARCH.md). PMC counters cannot be read from inside the timed process, so the number comes from
    profiles/pmc_traffic.json -- and only when that file was measured on this exact source tree (its "tree"
    equals rvcx.provenance.source_tree_hash()); otherwise None."""
    from rvcx.provenance import source_tree_hash

    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None, "profiles/pmc_traffic.json absent"
    tree = source_tree_hash()
    if rec.get("tree") != tree:
        return None, f"profiles/pmc_traffic.json is from tree {rec.get('tree')}, not this tree {tree}"
    step = None
    if rec.get("step_hbm_bytes") and rec.get("step_alg_bytes"):
        step = {"hbm_bytes": round(rec["step_hbm_bytes"]), "alg_bytes": round(rec["step_alg_bytes"]),
                "ratio": round(rec["step_hbm_bytes"] / rec["step_alg_bytes"], 3)}
    return (round(rec["traffic_bytes_per_launch"]), step), f"profiles/pmc_traffic.json (tree {tree}, {rec.get('file')})"


def _timed(step, args, dev, dist):
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    return time.perf_counter() - t0


def bench_c3(args, eng, dev, dist, rank, world):
    """configs[2]: HiFiGAN-NSF generator alone, batch 32 x 400 frames of random z, f0 walk, sid 0."""
    from rvcx import synthetic
    from rvcx.sharding import reduce_throughput

    B, T = 32, 400
    rng = np.random.Generator(np.random.PCG64(3))
    z = torch.as_tensor(rng.standard_normal((B, 192, T)).astype(np.float32), device=dev)
    f0 = torch.as_tensor(synthetic.f0_walk(B, T, seed=3), dtype=torch.float32, device=dev)
    sid = torch.zeros(B, dtype=torch.int32, device=dev)
    el = _timed(lambda i: eng.dec_only(z, f0, sid, seed=i), args, dev, dist)
    eng.check_device_status()
    # roofline: an identical K-step pass right after the timed one carries the per-conv events (they are not
    # in the timed region)
    eng.profile_read()
    eng.profile(True)
    for i in range(args.steps):
        eng.dec_only(z, f0, sid, seed=args.warmup + i)
    eng.profile(False)
    k_ms, k_flops, k_n, c_ms = eng.profile_read(with_ceiling=True)
    audio_sec = B * T * eng.upp / 48000.0
    tot = reduce_throughput(dist, args.steps * audio_sec, el, device=dev)
    tf = k_flops / (k_ms / 1e3) / 1e12 if k_ms > 0 else 0.0
    peak = k_flops / (c_ms / 1e3) / 1e12 if c_ms > 0 else SPLIT_PEAK_TFLOPS
    return {"metric": "audio-sec/sec HiFiGAN-NSF generator (C3)", "value": round(tot["value"], 3),
            "unit": "audio-sec/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(tot["elapsed"] / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32-accurate (two-plane fp16 MFMA split)", "data": "synthetic z ~ N(0,1), f0 random walk; random-init weights",
            "config": {"workload": "C3: generator alone, B=32 x 400 frames (128 s of 48 kHz audio) per step",
                       "parallelism": f"dp{world}"},
            "roofline": {"bound": "mfma", "achieved": round(tf, 3), "peak": round(peak, 1), "unit": "TFLOP/s",
                         "frac": round(tf / peak, 4), "traffic": None,
                         "peak_basis": "FLOP-weighted MFMA ceiling of the launches' arithmetic: dense 2500 TF / 3 "
                                       "products (two-plane fp16 split, the generator) or / 6 (three-plane bf16 split)",
                         "kernel": CONV_KERNEL + " (events on a separate K-step pass after the timed one)",
                         "alg_gflop_per_step": round(k_flops / args.steps / 1e9, 2)}}


def _c4_row(arg):
    n, seed = arg
    from rvcx import synthetic

    return synthetic.speech_like(n, seed=seed)


def c4_audio(job, ids, n, dev, workers=16):
    """Device audio [len(ids), n] fp64 of this rank's C4 utterances: speech_like(n, seed=1000 + i) per utterance
    (Utterance.seed), made by a pool of host processes (spawned: no GPU state is inherited; at most 16,
    the GPU box's CPU share) -- ~0.15 s of host time per 30 s clip."""
    import multiprocessing as mp

    args = [(n, job[i].seed) for i in ids]
    nw = max(1, min(workers, os.cpu_count() or 1, len(args)))
    if nw == 1:
        rows = [_c4_row(a) for a in args]
    else:
        with mp.get_context("spawn").Pool(nw) as pool:
            rows = pool.map(_c4_row, args, chunksize=max(1, len(args) // (4 * nw)))
    return torch.as_tensor(np.stack(rows), dtype=torch.float64, device=dev)


def bench_c4(args, eng, dev, dist, rank, world):
    """configs[3]: batched offline VC of the 512 x 30 s job (rvcx.offline). Every rank builds the same job
    list, takes its LPT shard (i::world for equal lengths, extract.py:101-117) and converts it in batched
    passes of --batch utterances (rvcx_pipeline_batch); one step = one pass. RCCL carries only bookkeeping:
    SUM/MAX of audio-seconds and wall time and an all_gather of the per-utterance records. Timed: the whole
    shard (or the first --steps passes when given), after --warmup untimed passes of the shard's first batch."""
    from rvcx import offline

    job = offline.c4_job(args.c4_utterances)
    p = offline.plan(job, world, rank, args.batch)
    n = job[0].n
    pos = {u: k for k, u in enumerate(p.shard)}
    audio = c4_audio(job, p.shard, n, dev)
    opts = eng.pipeline_opts(protect=0.33)
    ldo = ((n + 2 * int(opts.t_pad)) // 160) * eng.upp
    out = torch.empty((args.batch, ldo), dtype=torch.float32, device=dev)

    def convert(ids, step):
        rows = torch.tensor([pos[i] for i in ids], device=dev)
        y = eng.pipeline_batch(audio.index_select(0, rows), opts, sids=0, seed=step, out=out)
        rec = torch.empty((len(ids), 4), dtype=torch.float64, device=dev)
        rec[:, 0] = torch.tensor(ids, dtype=torch.float64, device=dev)
        rec[:, 1] = float(y.shape[1])
        rec[:, 2] = y.abs().amax(1).double()
        rec[:, 3] = y.double().pow(2).mean(1).sqrt()
        return rec

    for w in range(args.warmup):
        convert(p.batches[0], -1 - w)
    recs, el = offline.run(p, convert, sync=lambda: torch.cuda.synchronize(dev), dist=dist,
                           steps=args.steps if args.steps_given else None)
    eng.check_device_status()
    tot = offline.finish(p, job, recs, el, dist=dist, device=dev)
    nsteps = len(recs)
    r = tot["records"]
    assert bool(torch.isfinite(r).all()) and bool((r[:, 2] > 0).all()), "non-finite or silent C4 output"
    return {"metric": "audio-sec/sec batched offline VC (C4)", "value": round(tot["value"], 3),
            "unit": "audio-sec/sec", "n_gpus": world, "steps": nsteps, "warmup": args.warmup,
            "ms_per_step": round(tot["elapsed"] / max(1, nsteps) * 1e3, 3), "higher_is_better": True,
            "scaling": "weak" if args.steps_given else "strong", "vs_baseline": None, "dtype": "fp32-accurate (two-plane fp16 MFMA split)",
            "data": "synthetic speech-like 30 s utterances (speech_like(seed=1000+i) per utterance); random-init "
                    "weights",
            "config": {"workload": f"C4: {len(job)} x 30 s utterances, LPT-sharded over {world} GPU(s), batched "
                                   f"passes of {args.batch}", "utterances_converted": tot["utterances"],
                       "batch": args.batch, "parallelism": f"dp{world}"}}


def bench_c5(args, eng, dev, dist, rank, world):
    """configs[4]: S concurrent realtime streams, 256 ms hops (read_chunk_size 96), one hop per step;
    latency = wall time of one hop for all streams (input and output in HBM)."""
    from rvcx import synthetic
    from rvcx.realtime import StreamGroup
    from rvcx.sharding import reduce_throughput

    S = args.streams
    grp = StreamGroup(eng, S, read_chunk_size=96, cross_fade_overlap_size=0.1, extra_convert_size=0.5,
                      silent_threshold=-90.0)
    block = grp.block_frame
    nh = args.warmup + args.steps
    audio = np.stack([synthetic.speech_like(block * nh, seed=500 + 100 * rank + s, sr=48000).astype(np.float32)
                      for s in range(S)])
    x = torch.as_tensor(audio, device=dev)
    opts = grp.opts(protect=0.5, gen_precision=args.gen_precision)
    lat = []

    def step(i):
        t0 = time.perf_counter()
        grp.process(x[:, i * block:(i + 1) * block], opts, seed=i)
        torch.cuda.synchronize(dev)
        lat.append(time.perf_counter() - t0)

    el = _timed(step, args, dev, dist)
    eng.check_device_status()
    lat = np.array(lat[args.warmup:]) * 1e3
    hop_sec = block / 48000.0
    tot = reduce_throughput(dist, args.steps * S * hop_sec, el, device=dev)
    grp.close()
    return {"metric": "audio-sec/sec streaming VC (C5), hop latency p50/p99", "value": round(tot["value"], 3),
            "unit": "audio-sec/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(tot["elapsed"] / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("fp32-accurate (two-plane fp16 MFMA split)" if args.gen_precision == "fp32"
                      else "fp16 generator (fp32-accurate front end, TextEncoder, flow)"),
            "data": "synthetic speech-like 48 kHz streams; random-init weights",
            "config": {"workload": f"C5: {S} streams x 256 ms hop (block 12288 @48k, convert buffer 13920 @16k, "
                                   "87 frames) per step", "streams": S, "parallelism": f"dp{world}",
                       "generator_precision": args.gen_precision},
            "latency_ms": {"p50": round(float(np.percentile(lat, 50)), 3),
                           "p99": round(float(np.percentile(lat, 99)), 3), "budget": round(hop_sec * 1e3, 1)}}


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def self_launch(n: int) -> int:
    """`--gpus N` without an external launcher: start N fresh worker processes of this script, one per GPU, each
    with RANK = LOCAL_RANK = r, WORLD_SIZE = N and a 127.0.0.1 rendezvous, and wait for them (the reference's
    pattern: one process per device over files[i::len(devices)], rvc/train/extract/extract.py:101-117, :150-170).
    This process never touches the GPU (it only starts children; nothing is exec'd). Rank 0's stdout carries the
    JSON line. A worker that fails takes the others down (a rank left waiting at a barrier would hang). Returns
    the first non-zero exit code, else 0."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
    return rc


def selftest_launch(args, rank, world):
    """--selftest-launch: the N-rank plumbing of main() (rendezvous, barrier-bracketed timing, SUM/MAX reduction,
    rank-0 JSON) with a host loop standing in for the device step."""
    import torch.distributed as dist

    from rvcx.sharding import gather_records, reduce_throughput

    dist.init_process_group(os.environ.get("RVCX_DIST_BACKEND", "gloo"))
    x = torch.ones(64, 64)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x = x @ x / 64.0
    dist.barrier()
    tot = reduce_throughput(dist, float(args.steps), time.perf_counter() - t0)
    pids = gather_records(dist, [(rank, os.getpid(), int(os.environ.get("LOCAL_RANK", "-1")))])
    if rank == 0:
        print(json.dumps({"metric": "launcher self-test (host loop, no GPU)", "value": round(tot["value"], 3),
                          "unit": "steps/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ranks": [list(p) for p in pids], "backend": dist.get_backend()}))
    dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.selftest_launch:
        return selftest_launch(args, rank, world)
    # one process per GPU; ranks beyond the visible GPUs wrap around (rehearsing N > 1 on a 1-GPU box
    # with RVCX_DIST_BACKEND=gloo) -- device_count() does not initialise the GPU
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    dist = None
    if world > 1:
        import torch.distributed as dist

        backend = os.environ.get("RVCX_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI on the MI355X node
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from rvcx import synthetic
    from rvcx.config import SYNTH_48K_V2
    from rvcx.engine import Engine
    from rvcx.weights import normalize_state

    eng = Engine(local)
    eng.load_synth(normalize_state(synthetic.synth_state(2)), SYNTH_48K_V2)
    eng.load_hubert(normalize_state(synthetic.hubert_state(4)))
    eng.load_rmvpe(normalize_state(synthetic.rmvpe_state(5)))
    eng.set_pipeline_highpass(SR_IN)
    if args.config in ("c3", "c4", "c5"):
        rec = {"c3": bench_c3, "c4": bench_c4, "c5": bench_c5}[args.config](args, eng, dev, dist, rank, world)
        if rank == 0:
            print(json.dumps(rec))
        if dist:
            dist.destroy_process_group()
        eng.close()
        return

    n = args.samples
    # the utterance in pinned host memory and resident in HBM; the output buffer in HBM and pinned on the host
    audio_host = torch.as_tensor(synthetic.speech_like(n, seed=1000 + rank), dtype=torch.float64).pin_memory()
    audio = audio_host.to(dev)
    t_pad, t_pad_tgt = SR_IN * 1, 48000 * 1
    cap = ((n + 2 * t_pad) // 160) * eng.upp
    out = torch.empty((cap,), dtype=torch.float32, device=dev)
    out_host = torch.empty((cap,), dtype=torch.float32).pin_memory()

    def step(i, host_io=False):
        # host_io: SURVEY §8(d)'s host audio-in -> audio-out, the H2D and D2H copies on the compute stream
        if host_io:
            audio.copy_(audio_host, non_blocking=True)
        y = eng.pipeline(audio, sid=0, semitones=0.0, protect=0.33, t_pad=t_pad, t_pad_tgt=t_pad_tgt,
                         seed=1234 + i, out=out)
        if host_io:
            out_host[: y.numel()].copy_(y, non_blocking=True)
        return y

    for i in range(args.warmup):
        step(i, host_io=True)
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
    # the same K steps from pinned host input to pinned host output (PCIe-inclusive; reported beside value)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    th0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, host_io=True)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    th1 = time.perf_counter()
    if args.roofline_pass == "after":
        eng.profile(True)
        for i in range(args.steps):
            step(args.warmup + i)
        eng.profile(False)
    (k_ms, k_flops, k_launches, c_ms), fams = eng.profile_read_kinds()
    eng.check_device_status()  # a device-side fault flag (BiGRU hand-off) voids the run
    from rvcx.sharding import reduce_throughput

    audio_sec = n / SR_IN
    # whole job: audio-seconds summed over ranks / wall time maxed over ranks
    tot = reduce_throughput(dist, args.steps * audio_sec, t1 - t0, device=dev)
    tot_io = reduce_throughput(dist, args.steps * audio_sec, th1 - th0, device=dev)
    elapsed = tot["elapsed"]
    ms_per_step = elapsed / args.steps * 1000.0
    value = tot["value"]
    assert y.numel() > 0 and bool(torch.isfinite(y).all())

    achieved_tflops = k_flops / (k_ms / 1000.0) / 1e12 if k_ms > 0 else 0.0
    # FLOP-weighted ceiling of the launches' own arithmetic: the launches' time at their ceilings / their time
    peak = k_flops / (c_ms / 1000.0) / 1e12 if c_ms > 0 else SPLIT_PEAK_TFLOPS
    traffic, traffic_src = _pmc_traffic()
    _, traffic_step = traffic if traffic else (None, None)
    dom = _dominant(fams, args.steps)
    # the line's roofline is the DOMINANT kernel's (the family with the most time per step, priced at its own
    # arithmetic's ceiling; traffic = its PMC-measured HBM bytes per launch); the whole conv family's aggregate rides
    # along under "family"
    roofline = {"bound": "mfma", "achieved": dom["tflops"], "peak": dom["ceiling_tflops"], "unit": "TFLOP/s",
                "frac": dom["frac"], "traffic": dom["traffic_bytes_per_launch"],
                "traffic_unit": f"HBM bytes per {dom['kernel']} launch (PMC FETCH_SIZE x2 + WRITE_SIZE, "
                                f"profiles/pmc_traffic.json families; algorithmic {dom['alg_bytes_per_launch']} B)",
                "kernel": dom["kernel"], "dominant": dom,
                "peak_basis": "MFMA ceiling of the launch's fp32-accurate arithmetic: dense fp16/bf16 2500 TF / 3 plane "
                              f"products ({H16_PEAK_TFLOPS}: the two-plane fp16 split) or / 6 ({SPLIT_PEAK_TFLOPS}: the "
                              f"three-plane bf16 split); native f32 MFMA peak {FP32_PEAK_TFLOPS}",
                "family": {"kernel": CONV_KERNEL, "achieved": round(achieved_tflops, 3), "peak": round(peak, 1),
                           "frac": round(achieved_tflops / peak, 4),
                           "launches_per_step": k_launches // max(1, args.steps),
                           "kernel_ms_per_step": round(k_ms / args.steps, 3),
                           "alg_gflop_per_step": round(k_flops / args.steps / 1e9, 2),
                           # the family's measured HBM bytes per C2 step against its algorithmic bytes (operands read
                           # once, result written once), the same PMC record
                           "traffic_step": traffic_step, "traffic_source": traffic_src,
                           "by_kernel_ms_per_step": {k: round(v["ms"] / args.steps, 3) for k, v in
                                                     sorted(fams.items(), key=lambda kv: -kv[1]["ms"])}}}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(n)
        except Exception as e:  # reported, never fatal
            cpu = {"error": repr(e)}
    if rank == 0:
        rec = {
            "metric": "audio-sec/sec (realtime factor) RVCv2 48kHz pipeline",
            "value": round(value, 3), "unit": "audio-sec/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32-accurate (two-plane fp16 MFMA split)", "data": "synthetic (speech-like, seeded); "
            "random-init weights of the RVCv2-48k / ContentVec / RMVPE architectures",
            "config": {"workload": "C2: full RVCv2 48kHz pipeline, one 13.5 s utterance per step per GPU",
                       "samples_16k": n, "audio_sec_per_step_per_gpu": round(audio_sec, 5), "x_pad": 1,
                       "f0_method": "rmvpe", "index_rate": 0, "protect": 0.33, "parallelism": f"dp{world}"},
            "roofline": roofline, "cpu_baseline": cpu, "effective_config": eng.config_info(),
            # SURVEY §8(d)'s definition: pinned host audio in -> pinned host audio out, the H2D (1.7 MB fp64) and
            # D2H (2.6 MB fp32) copies on the compute stream inside the timed loop; value above is HBM-resident
            "host_io": {"value": round(tot_io["value"], 3), "unit": "audio-sec/sec",
                        "ms_per_step": round(tot_io["elapsed"] / args.steps * 1000.0, 3),
                        "timed": "pinned host input -> H2D -> pipeline -> D2H -> pinned host output, same K steps"},
        }
        print(json.dumps(rec))
    if dist:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
