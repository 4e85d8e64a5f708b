"""Time the fused ResBlock pair (rvcx_resblock_pair) at the C2 generator shapes, per tile configuration, beside
the two plain contractions of the unfused path (two rvcx_conv1d launches, activations not included: a lower
bound on the unfused pair). Prints TFLOP/s of the pair's algorithmic work (2 convs x 2*T*C*C*k).

usage: python tools/bench_rb.py [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "retrieval-based-voice-conversion-mlx_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rvcx.engine import Engine  # noqa: E402

SHAPES = [  # T, C, k, d  (C2: 1550 frames; stages 2-4 at x120, x240, x480)
    (744000, 32, 3, 1), (744000, 32, 7, 3), (744000, 32, 11, 5),
    (372000, 64, 3, 1), (372000, 64, 7, 3), (372000, 64, 11, 5),

]
CFGS = {32: (1, 2), 64: (1, 2), 128: ()}


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def one(argv):
    """--one T C k d cfg reps: only the fused kernel at one shape (for rocprofv3 --pmc passes, tools/pmc_rb.sh)"""
    T, C, k, d, cfg, reps = (int(v) for v in argv)
    eng = Engine(0)
    dev = eng.device
    x = torch.randn((1, T, C), device=dev)
    w1 = torch.randn((C, C, k), device=dev) / np.sqrt(C * k)
    w2 = torch.randn((C, C, k), device=dev) / np.sqrt(C * k)
    b1 = torch.randn(C, device=dev) * 0.1
    b2 = torch.randn(C, device=dev) * 0.1
    ms = timeit(lambda: eng.resblock_pair(x, w1, b1, w2, b2, d, cfg=cfg), reps)
    print(f"T={T} C={C} k={k} d={d} cfg{cfg}: {ms * 1e3:.1f} us {2 * 2.0 * T * C * C * k / ms / 1e9:.1f} TF")
    eng.close()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        return one(sys.argv[2:])
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    eng = Engine(0)
    dev = eng.device
    rng = np.random.Generator(np.random.PCG64(0))
    for T, C, k, d in SHAPES:
        x = torch.randn((1, T, C), device=dev)
        w1 = torch.randn((C, C, k), device=dev) / np.sqrt(C * k)
        w2 = torch.randn((C, C, k), device=dev) / np.sqrt(C * k)
        b1 = torch.randn(C, device=dev) * 0.1
        b2 = torch.randn(C, device=dev) * 0.1
        fl = 2 * 2.0 * T * C * C * k
        line = f"T={T:7d} C={C:3d} k={k:2d} d={d}:"
        for cfg in CFGS[C]:
            ms = timeit(lambda: eng.resblock_pair(x, w1, b1, w2, b2, d, cfg=cfg), reps)
            line += f"  cfg{cfg} {ms * 1e3:7.1f} us {fl / ms / 1e9:6.1f} TF"
        x2 = x[0]
        ms = timeit(lambda: (eng.conv1d(x2, w1, b1, dilation=d, padding=d * (k - 1) // 2),
                             eng.conv1d(x2, w2, b2, padding=(k - 1) // 2)), reps)
        line += f"  | 2x conv1d {ms * 1e3:7.1f} us {fl / ms / 1e9:6.1f} TF"
        print(line, flush=True)
    del rng
    eng.close()


if __name__ == "__main__":
    main()
