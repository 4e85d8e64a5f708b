"""Wall time of the C2 front-end stages run ALONE on device (RMVPE, HuBERT) vs the whole pipeline step, so the
critical path can be attributed: python tools/time_stages.py [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "retrieval-based-voice-conversion-mlx_amd"), ROOT]
import torch  # noqa: E402

from rvcx import synthetic  # noqa: E402
from rvcx.config import SYNTH_48K_V2  # noqa: E402
from rvcx.engine import Engine  # noqa: E402
from rvcx.weights import normalize_state  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    eng = Engine(0)
    eng.load_synth(normalize_state(synthetic.synth_state(2)), SYNTH_48K_V2)
    eng.load_hubert(normalize_state(synthetic.hubert_state(4)))
    eng.load_rmvpe(normalize_state(synthetic.rmvpe_state(5)))
    eng.set_pipeline_highpass()
    audio = torch.as_tensor(synthetic.speech_like(216100, seed=1000), dtype=torch.float64, device="cuda:0")
    _, p32 = eng.highpass_pad(audio, 16000)
    out = torch.empty(((216100 + 32000) // 160) * eng.upp, dtype=torch.float32, device="cuda:0")
    res = {
        "pipeline": timeit(lambda: eng.pipeline(audio, protect=0.33, out=out), reps),
        "rmvpe": timeit(lambda: eng.rmvpe(p32), reps),
        "hubert": timeit(lambda: eng.hubert(p32), reps),
    }
    f0 = eng.rmvpe(p32)
    coarse, pitchf, _ = eng.f0_post(f0, 0.0)
    P = p32.shape[0] // 160
    res["voice_conversion"] = timeit(lambda: eng.voice_conversion(p32, coarse[:P], pitchf[:P], 0, 0.33), reps)
    eng.check_device_status()
    print(" ".join(f"{k} {v:.3f} ms" for k, v in res.items()))


if __name__ == "__main__":
    main()
