"""Run one C2 stage alone, N times, for a rocprofv3 kernel trace: python tools/prof_stage.py {hubert|rmvpe|vc} [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "retrieval-based-voice-conversion-mlx_amd"), ROOT]
import torch  # noqa: E402

from rvcx import synthetic  # noqa: E402
from rvcx.config import SYNTH_48K_V2  # noqa: E402
from rvcx.engine import Engine  # noqa: E402
from rvcx.weights import normalize_state  # noqa: E402


def main():
    stage, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5
    eng = Engine(0)
    eng.load_synth(normalize_state(synthetic.synth_state(2)), SYNTH_48K_V2)
    eng.load_hubert(normalize_state(synthetic.hubert_state(4)))
    eng.load_rmvpe(normalize_state(synthetic.rmvpe_state(5)))
    eng.set_pipeline_highpass()
    audio = torch.as_tensor(synthetic.speech_like(216100, seed=1000), dtype=torch.float64, device="cuda:0")
    _, p32 = eng.highpass_pad(audio, 16000)
    f0 = eng.rmvpe(p32)
    coarse, pitchf, _ = eng.f0_post(f0, 0.0)
    P = p32.shape[0] // 160
    fn = {"hubert": lambda: eng.hubert(p32), "rmvpe": lambda: eng.rmvpe(p32),
          "vc": lambda: eng.voice_conversion(p32, coarse[:P], pitchf[:P], 0, 0.33)}[stage]
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    eng.check_device_status()


if __name__ == "__main__":
    main()
