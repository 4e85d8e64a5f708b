"""Host issue time of one C2 step (engine.pipeline returns once every kernel is enqueued) against the GPU time of
the same step: a host-bound step shows issue time ~ GPU time. usage: python tools/host_issue.py [steps]"""
import sys
import time

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "retrieval-based-voice-conversion-mlx_amd")
from rvcx import synthetic  # noqa: E402
from rvcx.config import SYNTH_48K_V2  # noqa: E402
from rvcx.engine import Engine  # noqa: E402
from rvcx.weights import normalize_state  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
e = Engine(0)
e.load_synth(normalize_state(synthetic.synth_state(2)), SYNTH_48K_V2)
e.load_hubert(normalize_state(synthetic.hubert_state(4)))
e.load_rmvpe(normalize_state(synthetic.rmvpe_state(5)))
e.set_pipeline_highpass(16000)
n = 216100
audio = torch.as_tensor(synthetic.speech_like(n, seed=1000), dtype=torch.float64, device="cuda:0")
out = torch.empty((((n + 32000) // 160) * e.upp,), dtype=torch.float32, device="cuda:0")
for i in range(3):
    e.pipeline(audio, t_pad=16000, t_pad_tgt=48000, seed=i, out=out)
torch.cuda.synchronize()
issue, total = [], []
for i in range(steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.pipeline(audio, t_pad=16000, t_pad_tgt=48000, seed=i, out=out)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    issue.append((t1 - t0) * 1e3)
    total.append((t2 - t0) * 1e3)
issue.sort()
total.sort()
print(f"host issue per step: median {issue[len(issue) // 2]:.2f} ms (min {issue[0]:.2f}); issue + drain: median "
      f"{total[len(total) // 2]:.2f} ms")
e.close()
