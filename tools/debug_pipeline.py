"""Debug: device pipeline intermediates vs the oracle on the 2.5 s golden clip."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "retrieval-based-voice-conversion-mlx_amd"), ROOT]
import numpy as np
import torch
from scipy import signal

from rvcx import synthetic
from rvcx.config import SYNTH_48K_V2
from rvcx.engine import Engine
from rvcx.weights import normalize_state

g = np.load(os.path.join(ROOT, "tests/golden/pipeline_2p5s.npz"))
e = Engine(0)
e.load_synth(normalize_state(synthetic.synth_state(2)), SYNTH_48K_V2)
e.load_hubert(normalize_state(synthetic.hubert_state(4)))
e.load_rmvpe(normalize_state(synthetic.rmvpe_state(5)))
b, a = signal.butter(N=5, Wn=48, btype="high", fs=16000)
e.set_highpass(b, a, signal.lfilter_zi(b, a))
out, f0 = e.pipeline(g["audio"], sid=0, semitones=0, protect=0.33, t_pad=16000, t_pad_tgt=48000,
                     eps_z=g["eps_z"], eps_src=g["eps_src"], want_f0=True)
# host-filtered reference path through device models
filt = signal.filtfilt(b, a, g["audio"])
pad = np.pad(filt, (16000, 16000), mode="reflect")
f0h, hid = e.rmvpe(pad.astype(np.float32), 0.03, want_hidden=True)
feats = e.hubert(pad.astype(np.float32))
torch.cuda.synchronize()
np.savez(os.path.join(ROOT, "gpurun_out/debug_pipeline.npz"), out=out.cpu().numpy(), f0=f0.cpu().numpy(),
         f0h=f0h.cpu().numpy(), hid=hid.cpu().numpy(), feats=feats.cpu().numpy())
print("saved")
