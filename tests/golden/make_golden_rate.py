"""Golden vectors for Synthesizer.infer(rate=) from the REFERENCE itself (survey container only; VERDICT r5 missing #2).

Run:  python tests/golden/make_golden_rate.py     (needs /root/reference; never on the GPU box)

rvc/lib/algorithm/synthesizers.py:230-234 keeps z_p[:, :, head:], x_mask[:, :, head:] and nsff0[:, head:] with
head = int(T * (1.0 - rate.item())) before the flow. The rates below cover a fraction (0.5), a float32 rate whose
product with T is not exact (0.3), rate 1 (head 0) and rate > 1, where head is negative and Python's slice keeps the
LAST -head frames (1.5). Each case records the reference's own noise draws (torch.randn_like patched to a seeded
numpy stream: the z_p noise over all T frames, then the decoder's over the kept ones) and its whole return value.
Weights are regenerated from the seeds of make_golden.py (rvcx.synthetic).
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402  (imports torch and transformers first, sets the repo paths)
import torch  # noqa: E402

from rvcx import synthetic  # noqa: E402

RATES = (0.5, 0.3, 1.0, 1.5)
SEED_INPUTS, SEED_NOISE = 21, 23


def main():
    mg.install_stubs()
    sys.path.insert(0, mg.REF)
    os.chdir(tempfile.mkdtemp(prefix="rvc_golden_rate_"))
    torch.manual_seed(0)
    net = mg.build_synth()
    rng = np.random.Generator(np.random.PCG64(SEED_INPUTS))
    T = 64
    phone = rng.standard_normal((1, T, 768)).astype(np.float32)
    f0 = synthetic.f0_walk(1, T, seed=SEED_INPUTS)
    pitch = rng.integers(1, 256, size=(1, T)).astype(np.int64)
    lengths = np.array([T], np.int64)
    sid = np.array([5], np.int64)
    out = {"phone": phone, "f0": f0, "pitch": pitch, "lengths": lengths, "sid": sid,
           "rates": np.array(RATES, np.float32)}
    orig = torch.randn_like
    for i, rate in enumerate(RATES):
        ns = mg.NoiseStream(SEED_NOISE + i)
        torch.randn_like = ns
        try:
            with torch.no_grad():
                o, x_mask, (z, z_p, m_p, logs_p) = net.infer(
                    torch.from_numpy(phone), torch.from_numpy(lengths), torch.from_numpy(pitch),
                    torch.from_numpy(f0), torch.from_numpy(sid), rate=torch.tensor([rate], dtype=torch.float32))
        finally:
            torch.randn_like = orig
        kept = int(z_p.shape[2])
        print(f"rate {rate}: kept {kept} of {T} frames, o {tuple(o.shape)}")
        out.update({f"eps_z{i}": ns.draws[0], f"eps_src{i}": ns.draws[1].reshape(1, -1), f"o{i}": o.numpy(),
                    f"z{i}": z.numpy(), f"z_p{i}": z_p.numpy(), f"m_p{i}": m_p.numpy(), f"logs_p{i}": logs_p.numpy(),
                    f"mask{i}": x_mask.numpy(), f"kept{i}": np.array(kept)})
    np.savez_compressed(os.path.join(mg.OUT, "synth_rate_t64.npz"), **out)


if __name__ == "__main__":
    main()
