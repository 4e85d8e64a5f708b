"""Copy the reference's own golden DATA (ios_test_data/*.npy) into one fixture.

Run in the survey container only:  python tests/golden/copy_reference_fixtures.py
Source: /root/reference/ios_test_data (produced by tools/export_ios_test_data.py:39-147
from the MLX path). Only data arrays are copied: the RMVPE salience ``rmvpe_hidden``
with its decoded ``rmvpe_f0`` (the decode known-answer test) and the 13.5 s speech
clip ``input_audio`` used as a real-speech C2 input.
"""
import os

import numpy as np

SRC = "/root/reference/ios_test_data"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ios_kat.npz")

if __name__ == "__main__":
    np.savez_compressed(
        OUT,
        rmvpe_hidden=np.load(os.path.join(SRC, "rmvpe_hidden.npy")),
        rmvpe_f0=np.load(os.path.join(SRC, "rmvpe_f0.npy")),
        input_audio=np.load(os.path.join(SRC, "input_audio.npy")),
    )
    print("wrote", OUT, os.path.getsize(OUT))
