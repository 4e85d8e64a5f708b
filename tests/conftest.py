import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "retrieval-based-voice-conversion-mlx_amd")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")
    config.addinivalue_line("markers", "slow: long-running")


def golden(name):
    import numpy as np

    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def synth_w():
    from rvcx import synthetic
    from rvcx.weights import normalize_state

    return normalize_state(synthetic.synth_state(2))


@pytest.fixture(scope="session")
def hubert_w():
    from rvcx import synthetic
    from rvcx.weights import normalize_state

    return normalize_state(synthetic.hubert_state(4))


@pytest.fixture(scope="session")
def rmvpe_w():
    from rvcx import synthetic
    from rvcx.weights import normalize_state

    return normalize_state(synthetic.rmvpe_state(5))


@pytest.fixture(scope="session")
def engine(synth_w, hubert_w, rmvpe_w):
    """One device context with the seeded synthetic weights (GPU tests only)."""
    from rvcx.config import SYNTH_48K_V2
    from rvcx.engine import Engine

    e = Engine(0)
    e.load_synth(synth_w, SYNTH_48K_V2)
    e.load_hubert(hubert_w)
    e.load_rmvpe(rmvpe_w)
    yield e
    e.close()
