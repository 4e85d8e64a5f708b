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
