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


def refinegan_noise(g):
    import numpy as np

    """Regenerate the fixture's RNG draws (make_golden_vocoders.py refinegan): z noise, then the flat C-ABI source
    noise = source randn, initial phase (torch.rand), 24 AdaIN draws."""
    rng = np.random.Generator(np.random.PCG64(int(g["noise_seed"])))
    draws = [rng.standard_normal(int(n)).astype(np.float32) for n in g["draw_sizes"]]
    ini = np.random.Generator(np.random.PCG64(int(g["uniform_seed"]))).random(int(g["phone"].shape[0]))
    eps_src = np.concatenate([draws[1], ini.astype(np.float32)] + draws[2:])
    return draws[0], eps_src


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


def fixture_noise(g):
    """The reference run's injected noise of a fixture that stores only its seed (make_golden.NoiseStream:
    PCG64 standard normals as float32, eps_z then eps_src), flattened to the device layout ([192*T], [T*upp])."""
    import numpy as np

    rng = np.random.Generator(np.random.PCG64(int(g["noise_seed"])))
    ez = rng.standard_normal(tuple(g["eps_z_shape"])).astype(np.float32)
    es = rng.standard_normal(tuple(g["eps_src_shape"])).astype(np.float32)
    s = g["eps_sum"]
    assert abs(float(ez.astype(np.float64).sum()) - s[0]) < 1e-6 * max(1.0, abs(s[0]))
    assert abs(float(es.astype(np.float64).sum()) - s[1]) < 1e-6 * max(1.0, abs(s[1]))
    return ez.reshape(-1), es.reshape(-1)


def c2_audio(name):
    """The 13.5 s input of pipeline_c2_<name>.npz: the reference's ios_test_data clip or the bench clip."""
    import numpy as np

    if name == "ios":
        return golden("ios_kat.npz")["input_audio"].astype(np.float64)
    return golden("pipeline_c2_synth.npz")["audio32"].astype(np.float64)
