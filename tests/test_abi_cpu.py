"""CPU-side checks of the C-ABI library: it exists, loads, and exports every symbol the header
declares (no compute calls: there is no GPU here)."""
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(REPO, "include", "rvcx.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(rvcx_[a-z0-9_]+)\s*\(", src, re.M)))


def test_header_lists_entry_points():
    syms = header_symbols()
    assert "rvcx_synth_infer" in syms and "rvcx_rmvpe" in syms and "rvcx_hubert" in syms
    assert len(syms) >= 12


def test_library_exports_every_header_symbol():
    from rvcx import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail(f"{_lib.LIB_PATH} missing: run __graft_entry__.build()")
    exported = set(_lib.exported_symbols())
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing
    assert set(_lib.EXPORTS) == set(header_symbols())


def test_engine_refuses_without_gpu():
    import torch

    from rvcx.engine import Engine

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        Engine(0)


def _ivf_bytes(nlist=4, direct_map=0):
    import numpy as np

    from oracle import ivf

    rng = np.random.default_rng(0)
    x = rng.standard_normal((300, 64)).astype(np.float32)
    return ivf.write_ivfflat(ivf.build_ivfflat(x, nlist=nlist, nprobe=2), sparse=False, direct_map=direct_map)


def test_index_parse_accepts_a_valid_file():
    """rvcx_index_parse (host only, the parser rvcx_index_load runs) on a well-formed IndexIVFFlat image."""
    from rvcx import _lib

    info = _lib.index_parse(_ivf_bytes())
    assert info == {"d": 64, "ntotal": 300, "nlist": 4, "nprobe": 2}


def test_index_parse_rejects_wrapping_list_sizes():
    """List sizes are untrusted: sizes whose sum wraps around 2^64 to ntotal, and whose byte counts
    (size * code_size) wrap to the true byte counts, must be refused (they would drive the device scan
    over ~2^63 rows)."""
    import struct

    from rvcx import _lib

    buf = bytearray(_ivf_bytes())
    at = buf.index(b"full") + 4
    (cnt,) = struct.unpack_from("<Q", buf, at)
    sizes = list(struct.unpack_from(f"<{cnt}Q", buf, at + 8))
    evil = list(sizes)
    evil[0] = (sizes[0] + (1 << 63)) % (1 << 64)
    evil[1] = (sizes[1] + (1 << 63)) % (1 << 64)
    assert sum(evil) % (1 << 64) == sum(sizes)  # the wrapped total still matches ntotal
    struct.pack_into(f"<{cnt}Q", buf, at + 8, *evil)
    with pytest.raises(_lib.RvcxError) as e:
        _lib.index_parse(bytes(buf))
    assert e.value.code == -1 and "exceeds ntotal" in str(e.value)


def test_index_parse_rejects_huge_counts():
    """A direct-map or size-vector count whose byte size wraps (count * 8 == 0 mod 2^64) is refused before
    anything is allocated from it."""
    import struct

    from rvcx import _lib

    buf = bytearray(_ivf_bytes(direct_map=1))
    # the direct map follows the quantizer: fourcc, header (33 B), centroid count u64, centroids [4][64] f32
    at = buf.index(b"IxF2") + 4 + 33 + 8 + 4 * 64 * 4
    assert buf[at] == 1 and struct.unpack_from("<Q", buf, at + 1)[0] == 300
    struct.pack_into("<Q", buf, at + 1, 1 << 61)
    with pytest.raises(_lib.RvcxError) as e:
        _lib.index_parse(bytes(buf))
    assert e.value.code == -1 and "truncated" in str(e.value)
    buf = bytearray(_ivf_bytes())
    at = buf.index(b"full") + 4
    struct.pack_into("<Q", buf, at, (1 << 61) + 4)
    with pytest.raises(_lib.RvcxError):
        _lib.index_parse(bytes(buf))


_KNOB_PROBE = r"""
import ctypes, json, sys
lib = ctypes.CDLL(sys.argv[1])
lib.rvcx_config_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
buf = ctypes.create_string_buffer(4096)
n = ctypes.c_int64(0)
assert lib.rvcx_config_info(None, ctypes.cast(buf, ctypes.c_void_p), 4096, ctypes.byref(n)) == 0
print(buf.value.decode())
"""


@pytest.mark.parametrize("experimental", [False, True])
def test_env_knobs_need_the_experimental_opt_in(experimental):
    """RVCX_* tuning / arithmetic switches are honoured only with RVCX_EXPERIMENTAL=1; without it
    RVCX_CONV_MATH=f32 is ignored (the default arithmetic stays) and rvcx_config_info lists it as not honoured."""
    import json
    import os
    import subprocess
    import sys

    from rvcx import _lib

    env = {k: v for k, v in os.environ.items() if not k.startswith("RVCX_")}
    env["RVCX_CONV_MATH"] = "f32"
    env["RVCX_NO_OVERLAP"] = "1"
    if experimental:
        env["RVCX_EXPERIMENTAL"] = "1"
    out = subprocess.run([sys.executable, "-c", _KNOB_PROBE, _lib.LIB_PATH], env=env, capture_output=True, text=True,
                         timeout=120, check=True).stdout
    info = json.loads(out.strip().splitlines()[-1])
    assert info["experimental"] is experimental
    assert info["conv_math_default"] == ("f32" if experimental else "h16")
    assert info["env"]["RVCX_CONV_MATH"] == {"value": "f32", "honoured": experimental}
    assert info["env"]["RVCX_NO_OVERLAP"]["honoured"] is experimental
