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
