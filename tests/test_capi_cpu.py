"""CPU-side checks of the C-ABI library: it builds for gfx950, loads, and exports every symbol
include/qce.h declares (no compute call without a GPU)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _declared_symbols():
    txt = open(os.path.join(ROOT, "include", "qce.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(qce_[a-z_0-9]+)\s*\(", txt, flags=re.M)))


def test_header_declares_entry_points():
    syms = _declared_symbols()
    for s in ("qce_model_create", "qce_prepare", "qce_estimate", "qce_log_prob", "qce_estimate_partial",
              "qce_get_tables", "qce_last_error", "qce_model_destroy"):
        assert s in syms


def test_library_exports_all_declared_symbols():
    from quantized_channel_estimation_amd import build, _lib
    build.build()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for s in _declared_symbols():
        assert hasattr(lib, s), s
    assert set(_declared_symbols()) == set(_lib.SIGNATURES), "ctypes table and header disagree"
    lib2 = _lib.load()
    assert lib2.qce_version() >= 100


def test_library_is_gfx950_code_object():
    from quantized_channel_estimation_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_no_device_is_a_loud_error():
    from quantized_channel_estimation_amd import _lib
    import numpy as np
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(RuntimeError):
        _lib.DeviceModel(np.zeros((2, 4), complex), np.stack([np.eye(4, dtype=complex)] * 2), np.array([0.5, 0.5]))


def test_library_build_id_is_this_tree():
    """qce_build_id() of the library the package loads is the digest of the csrc/ it sits next to
    (smoke() asserts the same on the GPU box), so a stale prebuilt .so cannot pass for HEAD's."""
    from quantized_channel_estimation_amd import build, _lib
    build.build()
    assert _lib.build_id() == build.source_digest()
    _lib.check_build_current()
