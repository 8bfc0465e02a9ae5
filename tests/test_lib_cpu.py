"""CPU-side checks of the C-ABI library: it is built, loads, and exports every symbol the
header declares (no compute calls — there is no GPU here)."""
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(REPO, "include", "optimobo_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(omb_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_entry_points():
    syms = header_symbols()
    for s in ["omb_create", "omb_destroy", "omb_set_gp", "omb_posterior", "omb_kernel_block", "omb_ehvi2d",
              "omb_ehvi3d_mc", "omb_hvpoi", "omb_expdec", "omb_ei", "omb_argmax", "omb_argmax_dev"]:
        assert s in syms


def test_library_loads_and_exports_header_symbols():
    from optimobo_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("liboptimobo_hip.so not built (run __graft_entry__.build())")
    lib = _lib.load()
    for s in header_symbols():
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} declared in the header but not typed in _lib.SIGNATURES"
    assert lib.omb_abi_version() == 1


def test_create_without_gpu_fails_cleanly():
    import ctypes

    import torch
    from optimobo_amd import _lib
    if not os.path.exists(_lib.LIB_PATH) or torch.cuda.is_available():
        pytest.skip("needs the built library and no GPU")
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.omb_create(0, ctypes.byref(h)) != 0


def test_device_context_refuses_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from optimobo_amd.device import AcqContext
    with pytest.raises(RuntimeError):
        AcqContext(0)


def test_host_limits_match_header():
    """The ctypes layer's limits are the header's (#define OMB_MAX_*)."""
    import re

    from optimobo_amd import _lib
    src = open(os.path.join(REPO, "include", "optimobo_hip.h")).read()
    val = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define OMB_(MAX_\w+)\s+(\d+)", src)}
    assert val["MAX_OBJ"] == _lib.MAX_OBJ
    assert val["MAX_DIM"] == _lib.MAX_DIM
    assert val["MAX_TRAIN"] == _lib.MAX_TRAIN
    assert val["MAX_TRAIN_DENSE"] == _lib.MAX_TRAIN_DENSE


def test_debug_knob_codes_match_header():
    """The ctypes layer's omb_debug_set codes are the header's OMB_DEBUG_* enum values."""
    import re

    from optimobo_amd import _lib
    src = open(os.path.join(REPO, "include", "optimobo_hip.h")).read()
    val = {m.group(1): int(m.group(2)) for m in re.finditer(r"OMB_(DEBUG_\w+)\s*=\s*(\d+)", src)}
    assert val and all(getattr(_lib, k) == v for k, v in val.items()), val
    assert {"DEBUG_FUSED_CHAIN", "DEBUG_TIMING_STRIDE", "DEBUG_CHOL_MODE"} <= set(val)
