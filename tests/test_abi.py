"""The C ABI: the shared library builds for gfx950, loads next to torch's HIP
runtime, and exports every symbol include/mmseg_hip.h declares (no compute
calls: this runs without a GPU)."""
import ctypes
import os
import subprocess

import pytest

import mmseg_amd  # noqa: F401
from mmseg_amd import _lib


def test_header_parses_and_symbols_exported():
    protos = _lib.parse_header()
    assert len(protos) >= 25
    so = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in protos if not hasattr(so, n)]
    assert not missing, missing


def test_nm_exports_match_header():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = {l.split()[-1] for l in out.stdout.splitlines() if " T " in l and "mmseg_" in l}
    assert set(_lib.parse_header()) <= exported


def test_library_has_gfx950_code_object():
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_abi_version_and_errors():
    L = _lib.lib()
    assert L.mmseg_abi_version() == 1
    # argument validation happens before any launch: a bad call must raise, not crash
    with pytest.raises(_lib.MmsegError):
        L.mmseg_instnorm_stats(None, 8, 1, 8, 12, 1e-5, None, 12, None, None, 0, None)


def test_no_cpu_fallback():
    import torch
    from mmseg_amd.engine.runtime import Runtime
    with pytest.raises(RuntimeError):
        Runtime(torch.device("cpu"), torch.float32)


def test_value_returning_entry_points_do_not_raise():
    L = _lib.lib()
    assert L.mmseg_wgrad_splits(1 << 20, 64) >= 1
    assert L.mmseg_wgrad_splits_conv3(2 * 96 ** 3, 512, 32, 2, 96, 96, 96, 32, 32, 1) >= 1
    assert L.mmseg_conv3_splits(2 * 12 ** 3, 256, 256, 27 * 32, 5, 12, 12, 12, 256, 256, 1) >= 1
    assert L.mmseg_pack_desc_bytes() == 56
