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


def test_head_loss_size_queries_agree():
    """The fused head + loss backward has its own voxel chunking (whole rounds of its 2-blocks-per-CU grid); the
    weight-gradient partials it writes and the InstanceNorm partials it hands to mmseg_instnorm_bwd_part must be
    counted over the same chunks, and the loss workspace over the statistics pass's."""
    L = _lib.lib()
    for N, V in ((2, 96 ** 3), (1, 64 ** 3), (2, 32 ** 3), (1, 7)):
        for C in (3, 6, 7):
            nch = L.mmseg_head_loss_in_chunks(C, 32, V)
            assert nch >= 1
            assert L.mmseg_head_loss_wpart_floats(C, 32, N, V) == N * nch * (C * 32 + C)
            assert L.mmseg_loss_ws_floats(N, C, V) >= N * (3 * C + 3) + 2 * N * C + 2
    assert L.mmseg_head_loss_in_chunks(6, 32, 96 ** 3) == 256   # 3,456 voxels per block at 96^3
    assert L.mmseg_head_loss_in_chunks(6, 16, 96 ** 3) == 0     # partials only for Cin = 32
