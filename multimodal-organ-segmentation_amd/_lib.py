"""ctypes binding of libmmseg_hip.so (the C ABI declared in include/mmseg_hip.h).

The prototypes are read from the committed header so the Python binding and
the ABI cannot drift apart.  There is deliberately NO fallback: if the shared
library is missing or a call fails, this raises — the product path never
silently drops to a CPU / eager implementation.
"""
from __future__ import annotations

import ctypes
import os
import re
from typing import Dict, Optional

import torch  # noqa: F401  (must be imported first: loads torch's libamdhip64 so we share one HIP runtime)

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
_REPO_DIR = os.path.dirname(_PKG_DIR)
LIB_PATH = os.path.join(_PKG_DIR, "libmmseg_hip.so")
HEADER_PATH = os.path.join(_REPO_DIR, "include", "mmseg_hip.h")

_CTYPE = {
    "int": ctypes.c_int,
    "long long": ctypes.c_longlong,
    "float": ctypes.c_float,
    "double": ctypes.c_double,
    "size_t": ctypes.c_size_t,
    "void": None,
    "const char*": ctypes.c_char_p,
}


def _arg_ctype(decl: str):
    decl = decl.strip()
    if "*" in decl:
        return ctypes.c_void_p
    typ = re.sub(r"\s+\w+$", "", decl).replace("const ", "").strip()
    if typ not in _CTYPE:
        raise RuntimeError(f"mmseg_hip.h: unsupported argument type in '{decl}'")
    return _CTYPE[typ]


def parse_header(path: str = HEADER_PATH) -> Dict[str, tuple]:
    """{name: (restype, [argtypes])} for every mmseg_* prototype in the header."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    protos = {}
    for m in re.finditer(r"(const char\*|int|long long|void)\s+(mmseg_\w+)\s*\(([^;]*?)\)\s*;", src, flags=re.S):
        ret, name, args = m.group(1), m.group(2), " ".join(m.group(3).split())
        argtypes = [] if args in ("", "void") else [_arg_ctype(a) for a in args.split(",")]
        protos[name] = (_CTYPE[ret], argtypes)
    return protos


class MmsegError(RuntimeError):
    pass


# int-returning entry points that return a value, not a status
_VALUE_FUNCS = ("mmseg_abi_version", "mmseg_wgrad_splits", "mmseg_wgrad_splits_conv3", "mmseg_conv3_splits", "mmseg_pack_desc_bytes", "mmseg_pack3_desc_bytes",
                "mmseg_adamw_pack_desc_bytes",
                "mmseg_stem_ok", "mmseg_stem_kp", "mmseg_stem_wgrad_splits", "mmseg_conv3_stats_bricks",
                "mmseg_head_loss_ok", "mmseg_conv3_norm_ok", "mmseg_conv3_wgrad_norm_ok", "mmseg_head_loss_in_chunks",
                "mmseg_conv3_dgrad_in_chunks", "mmseg_stem_stats_bricks", "mmseg_conv3_fp8_ok",
                "mmseg_conv3_group_ok", "mmseg_conv3_wgrad_group_ok", "mmseg_conv3_group_splits", "mmseg_winattn_sum_groups",
                "mmseg_conv3_group_stats_bricks", "mmseg_instnorm_part_chunks",
                "mmseg_wgrad_reduce_flush", "mmseg_wgrad_reduce_pending", "mmseg_wgrad_reduce_discard")


class _Lib:
    def __init__(self, path: Optional[str] = None):
        path = path or LIB_PATH
        if not os.path.exists(path):
            raise ImportError(
                f"{path} not found: the HIP kernels are not built. Run `python -c \"import __graft_entry__ as g; g.build()\"` "
                "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        self.path = path
        self.dll = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        self.protos = parse_header()
        for name, (res, args) in self.protos.items():
            fn = getattr(self.dll, name)  # AttributeError here = header/library mismatch
            fn.restype = res
            fn.argtypes = args
        self.dll.mmseg_last_error.restype = ctypes.c_char_p

    def __getattr__(self, name: str):
        if not name.startswith("mmseg_"):
            raise AttributeError(name)
        fn = getattr(self.dll, name)

        def call(*args):
            # numpy scalars (e.g. channel counts read from configs / fixtures) are not ctypes-convertible
            args = tuple(a.item() if hasattr(a, "item") and not hasattr(a, "data_ptr") and not isinstance(a, (int, float))
                         else a for a in args)
            rc = fn(*args)
            if self.protos[name][0] is ctypes.c_int and name not in _VALUE_FUNCS and rc != 0:
                raise MmsegError(f"{name} failed: {self.dll.mmseg_last_error().decode(errors='replace')}")
            return rc

        call.__name__ = name
        setattr(self, name, call)
        return call


_LIB: Optional[_Lib] = None


def lib() -> _Lib:
    global _LIB
    if _LIB is None:
        _LIB = _Lib()
    return _LIB


def set_library_path(path: str) -> None:
    """Bind another build of the same ABI (A/B of two in-tree builds from tools/); must precede the first
    lib() call.  The package itself always loads the in-tree libmmseg_hip.so: no environment variable can
    swap the library under a training run."""
    global LIB_PATH
    if _LIB is not None:
        raise RuntimeError("set_library_path: the library is already loaded")
    LIB_PATH = path


def ptr(t) -> Optional[int]:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return t.data_ptr()


def stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


DTYPE_CODE = {torch.float32: 0, torch.bfloat16: 1}
