"""Diagnostic (GPU): elementwise passes over 128^3 x 48-channel tensors stored with row pitch 64 (SwinUNETR's
padded layout) vs 64 real channels, and vs dense 48-channel rows -- does a partial-row pass lose bandwidth?
usage: python tools/diag_rows.py"""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
import mmseg_amd  # noqa: E402,F401
from mmseg_amd._lib import lib, ptr, stream_handle  # noqa: E402

dev = "cuda"
L = lib()
V = 128 ** 3


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for C, ld, CW in [(48, 64, 48), (48, 64, 64), (64, 64, 64), (48, 48, 48), (96, 128, 96), (96, 128, 128),
                  (128, 128, 128)]:
    a, b, y = [torch.randn(V * ld, device=dev).to(torch.bfloat16) for _ in range(3)]
    m, r = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    s = stream_handle()
    t_res = timeit(lambda: L.mmseg_res_apply(ptr(a), ld, ptr(m), ptr(r), ptr(b), ld, ptr(m), ptr(r), ptr(y), ld, 1, V,
                                             C, CW, 0.01, 1, s))
    t_lb = timeit(lambda: L.mmseg_lrelu_bwd(ptr(a), ld, ptr(b), ld, ptr(y), ld, V, C, CW, 0.01, 1, s))
    ws = torch.empty(L.mmseg_instnorm_ws_floats(1, V, C), device=dev)
    t_in = timeit(lambda: L.mmseg_instnorm_act_bwd(ptr(a), ld, ptr(m), ptr(r), ptr(b), ld, ptr(y), ld, 1, 128, 128,
                                                   128, C, CW, 0, 0.0, None, 0, ptr(ws), 1, s))
    t_cp = timeit(lambda: y.copy_(a))
    real = V * C * 2 / 1e9
    print(f"C {C} ld {ld} Cw {CW}: res_apply {t_res:7.1f} us ({3 * real / t_res * 1e6:5.2f} GB/ms real), lrelu_bwd {t_lb:7.1f} us "
          f"({3 * real / t_lb * 1e6:5.2f}), instnorm_bwd {t_in:7.1f} us ({5 * real / t_in * 1e6:5.2f}), "
          f"copy whole {t_cp:6.1f} us ({2 * V * ld * 2 / 1e9 / t_cp * 1e6:5.2f})", flush=True)
