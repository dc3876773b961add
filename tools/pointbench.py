"""Token-linear (1x1 / MODE_POINT) GEMMs at SwinUNETR c4's shapes (128^3, feature_size 48): forward, data gradient and
weight gradient of engine.swin.Lin, timed with HIP events; prints achieved GB/s against the compulsory bytes
(A + out + weights).  --lib PATH times another build of the library (A/B runs in one GPU call).
    python tools/pointbench.py [--lib /path/libmmseg_hip.so] [--reps 20]"""
import argparse
import sys

import torch

sys.path.insert(0, "/root/repo")
import mmseg_amd  # noqa: F401,E402
from mmseg_amd import _lib  # noqa: E402

# (M tokens, K = Ci, N = Co): stage-0 / stage-1 swin linears, the merge reductions, the decoder's 1x1 residual convs
SHAPES = [(262144, 48, 144), (262144, 48, 48), (262144, 48, 192), (262144, 192, 48), (32768, 384, 96),
          (32768, 96, 288), (32768, 96, 96), (32768, 96, 384), (32768, 384, 96), (2097152, 96, 48),
          (262144, 192, 96), (2097152, 48, 128), (262144, 48, 128)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    if args.lib:
        _lib._LIB = _lib._Lib(args.lib)
    from mmseg_amd.engine.runtime import FlatParams, Runtime
    from mmseg_amd.engine.swin import Lin
    dev = torch.device("cuda", 0)
    rt = Runtime(dev, torch.bfloat16)
    L = _lib.lib()
    print("library", L.path, flush=True)
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for M, K, N in SHAPES:
        torch.manual_seed(M + K + N)
        lin = torch.nn.Linear(K, N).to(dev)
        flat = FlatParams(list(lin.parameters()))
        ln = Lin(rt, lin.weight, lin.bias, flat)
        for d in ln.descs():
            L.mmseg_pack_weight(*d, rt.code, rt.stream)
        x = torch.randn(M * K, device=dev).to(torch.bfloat16)
        y = torch.empty(M * N, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(M * N, device=dev).to(torch.bfloat16)
        dx = torch.empty(M * K, device=dev, dtype=torch.bfloat16)
        res = {}

        def fwd():
            ln.fwd(x, K, M, y, N)

        def dgrad():
            ln.bwd(x, K, dy, N, M, dx, K, False)

        def wgrad():
            ln.bwd(x, K, dy, N, M, None, K, False)

        for nm, fn in (("fwd", fwd), ("bwd", dgrad), ("wgrad", wgrad)):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[nm] = e0.elapsed_time(e1) / args.reps * 1000
        gb = (M * K + M * N) * 2 / 1e9
        tot["fwd"] += res["fwd"]
        tot["dgrad"] += res["bwd"]
        tot["wgrad"] += res["wgrad"]
        print(f"M={M:8d} K={K:4d} N={N:4d}: fwd {res['fwd']:7.1f} us ({gb / res['fwd'] * 1e6:6.0f} GB/s)  "
              f"bwd (wgrad + dgrad) {res['bwd']:7.1f} us ({2 * gb / res['bwd'] * 1e6:6.0f} GB/s)  "
              f"wgrad {res['wgrad']:7.1f} us ({gb / res['wgrad'] * 1e6:6.0f} GB/s)  "
              f"y {y.float().abs().sum().item():.5e} dx {dx.float().abs().sum().item():.5e} "
              f"dw {flat.grad(lin.weight).abs().sum().item():.5e}", flush=True)
    print("total fwd %.1f us, bwd %.1f us, wgrad alone %.1f us" % (tot["fwd"], tot["dgrad"], tot["wgrad"]))


if __name__ == "__main__":
    main()
