"""Stem (first 3^3 conv, Cr real input channels -> Co) microbenchmark at the bench shape: forward and weight
gradient through the C ABI on a compact (ld = Cr) bf16 input.  Run it under rocprofv3 for kernel durations.

    python tools/stembench.py [--iters 20] [--cr 1] [--co 32] [--size 96] [--n 2]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cr", type=int, default=1)
    ap.add_argument("--co", type=int, default=32)
    ap.add_argument("--size", type=int, default=96)
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--only", default="fwd,wgrad")
    ap.add_argument("--want", type=int, default=2048, help="weight-gradient splits asked for")
    args = ap.parse_args()
    import mmseg_amd  # noqa: F401
    from mmseg_amd._lib import lib, ptr
    L = lib()
    dev = torch.device("cuda", 0)
    N, S, cr, Co = args.n, args.size, args.cr, args.co
    V = S ** 3
    code = 1   # MMSEG_BF16
    s = torch.cuda.current_stream().cuda_stream
    x = torch.randn(N * V * cr, device=dev).to(torch.bfloat16)
    w = torch.randn(Co, cr, 27, device=dev) * 0.2
    b = torch.randn(Co, device=dev)
    y = torch.empty(N * V * Co, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(N * V * Co, device=dev).to(torch.bfloat16)
    ks = L.mmseg_stem_wgrad_splits(N, S, S, S, args.want)
    kp = L.mmseg_stem_kp(cr)
    part = torch.empty(ks * Co * kp + ks * Co, device=dev)
    gw = torch.empty(Co * cr * 27, device=dev)
    gb = torch.empty(Co, device=dev)
    for _ in range(args.iters):
        if "fwd" in args.only:
            L.mmseg_stem_fwd(ptr(x), cr, cr, ptr(w), ptr(b), ptr(y), Co, N, S, S, S, Co, code, s)
        if "wgrad" in args.only:
            L.mmseg_stem_wgrad(ptr(dy), Co, ptr(x), cr, cr, ptr(part), part.data_ptr() + ks * Co * kp * 4, N, S, S, S,
                               Co, ks, code, s)
            L.mmseg_wgrad_reduce(ptr(part), ptr(gw), part.data_ptr() + ks * Co * kp * 4, ptr(gb), Co, kp, ks, cr, cr,
                                 27, 0, s)
    torch.cuda.synchronize()
    print("ok", ks, kp)


if __name__ == "__main__":
    main()
