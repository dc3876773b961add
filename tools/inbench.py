"""InstanceNorm + ReLU backward microbenchmark (mmseg_instnorm_relu_bwd) at the 96^3 encoder shapes: the plain
case (dy = p1) and the DualEncoder encoder-output case (dy = scale * p1 + MaxPool backward gather), with p1 in a
strided (ld = 2C, the decoder's skip-gradient slot) or dense buffer.  Run under rocprofv3 for the durations.

    python tools/inbench.py [--size 96] [--c 32] [--iters 10]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=96)
    ap.add_argument("--c", type=int, default=32)
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cases", default="copy,fwd,stats,apply,plain,pool_ld2,pool_ld1,plain_ld2")
    args = ap.parse_args()
    import mmseg_amd  # noqa: F401
    from mmseg_amd._lib import lib, ptr
    L = lib()
    dev = torch.device("cuda", 0)
    N, S, C = args.n, args.size, args.c
    V = S ** 3
    bf = torch.bfloat16
    s = torch.cuda.current_stream().cuda_stream
    x = torch.randn(N * V * C, device=dev).to(bf)
    dx = torch.empty_like(x)
    p1_dense = torch.randn(N * V * C, device=dev).to(bf)
    p1_wide = torch.randn(N * V * 2 * C, device=dev).to(bf)
    pool = torch.randn(N * V // 8 * C, device=dev).to(bf)
    idx = torch.randint(0, 8, (N * V // 8 * C,), device=dev, dtype=torch.uint8)
    mean = torch.randn(N * C, device=dev) * 0.1
    rstd = torch.rand(N * C, device=dev) + 0.5
    ws = torch.empty(L.mmseg_instnorm_ws_floats(N, V, C), device=dev)
    for case in args.cases.split(","):
        if case == "copy":   # torch's bf16 copy of the same tensor: the box's streaming reference
            for _ in range(args.iters):
                dx.copy_(x)
            torch.cuda.synchronize()
            print("case", case, flush=True)
            continue
        if case in ("stats", "apply", "fwd"):
            for _ in range(args.iters):
                if case == "fwd":
                    L.mmseg_instnorm_fwd(ptr(x), C, ptr(dx), C, N, V, C, 1e-5, ptr(mean), C, ptr(rstd), 1, ptr(ws), 1, s)
                elif case == "stats":
                    L.mmseg_instnorm_stats(ptr(x), C, N, V, C, 1e-5, ptr(mean), C, ptr(rstd), ptr(ws), 1, s)
                else:
                    L.mmseg_instnorm_relu_fwd(ptr(x), C, ptr(dx), C, N, V, C, ptr(mean), ptr(rstd), 1, s)
            torch.cuda.synchronize()
            print("case", case, flush=True)
            continue
        ld1 = 2 * C if "ld2" in case else C
        p1 = p1_wide if ld1 == 2 * C else p1_dense
        has_pool = case.startswith("pool")
        for _ in range(args.iters):
            L.mmseg_instnorm_relu_bwd(ptr(x), C, ptr(mean), ptr(rstd), ptr(p1), ld1, 0.5, None, 0, None, 0,
                                      ptr(pool) if has_pool else None, C if has_pool else 0,
                                      ptr(idx) if has_pool else None, ptr(dx), C, N, S, S, S, C, ptr(ws), 1, s)
        torch.cuda.synchronize()
        print("case", case, flush=True)


if __name__ == "__main__":
    main()
