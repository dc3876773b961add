"""Microbenchmark of one 3^3 conv layer on the engine (fwd, dgrad, wgrad), HIP-event timed.

    python tools/convbench.py [--shape N,S,Cin,Cout | N,D,H,W,Cin,Cout ...] [--iters 20] [--only fwd,dgrad,wgrad]
Env knobs (MMSEG_*) select kernel variants; prints one JSON line per (shape, op) with
the kernel the library launched, us per launch and TFLOP/s (2*27*Cin*Cout per voxel).
"""
import argparse
import json
import os
import sys

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", nargs="*", default=["2,96,32,32", "2,96,64,32", "2,96,32,64", "2,48,32,64",
                                                    "2,48,64,64", "2,24,128,128", "2,12,256,256", "2,6,512,512"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="fwd,dgrad,wgrad")
    ap.add_argument("--dtype", default="bf16")
    args = ap.parse_args()
    import mmseg_amd  # noqa: F401
    from mmseg_amd.engine.layers import Conv3
    from mmseg_amd.engine.runtime import FlatParams, Runtime

    dev = torch.device("cuda", 0)
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    rt = Runtime(dev, dt)
    ops = args.only.split(",")
    for sh in args.shape:
        vals = [int(v) for v in sh.split(",")]
        if len(vals) == 4:
            N, S, Ci, Co = vals
            D = H = W = S
        else:
            N, D, H, W, Ci, Co = vals
        torch.manual_seed(0)
        conv = nn.Conv3d(Ci, Co, 3, padding=1).to(dev)
        flat = FlatParams(list(conv.parameters()))
        layer = Conv3(rt, conv, flat)
        layer.pack()
        x = rt.act(N, D, H, W, Ci)
        y = rt.act(N, D, H, W, Co)
        dx = rt.act(N, D, H, W, Ci)
        x.buf.normal_()
        y.buf.normal_()
        flops = 2.0 * N * D * H * W * 27 * Ci * Co
        L, s, code = rt.lib, rt.stream, rt.code

        def run(op):
            if op == "fwd":
                layer.fwd(x, y)
            elif op == "dgrad":
                M = N * D * H * W
                ks = L.mmseg_conv3_splits(M, Ci, layer.Cpad_d, layer.KGd, layer.dshift, D, H, W, y.ld, dx.ld, code)
                ws = rt.ws(ks * M * Ci) if ks > 1 else None
                L.mmseg_conv_gemm(y.ptr, y.ld, layer.wd.data_ptr(), None, dx.ptr, dx.ld,
                                  ws.data_ptr() if ws is not None else None, 0, M, Ci, layer.Cpad_d, layer.KGd,
                                  layer.dshift, D, H, W, ks, code, s)
            else:
                V = N * D * H * W
                wsf = L.mmseg_conv3_wgrad_ws_floats(V, Co, layer.Cip, Ci, layer.cpg_shift, D, H, W, y.ld, x.ld, code)
                ws = rt.ws(wsf) if wsf > 0 else None
                L.mmseg_conv3_wgrad(y.ptr, y.ld, x.ptr, x.ld, flat.grad(conv.weight).data_ptr(),
                                    flat.grad(conv.bias).data_ptr(), Co, layer.Cip, Ci, layer.cpg_shift, V, D, H, W,
                                    ws.data_ptr() if ws is not None else None, wsf, 0, code, s)

        for op in ops:
            for _ in range(3):
                run(op)
            kname = L.mmseg_last_kernel().decode()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                run(op)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            print(json.dumps({"shape": sh, "op": op, "kernel": kname, "us": round(us, 1),
                              "tflops": round(flops / (us * 1e-6) / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
