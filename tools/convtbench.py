"""Transposed-conv (k2 s2) microbenchmark through the engine's ConvT2 layer: forward into a concat-style output
(ld = 2 Co, as the decoder's upconv writes the first half of the skip concat), backward (weight + bias gradient,
data gradient).  Run under rocprofv3 for the kernel durations.

    python tools/convtbench.py [--shape N,S,Cin,Cout ...] [--iters 10]
S is the input (coarse) size; the output grid is 2S.
"""
import argparse
import os
import sys

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", nargs="*", default=["2,48,64,32", "2,24,128,64", "2,12,256,128", "2,6,320,256"])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="fwd,bwd")
    args = ap.parse_args()
    import mmseg_amd  # noqa: F401
    from mmseg_amd.engine.layers import ConvT2
    from mmseg_amd.engine.runtime import FlatParams, Runtime
    dev = torch.device("cuda", 0)
    rt = Runtime(dev, torch.bfloat16)
    for sh in args.shape:
        N, S, Ci, Co = (int(v) for v in sh.split(","))
        torch.manual_seed(0)
        up = nn.ConvTranspose3d(Ci, Co, 2, 2).to(dev)
        flat = FlatParams(list(up.parameters()))
        layer = ConvT2(rt, up, flat)
        layer.pack()
        x = rt.act(N, S, S, S, Ci)
        x.buf.normal_()
        cat = rt.act(N, 2 * S, 2 * S, 2 * S, 2 * Co)
        cat.buf.normal_()
        y = cat.slot(0, Co)
        dx = rt.act(N, S, S, S, Ci)
        for _ in range(args.iters):
            if "fwd" in args.only:
                layer.fwd(x, y)
            if "bwd" in args.only:
                layer.bwd(x, y, dx, False)
        torch.cuda.synchronize()
        print("ok", sh, flush=True)


if __name__ == "__main__":
    main()
