"""Microbenchmark of one 3^3 conv layer on the engine (fwd, dgrad, wgrad), HIP-event timed.

    python tools/convbench.py [--shape N,S,Cin,Cout | N,D,H,W,Cin,Cout ...] [--iters 20] [--only fwd,dgrad,wgrad]
Env knobs (MMSEG_*) select kernel variants; prints one JSON line per (shape, op) with
the kernel the library launched, us per launch and TFLOP/s (2*27*Cin*Cout per voxel).
Ops: fwd, fwds (forward with the fused InstanceNorm partials, as ConvBlock3D runs it), fwdn (forward of
relu(IN(x)) with the norm applied on staging: Block.defer1's conv2), dgrad, dgradin (data gradient that also sums
the InstanceNorm-backward partials of its output: Block.bwd's conv2 at 96^3), wgrad, wgradn (weight gradient with
the deferred norm of x).
--probe: load libmmseg_hip_probe.so (make -C csrc probe) and print the block timeline of one launch per op
(per-CU residency, block lifetimes, per-phase cycles of block 0's waves; see conv_gemm.hip PROBE_*).
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
    ap.add_argument("--probe", action="store_true")
    ap.add_argument("--lib", default=None, help="another in-tree build of the library (A/B), e.g. libmmseg_hip_old.so")
    args = ap.parse_args()
    if args.probe or args.lib:
        from mmseg_amd import _lib
        _lib.set_library_path(os.path.join(ROOT, "multimodal-organ-segmentation_amd",
                                           args.lib or "libmmseg_hip_probe.so"))
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

        nb = layer.stats_bricks(x, y)
        part = torch.empty(N * max(nb, 1) * Co * 2, dtype=torch.float32, device=dev)
        mean = torch.zeros(N * Ci, dtype=torch.float32, device=dev)
        rstd = torch.ones(N * Ci, dtype=torch.float32, device=dev)
        inpart = torch.empty(N * 4096 * Ci * 2, dtype=torch.float32, device=dev)

        def run(op):
            if op == "fwd":
                layer.fwd(x, y)
            elif op == "fwds":
                assert nb > 0, "no fused-statistics kernel for this shape (the library offers none since round 5)"
                layer.fwd(x, y, stats_part=part)
            elif op == "fwdn":
                layer.fwd_norm(x, mean, rstd, y)
            elif op == "dgradin":
                M = N * D * H * W
                nch = L.mmseg_conv3_dgrad_in_chunks(M, Ci, layer.Cpad_d, layer.KGd, layer.dshift, D, H, W, y.ld,
                                                    dx.ld, code)
                assert nch > 0 and N * nch * Ci * 2 <= inpart.numel(), "no INP data-gradient kernel for this shape"
                L.mmseg_conv3_dgrad_in(y.ptr, y.ld, layer.wd.data_ptr(), dx.ptr, dx.ld, M, Ci, layer.Cpad_d,
                                       layer.KGd, layer.dshift, D, H, W, x.ptr, x.ld, mean.data_ptr(),
                                       rstd.data_ptr(), inpart.data_ptr(), code, s)
            elif op == "dgrad":
                M = N * D * H * W
                ks = L.mmseg_conv3_splits(M, Ci, layer.Cpad_d, layer.KGd, layer.dshift, D, H, W, y.ld, dx.ld, code)
                ws = rt.ws(ks * M * Ci) if ks > 1 else None
                L.mmseg_conv_gemm(y.ptr, y.ld, layer.wd.data_ptr(), None, dx.ptr, dx.ld,
                                  ws.data_ptr() if ws is not None else None, 0, M, Ci, layer.Cpad_d, layer.KGd,
                                  layer.dshift, D, H, W, ks, code, s)
            elif op == "wgradn":   # deferred-norm weight gradient (Block.defer1's conv2 backward)
                V = N * D * H * W
                wsf = L.mmseg_conv3_wgrad_ws_floats(V, Co, layer.Cip, Ci, layer.cpg_shift, D, H, W, y.ld, x.ld, code)
                ws = rt.ws(wsf) if wsf > 0 else None
                L.mmseg_conv3_wgrad_norm(y.ptr, y.ld, x.ptr, x.ld, mean.data_ptr(), rstd.data_ptr(),
                                         flat.grad(conv.weight).data_ptr(), flat.grad(conv.bias).data_ptr(), Co,
                                         layer.Cip, Ci, layer.cpg_shift, V, D, H, W,
                                         ws.data_ptr() if ws is not None else None, wsf, 0, code, s)
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
            if args.probe:
                probe(L, lambda: run(op), dev)


def probe(L, fn, dev):
    """One launch with the block timeline probe on; prints residency and phase statistics."""
    import ctypes
    import numpy as np
    nb_max = 16384
    buf = torch.zeros(8 * nb_max + 32 * 16 * 64, dtype=torch.int64, device=dev)
    setp = L.dll.mmseg_probe_set
    setp.argtypes = [ctypes.c_void_p]
    torch.cuda.synchronize()
    assert setp(buf.data_ptr()) == 0
    fn()
    torch.cuda.synchronize()
    assert setp(None) == 0
    h = buf.cpu().numpy()
    blk = h[:8 * nb_max].reshape(nb_max, 8)
    nblk = int((blk[:, 0] != 0).sum())
    if nblk == 0:
        print("  probe: this kernel records no timeline", flush=True)
        return
    blk = blk[:nblk]
    t0 = blk[:, 0].min()
    st, en = (blk[:, 0] - t0) * 0.01, (blk[:, 1] - t0) * 0.01          # us (100 MHz realtime)
    cyc = blk[:, 3] - blk[:, 2]
    hw, xcc = blk[:, 4], blk[:, 5] & 0xF
    cu = xcc * 4096 + ((hw >> 8) & 0xFF)                                   # XCC, SE / SH / CU
    span = en.max()
    ucu = np.unique(cu)
    # per-CU concurrency sampled on a 0.1 us grid
    grid = np.arange(0, span, 0.1)
    conc = np.zeros((len(ucu), len(grid)))
    for k, c in enumerate(ucu):
        for s_, e_ in zip(st[cu == c], en[cu == c]):
            conc[k, (grid >= s_) & (grid < e_)] += 1
    per_cu = np.array([(cu == c).sum() for c in ucu])
    print(f"  probe: {nblk} blocks on {len(ucu)} CUs (blocks/CU min {per_cu.min()} max {per_cu.max()}), span "
          f"{span:.1f} us, last start {st.max():.1f} us; block lifetime mean {np.mean(en - st):.2f} us "
          f"(p10 {np.percentile(en - st, 10):.2f} p90 {np.percentile(en - st, 90):.2f}), {np.mean(cyc):.0f} cycles "
          f"-> clock {np.mean(cyc) / np.mean((en - st) * 1e3):.2f} GHz; mean resident blocks/CU {conc.mean():.2f} "
          f"(max {conc.max():.0f}); CU-time with 0/1/2+ blocks {np.mean(conc == 0):.2f}/{np.mean(conc == 1):.2f}/"
          f"{np.mean(conc >= 2):.2f}", flush=True)
    ph = h[8 * nb_max:].reshape(32, 16, 64)
    for w in (0, 1, 4, 7):
        q = ph[0, w]
        n = int((q != 0).sum())
        if n > 1:
            print(f"  block0 wave{w} phases (cycles): {list(np.diff(q[:n]))}", flush=True)


if __name__ == "__main__":
    main()
