"""Head + loss microbenchmark at the bench's shape (96^3, B=2, 32 -> 6, DiceCE, bf16): the unfused sequence
(head_fwd, loss stats + finalize, loss_bwd, head_bwd) against the fused head + loss kernels, HIP-event timed.

    python tools/headbench.py [--iters 20] [--step-only]

The step form (deferred InstanceNorm input, InstanceNorm-backward partials) is timed too; its loss / checksums
let two builds of the library be compared (the round-4 chunking / prefetch variants are fixed constants now).
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--size", type=int, default=96)
    ap.add_argument("--step-only", action="store_true", help="only the training step's form (deferred norm + IN partials)")
    args = ap.parse_args()
    import mmseg_amd  # noqa: F401
    from mmseg_amd._lib import lib, ptr
    dev = torch.device("cuda", 0)
    L = lib()
    N, C, Cin, S = 2, 6, 32, args.size
    V = S ** 3
    s = torch.cuda.current_stream().cuda_stream
    x = torch.randn(N * V * Cin, device=dev).to(torch.bfloat16)
    dx = torch.empty_like(x)
    W = torch.randn(C * Cin, device=dev) * 0.1
    b = torch.randn(C, device=dev) * 0.1
    y = torch.randint(0, C, (N * V,), device=dev)
    gW = torch.zeros(C * Cin, device=dev)
    gb = torch.zeros(C, device=dev)
    logits = torch.empty(N * C * V, device=dev)
    dlog = torch.empty_like(logits)
    ws = torch.empty(L.mmseg_loss_ws_floats(N, C, V), device=dev)
    hws = torch.empty(L.mmseg_head_ws_floats(C, Cin, N, V), device=dev)
    wpart = torch.empty(L.mmseg_head_loss_wpart_floats(C, Cin, N, V), device=dev)
    loss = torch.empty((), device=dev)
    g = torch.ones((), device=dev)
    args8 = (0, 0.5, 0.5, 1.0, 0.0, 0.0, 1, None)

    def unfused_fwd():
        L.mmseg_head_fwd(ptr(x), Cin, Cin, ptr(W), ptr(b), None, C, N, V, ptr(logits), 1, s)
        L.mmseg_loss_fwd(ptr(logits), ptr(y), 8, N, C, V, *args8, ptr(loss), ptr(ws), s)

    def unfused_bwd():
        L.mmseg_loss_bwd(ptr(logits), ptr(y), 8, N, C, V, *args8, ptr(g), 1.0, ptr(dlog), ptr(ws), s)
        L.mmseg_head_bwd(ptr(x), Cin, Cin, ptr(W), None, C, N, V, ptr(dlog), ptr(dx), Cin, ptr(gW), ptr(gb),
                         ptr(hws), 0, 1, s)

    def fused_fwd():
        L.mmseg_head_loss_fwd(ptr(x), Cin, Cin, None, None, ptr(W), ptr(b), None, C, N, V, ptr(y), 8, *args8, ptr(loss), ptr(ws),
                              1, s)

    def fused_bwd():
        L.mmseg_head_loss_bwd(ptr(x), Cin, Cin, None, None, ptr(W), ptr(b), None, C, N, V, ptr(y), 8, *args8, ptr(g), 1.0,
                              ptr(ws), ptr(dx), Cin, ptr(gW), ptr(gb), ptr(wpart), 0, 1, s)

    # the training step's form: deferred InstanceNorm + ReLU of the input on load, InstanceNorm-backward partials
    nmean = (torch.randn(N * Cin, device=dev) * 0.1).contiguous()
    nrstd = (torch.rand(N * Cin, device=dev) + 0.5).contiguous()
    inpart = torch.empty(N * max(L.mmseg_head_loss_in_chunks(C, Cin, V), 1) * Cin * 2, device=dev)

    def step_fwd():
        L.mmseg_head_loss_fwd(ptr(x), Cin, Cin, ptr(nmean), ptr(nrstd), ptr(W), ptr(b), None, C, N, V, ptr(y), 8,
                              *args8, ptr(loss), ptr(ws), 1, s)

    def step_bwd():
        L.mmseg_head_loss_bwd_in(ptr(x), Cin, Cin, ptr(nmean), ptr(nrstd), ptr(W), ptr(b), None, C, N, V, ptr(y), 8,
                                 *args8, ptr(g), 1.0, ptr(ws), ptr(dx), Cin, ptr(gW), ptr(gb), ptr(wpart), ptr(inpart),
                                 0, 1, s)

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / args.iters

    unfused_fwd()
    unfused_bwd()
    ref = (loss.item(), dx.float().clone(), gW.clone())
    fused_fwd()
    fused_bwd()
    torch.cuda.synchronize()
    err = {"loss": abs(loss.item() - ref[0]), "dx": ((dx.float() - ref[1]).abs().max() / ref[1].abs().max()).item(),
           "gW": ((gW - ref[2]).abs().max() / ref[2].abs().max()).item()}
    res = {"env": {k: v for k, v in os.environ.items() if k.startswith("MMSEG_")}}
    if not args.step_only:
        res.update({"unfused_fwd_us": timeit(unfused_fwd), "unfused_bwd_us": timeit(unfused_bwd),
                    "fused_fwd_us": timeit(fused_fwd), "fused_bwd_us": timeit(fused_bwd), "err": err})
    step_fwd()
    step_bwd()
    torch.cuda.synchronize()
    res.update({"step_fwd_us": timeit(step_fwd), "step_bwd_us": timeit(step_bwd), "step_loss": loss.item(),
                "step_dx_sum": dx.float().sum().item(), "step_gW_sum": gW.sum().item(),
                "step_in_sum": inpart.sum().item()})
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
