"""Window-attention kernels at SwinUNETR c4's shapes (128^3, feature_size 48: 64^3 / 32^3 / 16^3 / 8^3 tokens,
7^3 windows, head_dim 16): times mmseg_winattn_fwd, mmseg_winattn_bwd_sum (key pass + grouped query pass) and
mmseg_winattn_bwd per stage with HIP events; run under rocprofv3 --kernel-trace --stats for the per-kernel split.
    python tools/wabench.py [--reps 20] [--stages 0,1] [--lib PATH]"""
import argparse
import sys

import torch

sys.path.insert(0, "/root/repo")
import mmseg_amd  # noqa: F401,E402
from mmseg_amd._lib import lib, ptr, stream_handle  # noqa: E402

STAGES = [(1000, 3), (125, 6), (27, 12), (8, 24)]   # (windows, heads) at 128^3, batch 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--stages", default="0,1")
    ap.add_argument("--masked", type=int, default=1)
    ap.add_argument("--lib", default="", help="time another build of the library")
    args = ap.parse_args()
    if args.lib:
        from mmseg_amd import _lib as _l
        _l._LIB = _l._Lib(args.lib)
    dev = torch.device("cuda", 0)
    L, s = lib(), stream_handle()
    N, hd, nwin = 343, 16, 8
    for si in [int(x) for x in args.stages.split(",")]:
        B, heads = STAGES[si]
        C = heads * hd
        g = torch.Generator().manual_seed(5 + si)
        qkv = torch.randn(B * N, 3 * C, generator=g).to(torch.bfloat16).to(dev)
        tabt = (torch.randn(heads, 13 ** 3, generator=g) * 0.5).to(dev)
        region = torch.randint(0, 4, (nwin, N), generator=g).to(torch.uint8).to(dev) if args.masked else None
        nwm = nwin if args.masked else 0
        dO = torch.randn(B * N, C, generator=g).to(torch.bfloat16).to(dev)
        O = torch.empty(B * N, C, dtype=torch.bfloat16, device=dev)
        lse = torch.empty(L.mmseg_winattn_lse_floats(B, heads), device=dev)
        ldn = (N + 7) // 8 * 8
        ng = L.mmseg_winattn_sum_groups(B, N, heads)
        dqkv = torch.empty(B * N, 3 * C, dtype=torch.bfloat16, device=dev)
        dsum = torch.empty(max(ng, 1) * heads * N * ldn, device=dev)
        dS = torch.empty(B * heads * N * ldn, dtype=torch.bfloat16, device=dev) if ng == 0 else None
        sc = hd ** -0.5

        def fwd():
            L.mmseg_winattn_fwd(ptr(qkv), B, N, C, heads, ptr(tabt), 13 ** 3, 7, 7, 7, ptr(region), nwm, sc, ptr(O),
                                ptr(lse), s)

        def bwd():
            if ng > 0:
                L.mmseg_winattn_bwd_sum(ptr(qkv), ptr(O), ptr(dO), ptr(lse), B, N, C, heads, ptr(tabt), 13 ** 3, 7, 7,
                                        7, ptr(region), nwm, sc, ptr(dqkv), ptr(dsum), ldn, s)
            else:
                L.mmseg_winattn_bwd(ptr(qkv), ptr(O), ptr(dO), ptr(lse), B, N, C, heads, ptr(tabt), 13 ** 3, 7, 7, 7,
                                    ptr(region), nwm, sc, ptr(dqkv), ptr(dS), ldn, s)

        for fn, nm in ((fwd, "fwd"), (bwd, "bwd")):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            print(f"stage {si} B={B} heads={heads} groups={ng} {nm}: {e0.elapsed_time(e1) / args.reps * 1000:.1f} us",
                  flush=True)
        print(f"  checksum dq {dqkv[:, :C].float().abs().sum().item():.6e} dk {dqkv[:, C:2 * C].float().abs().sum().item():.6e}"
              f" dv {dqkv[:, 2 * C:].float().abs().sum().item():.6e} dsum {dsum.abs().sum().item():.6e}", flush=True)


if __name__ == "__main__":
    main()
