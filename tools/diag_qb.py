import sys, torch, numpy as np
sys.path.insert(0, '/root/repo')
import mmseg_amd
from mmseg_amd._lib import lib, ptr, stream_handle
dev = torch.device("cuda", 0)
import os, itertools
for (f1, b2), masked in itertools.product(((1, 1), (0, 1), (1, 0), (0, 0)), (True,)):
    os.environ['MMSEG_WINATTN_FWD1'] = str(f1); os.environ['MMSEG_WINATTN_BWD2'] = str(b2); print('FWD1', f1, 'BWD2', b2)
    N, hd, heads, nwin = 343, 16, 2, 4
    C, B = heads * hd, 360
    L, s = lib(), stream_handle()
    ng = L.mmseg_winattn_sum_groups(B, N, heads)
    g = torch.Generator().manual_seed(5)
    qkv = torch.randn(B * N, 3 * C, generator=g).to(torch.bfloat16).to(dev)
    table = (torch.randn(13 ** 3, heads, generator=g) * 0.5).to(dev)
    region = torch.randint(0, 4, (nwin, N), generator=g).to(torch.uint8).to(dev) if masked else None
    dO = torch.randn(B * N, C, generator=g).to(torch.bfloat16).to(dev)
    tabt = table.t().contiguous(); scale = hd ** -0.5; nwm = nwin if masked else 0
    O = torch.full((B * N, C), float('nan'), dtype=torch.bfloat16, device=dev)
    lse = torch.full((L.mmseg_winattn_lse_floats(B, heads),), float('nan'), device=dev)
    L.mmseg_winattn_fwd(ptr(qkv), B, N, C, heads, ptr(tabt), 13 ** 3, 7, 7, 7, ptr(region), nwm, scale, ptr(O), ptr(lse), s)
    ldn = (N + 7) // 8 * 8
    torch.cuda.synchronize(); print('O nan', int(torch.isnan(O.float()).sum()), 'lse nan (valid)', int(torch.isnan(lse.view(B*heads, -1)[:, :N]).sum()))
    d1 = torch.full((B * N, 3 * C), float('nan'), dtype=torch.bfloat16, device=dev)
    dsum = torch.empty(ng * heads * N * ldn, device=dev)
    L.mmseg_winattn_bwd_sum(ptr(qkv), ptr(O), ptr(dO), ptr(lse), B, N, C, heads, ptr(tabt), 13 ** 3, 7, 7, 7, ptr(region), nwm, scale, ptr(d1), ptr(dsum), ldn, s)
    d2 = torch.full((B * N, 3 * C), float('nan'), dtype=torch.bfloat16, device=dev)
    dS = torch.empty(B * heads * N * ldn, dtype=torch.bfloat16, device=dev)
    L.mmseg_winattn_bwd(ptr(qkv), ptr(O), ptr(dO), ptr(lse), B, N, C, heads, ptr(tabt), 13 ** 3, 7, 7, 7, ptr(region), nwm, scale, ptr(d2), ptr(dS), ldn, s)
    torch.cuda.synchronize()
    diff = (d1.float() - d2.float()).abs()
    for nm, sl in (("dq", slice(0, C)), ("dk", slice(C, 2 * C)), ("dv", slice(2 * C, 3 * C))):
        dd = diff[:, sl]
        nz = (dd > 0).nonzero()
        if nm == "dk":
            bad = torch.isnan(d1[:, sl].float()).any(1).nonzero()[:, 0]
            print("nan rows: windows", sorted(set((bad // N).tolist()))[:20], "tokens", sorted(set((bad % N).tolist()))[:40])
            badc = torch.isnan(d1[:, sl].float()).any(0).nonzero()[:, 0]
            print("nan cols", badc.tolist())
        print(masked, nm, "nan1", int(torch.isnan(d1[:, sl].float()).sum()), "nan2", int(torch.isnan(d2[:, sl].float()).sum()), "ndiff", int((dd > 0).sum()), "max", float(dd.max()), "rows", nz[:5, 0].tolist() if len(nz) else [])
