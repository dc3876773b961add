"""Diagnostic: brick2 BN64 forward with MMSEG_BRICK2_B32=1 vs 0 on one shape; prints where outputs differ."""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mmseg_amd  # noqa: F401,E402
from mmseg_amd.engine.layers import Conv3  # noqa: E402
from mmseg_amd.engine.runtime import FlatParams, Runtime  # noqa: E402

dev = torch.device("cuda", 0)
rt = Runtime(dev, torch.bfloat16)
N, S, Ci, Co = 2, 48, 64, 64
torch.manual_seed(0)
conv = nn.Conv3d(Ci, Co, 3, padding=1).to(dev)
flat = FlatParams(list(conv.parameters()))
layer = Conv3(rt, conv, flat)
layer.pack()
x = rt.act(N, S, S, S, Ci)
x.buf.normal_()
outs = []
for v in ("0", "1"):
    os.environ["MMSEG_BRICK2_B32"] = v
    y = rt.act(N, S, S, S, Co)
    y.buf.zero_()
    layer.fwd(x, y)
    torch.cuda.synchronize()
    print(v, rt.lib.mmseg_last_kernel().decode())
    outs.append(y.buf.float().reshape(N, S, S, S, -1)[..., :Co].clone())
d = (outs[0] - outs[1]).abs()
print("max diff", d.max().item(), "frac differing", (d > 0).float().mean().item())
idx = (d.amax(dim=-1) > 0).nonzero()
print("first differing voxels (n,z,y,x):", idx[:10].tolist())
for ax, name in ((1, "z"), (2, "y"), (3, "x")):
    m = (d.amax(dim=-1) > 0).float()
    dims = [a for a in (0, 1, 2, 3) if a != ax]
    print(name, "differing fraction by coordinate:", [round(v, 2) for v in m.mean(dim=dims).tolist()][:16])
chan = (d > 0).float().mean(dim=(0, 1, 2, 3))
print("by channel:", [round(v, 2) for v in chan.tolist()])
