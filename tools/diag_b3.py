import os, sys, torch, torch.nn as nn, torch.nn.functional as F
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import mmseg_amd
from mmseg_amd.engine.layers import Conv3
from mmseg_amd.engine.runtime import Act, FlatParams, Runtime
from tests.helpers import from_ndhwc, to_ndhwc
dev = torch.device("cuda", 0)
for dtype in (torch.float32, torch.bfloat16):
    torch.manual_seed(0)
    cin, cout, (N, D, H, W) = 32, 32, (1, 4, 8, 8)
    conv = nn.Conv3d(cin, cout, 3, padding=1).to(dev)
    with torch.no_grad():
        conv.weight.zero_(); conv.bias.zero_()
        for c in range(32): conv.weight[c, c, 1, 1, 1] = 1.0   # identity
    rt = Runtime(dev, dtype); flat = FlatParams(list(conv.parameters())); layer = Conv3(rt, conv, flat)
    x = torch.zeros(N, cin, D, H, W, device=dev)
    x[0, :, 1, 2, 3] = torch.arange(32, device=dev).float() + 1
    xa = Act(to_ndhwc(x, dtype), 0, cin, cin, N, D, H, W); ya = rt.act(N, D, H, W, cout)
    layer.pack(); layer.fwd(xa, ya)
    out = from_ndhwc(ya.buf, N, cout, D, H, W).float().cpu()
    nz = out.nonzero()
    print(dtype, rt.lib.mmseg_last_kernel(), "nonzeros", nz.shape[0])
    for idx in nz[:40].tolist():
        print(idx, out[tuple(idx)].item())
