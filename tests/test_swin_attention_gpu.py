"""MONAI SwinUNETR WindowAttention on the engine (csrc/attention.hip + mmseg_bgemm_nt) against the CPU
restatement of MONAI's forward in oracle/ (MONAI is absent: parity vs MONAI itself is unpinned).
Window 4x4x4 (64 tokens) and the SwinUNETR 7x7x7 window at head_dim 16 (feature_size 48 / 3 heads), with
and without the shifted-window mask; forward, input gradient and every parameter gradient (including the
relative-position bias table).  fp32 1e-4, bf16 3e-2 (L2) normwise."""
import pytest
import torch

import mmseg_amd  # noqa: F401
from mmseg_amd.models.backbones.swin_unetr import WindowAttention, relative_position_index
from oracle import mmseg_oracle as O
from tests.helpers import rel

pytestmark = pytest.mark.gpu


def rel2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 3e-2)])
@pytest.mark.parametrize("dim,heads,ws,nwin,nb,masked", [
    (32, 2, (4, 4, 4), 4, 2, True),      # 2 images x 4 windows, shifted-window mask
    (48, 3, (7, 7, 7), 2, 1, False),     # SwinUNETR stage-1 geometry (343 tokens, head_dim 16)
    (48, 3, (7, 7, 7), 2, 2, True),
])
def test_window_attention_vs_oracle(dev, dtype, tol, dim, heads, ws, nwin, nb, masked):
    torch.manual_seed(dim + heads)
    m = WindowAttention(dim, heads, ws, qkv_bias=True, engine_dtype=dtype).to(dev)
    with torch.no_grad():
        m.relative_position_bias_table.normal_(0, 0.5)      # make the bias matter
    n = ws[0] * ws[1] * ws[2]
    g = torch.Generator().manual_seed(7)
    x = torch.randn(nb * nwin, n, dim, generator=g)
    mask = None
    if masked:    # shifted-window style mask: 0 within a region, -100 across regions
        region = torch.randint(0, 3, (nwin, n), generator=g)
        mask = torch.where(region[:, :, None] == region[:, None, :], 0.0, -100.0)
    cot = torch.randn(nb * nwin, n, dim, generator=g)
    xd = x.to(dev).requires_grad_(True)
    out = m(xd, None if mask is None else mask.to(dev))
    (out * cot.to(dev)).sum().backward()
    p = {k: v.detach().cpu().double().requires_grad_(True) for k, v in m.named_parameters()}
    xr = x.double().requires_grad_(True)
    ref = O.window_attention(p, "", xr, None if mask is None else mask.double(), heads,
                             relative_position_index(ws))
    (ref * cot.double()).sum().backward()
    cmp = rel if dtype == torch.float32 else rel2
    assert cmp(out, ref) < tol
    assert cmp(xd.grad, xr.grad) < tol
    for name, prm in m.named_parameters():
        assert cmp(prm.grad, p[name].grad) < 2 * tol, name


def test_relative_position_index_matches_monai_layout():
    idx = relative_position_index((2, 3, 4))
    assert idx.shape == (24, 24)
    assert idx.min() == 0 and idx.max() == (3 * 5 * 7) - 1
    assert torch.equal(idx.diagonal(), torch.full((24,), (1 * 5 * 7) + 2 * 7 + 3))   # zero offset -> centre row
