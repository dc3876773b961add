"""Mixed bf16/fp8 (config c5, `hardware.fp8: true`): the forward 3^3 convolutions the brick6 kernel takes run with
OCP e4m3 operands (weights scaled per output channel to max |w| = 448, activations at unit scale) and fp32
accumulation; everything else stays bf16 / fp32.

Parity is stated two ways:
  * the kernel against an fp64 evaluation of the same e4m3-quantised operands (torch.float8_e4m3fn, round to
    nearest even): only the fp32 accumulation and the bf16 output rounding differ -> 1e-2 normwise;
  * the model (tiny c5: DualEncoder, CT+PET+MRI, Tversky) in mixed bf16/fp8 against the same model in bf16:
    e4m3 keeps 3 mantissa bits (rounding error ~3.6 % rms per operand), so every fp8 conv output moves by ~5 % of
    its norm on a random-init net, and the two fp8 layers on each path compound: logits within 0.2 normwise
    (measured 0.118; max-abs 0.144 of the largest logit), training loss within 3e-2 relative (measured 1.5e-5).
There is no reference number for fp8 (the reference runs fp16 autocast); parity vs the reference is the bf16 path's.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import mmseg_amd  # noqa: F401
from mmseg_amd.engine.layers import Conv3
from mmseg_amd.engine.runtime import Act, FlatParams, Runtime
from mmseg_amd.models.build import build_model
from mmseg_amd.trainer.trainer import Trainer
from tests.helpers import from_ndhwc, rel, to_ndhwc
from tests.test_model_gpu import make_config

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _brick2_small_volumes(monkeypatch):
    """The e4m3 forward is a brick2-family kernel; these small test volumes would otherwise fall under
    MMSEG_BRICK2_MINUNITS and take the runtime-brick kernel, which has no fp8 form (the 96^3 layers fp8 serves
    are far above it)."""
    monkeypatch.setenv("MMSEG_BRICK2_MINUNITS", "0")


def _e4m3(t):
    return t.float().to(torch.float8_e4m3fn).double()


@pytest.mark.parametrize("norm", [False, True])
@pytest.mark.parametrize("shape", [(2, 8, 8, 16), (1, 8, 16, 32), (2, 4, 8, 16)])
def test_conv3_fp8_matches_quantized_reference(dev, norm, shape):
    N, D, H, W = shape
    torch.manual_seed(1)
    rt = Runtime(dev, torch.bfloat16, fp8=True)
    conv = nn.Conv3d(32, 32, 3, padding=1).to(dev)
    flat = FlatParams(list(conv.parameters()))
    layer = Conv3(rt, conv, flat)
    x = torch.randn(N, 32, D, H, W, device=dev) * 2.0 + 0.3
    xa = Act(to_ndhwc(x, torch.bfloat16), 0, 32, 32, N, D, H, W)
    ya = rt.act(N, D, H, W, 32)
    assert layer.fp8_ok(xa, ya)
    mean = (torch.randn(N * 32, device=dev) * 0.3).contiguous()
    rstd = (torch.rand(N * 32, device=dev) + 0.5).contiguous()
    layer.fwd_fp8(xa, ya, norm=(mean, rstd) if norm else None)
    torch.cuda.synchronize()
    assert rt.lib.mmseg_last_kernel().decode() == "conv3_brick6_kernel<BN32,F8>"
    out = from_ndhwc(ya.buf, N, 32, D, H, W).double().cpu()
    # reference: the kernel's staged values (bf16 input, optional fp32 norm + ReLU) and weights, e4m3-rounded
    xb = x.to(torch.bfloat16).float().cpu()
    if norm:
        mu = mean.view(N, 32, 1, 1, 1).cpu()
        rs = rstd.view(N, 32, 1, 1, 1).cpu()
        xb = torch.relu((xb - mu) * rs)
    w = conv.weight.detach().float().cpu()
    s = 448.0 / w.abs().amax(dim=(1, 2, 3, 4))
    wq = _e4m3(w * s.view(-1, 1, 1, 1, 1))
    ref = F.conv3d(_e4m3(xb), wq, padding=1) / s.double().view(1, -1, 1, 1, 1) + conv.bias.detach().double().cpu().view(1, -1, 1, 1, 1)
    assert rel(out, ref) < 1e-2, rel(out, ref)


def _c5_tiny(fp8):
    cfg = make_config("dual_encoder", ["CT", "PET", "MRI"], 4, [32, 64, 128], loss="tversky", dtype="bfloat16")
    cfg["hardware"]["fp8"] = fp8
    torch.manual_seed(3)
    return cfg, build_model(cfg)


def test_fp8_c5_tiny_close_to_bf16(dev):
    gen = torch.Generator().manual_seed(7)
    x = torch.randn(2, 3, 32, 32, 32, generator=gen)
    y = torch.randint(0, 4, (2, 32, 32, 32), generator=gen)
    res = {}
    for fp8 in (False, True):
        cfg, m = _c5_tiny(fp8)
        m.eval()
        with torch.no_grad():
            logits = m(x.to(dev)).float().cpu()
        tr = Trainer(cfg, m)
        losses = [tr.train_step({"image": x, "label": y}, i) for i in range(2)]
        res[fp8] = (logits, losses)
        if fp8:   # the encoders' and the decoder's top conv2 ran on the e4m3 kernel
            prog = m.backbone.__dict__["_engine"].program
            assert all(prog.encs[k][0].c2._f8 is not None for k in range(3)) and prog.dec.blocks[-1].c2._f8 is not None
    a, b = res[True][0].double(), res[False][0].double()
    nrel = ((a - b).norm() / b.norm()).item()
    print(f"fp8 vs bf16: logits normwise {nrel:.4f}, max-abs rel {rel(a, b):.4f}, losses {res[True][1]} vs {res[False][1]}")
    assert nrel < 0.2, nrel
    assert all(np.isfinite(res[True][1]))
    assert abs(res[True][1][0] - res[False][1][0]) < 3e-2 * abs(res[False][1][0]), (res[True][1], res[False][1])
