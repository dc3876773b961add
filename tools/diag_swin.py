"""Diagnostic: per-parameter gradient errors of the SwinUNETR engine vs the fp64 oracle."""
import sys
import torch
sys.path.insert(0, ".")
import mmseg_amd  # noqa
from tests.test_swin_unetr_gpu import _model, _oracle
from tests.helpers import rel

dev = torch.device("cuda", 0)
size = int(sys.argv[1]) if len(sys.argv) > 1 else 64
g = torch.Generator().manual_seed(21)
x = torch.randn(2, 2, size, size, size, generator=g)
cot = torch.randn(2, 3, size, size, size, generator=g)
m = _model(dev, torch.float32)
out = m(x.to(dev))
(out * cot.to(dev)).sum().backward()
ref, grads = _oracle(m, x, cot)
print("logits", rel(out, ref))
for name, prm in m.model.named_parameters():
    r = grads[name]
    print(f"{name:60s} {rel(prm.grad, r):.3e}  |g|max {r.abs().max().item():.3e}")
