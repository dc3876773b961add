"""Diagnostic: bf16 SwinUNETR engine per-parameter L2 gradient errors vs the fp32 oracle."""
import sys
import torch
sys.path.insert(0, ".")
import mmseg_amd  # noqa
from tests.test_swin_unetr_gpu import _model, _oracle, rel2

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(21)
x = torch.randn(2, 2, 64, 64, 64, generator=g)
cot = torch.randn(2, 3, 64, 64, 64, generator=g)
m = _model(dev, torch.bfloat16)
out = m(x.to(dev))
(out * cot.to(dev)).sum().backward()
ref, grads = _oracle(m, x, cot, torch.float32)
print("logits", rel2(out, ref))
errs = sorted(((rel2(p.grad, grads[n]), n) for n, p in m.model.named_parameters() if grads[n].norm() > 0),
              reverse=True)
for e, n in errs:
    print(f"{n:60s} {e:.3e}")
got = torch.cat([p.grad.reshape(-1).double().cpu() for n, p in m.model.named_parameters() if grads[n].norm() > 0])
want = torch.cat([grads[n].reshape(-1).double() for n, p in m.model.named_parameters() if grads[n].norm() > 0])
print("all-gradient L2", ((got - want).norm() / want.norm()).item())
