"""Diagnostic: decoder1 backward intermediates of the SwinUNETR engine vs fp64 oracle."""
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, ".")
import mmseg_amd  # noqa
from tests.test_swin_unetr_gpu import _model
from tests.helpers import rel
from oracle import swin_oracle as SO

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(21)
x = torch.randn(2, 2, 64, 64, 64, generator=g)
cot = torch.randn(2, 3, 64, 64, 64, generator=g)
m = _model(dev, torch.float32)
out = m(x.to(dev))
(out * cot.to(dev)).sum().backward()
prog = m.__dict__["_engine"].program
p = {k: v.detach().cpu().double().requires_grad_(True) for k, v in m.model.named_parameters()}
xr = x.double()
idx = SO.relative_position_index((7, 7, 7))
hs = SO.swin_transformer(p, "swinViT.", xr, m.depths, m.num_heads, (7, 7, 7), idx)
enc0 = SO.unet_res_block(p, "encoder1.layer.", xr)
enc1 = SO.unet_res_block(p, "encoder2.layer.", hs[0])
enc2 = SO.unet_res_block(p, "encoder3.layer.", hs[1])
enc3 = SO.unet_res_block(p, "encoder4.layer.", hs[2])
dec4 = SO.unet_res_block(p, "encoder10.layer.", hs[4])
dec3 = SO.unetr_up_block(p, "decoder5.", dec4, hs[3])
dec2 = SO.unetr_up_block(p, "decoder4.", dec3, enc3)
dec1 = SO.unetr_up_block(p, "decoder3.", dec2, enc2)
dec0 = SO.unetr_up_block(p, "decoder2.", dec1, enc1)
pre = "decoder1."
up = F.conv_transpose3d(dec0, p[pre + "transp_conv.conv.weight"], stride=2)
cat = torch.cat([up, enc0], 1)
cat.retain_grad()
b = pre + "conv_block."
a1 = F.conv3d(cat, p[b + "conv1.conv.weight"], padding=1); a1.retain_grad()
h1 = F.leaky_relu(F.instance_norm(a1, eps=1e-5), 0.01); h1.retain_grad()
a2 = F.conv3d(h1, p[b + "conv2.conv.weight"], padding=1); a2.retain_grad()
n2 = F.instance_norm(a2, eps=1e-5)
a3 = F.conv3d(cat, p[b + "conv3.conv.weight"]); a3.retain_grad()
n3 = F.instance_norm(a3, eps=1e-5)
prey = n2 + n3; prey.retain_grad()
o = F.leaky_relu(prey, 0.01); o.retain_grad()
logits = F.conv3d(o, p["out.conv.conv.weight"], p["out.conv.conv.bias"])
print("logits", rel(out, logits))
(logits * cot.double()).sum().backward()
u = prog.dec[4]
rb = u.res
print("d out   ", rel(prog.ddout[4].to_ncdhw(), o.grad))
print("g (pre) ", rel(rb.g.to_ncdhw(), prey.grad))
print("h1      ", rel(rb.h1.to_ncdhw(), h1))
print("a1      ", rel(rb.a1.to_ncdhw(), a1))
print("a2      ", rel(rb.a2.to_ncdhw(), a2))
print("d cat   ", rel(u.dcat.to_ncdhw(), cat.grad))
print("dW conv2", rel(m.model.decoder1.conv_block.conv2.conv.weight.grad, p[b + "conv2.conv.weight"].grad))
print("dW conv1", rel(m.model.decoder1.conv_block.conv1.conv.weight.grad, p[b + "conv1.conv.weight"].grad))
print("dW conv3", rel(m.model.decoder1.conv_block.conv3.conv.weight.grad, p[b + "conv3.conv.weight"].grad))
# conv2 weight grad from engine's own intermediates (fp64 torch): isolates the wgrad kernel
ye = prog.dout[4].to_ncdhw().cpu()
flips = ((ye > 0) != (o.detach() > 0))
print("flip count", flips.sum().item(), "of", flips.numel())
ge = rb.g.to_ncdhw().cpu().double()
print("g error outside flips", rel(ge * (~flips), prey.grad * (~flips)))
