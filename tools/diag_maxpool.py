"""Diagnostic: are the engine-vs-fp64 gradient differences at the first layers
explained by MaxPool argmax near-ties?  Re-run the fp64 oracle with every
MaxPool3d routed through the ENGINE's argmax indices and compare."""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mmseg_amd  # noqa: E402,F401
from oracle import mmseg_oracle as O  # noqa: E402
from tests.helpers import rel  # noqa: E402
from tests.test_model_gpu import TINY, _build, _inputs  # noqa: E402
from mmseg_amd.trainer.trainer import Trainer  # noqa: E402


def routed_pool_factory(idx_list):
    it = iter(idx_list)
    orig = F.max_pool3d

    def pool(x, k, *a, **kw):
        idx = next(it)  # [N, Do, Ho, Wo, C] uint8 sub-index 0..7
        N, C, D, H, W = x.shape
        t = idx.permute(0, 4, 1, 2, 3).long().cpu()
        parts = []
        for s in range(8):
            a_, b_, c_ = s >> 2, (s >> 1) & 1, s & 1
            parts.append(x[:, :, a_::2, b_::2, c_::2])
        stack = torch.stack(parts, dim=-1)
        return torch.gather(stack, -1, t.unsqueeze(-1)).squeeze(-1)
    return pool, orig


def main(tag="dual_tiny_attention"):
    dev = torch.device("cuda", 0)
    cfg, m, g, M, C = _build(tag)
    xs, ys = _inputs(g, M, C)
    kind, _, _, fusion, lossname = TINY[tag]
    fwd = O.unet3d_forward if kind == "unet" else (lambda pp, x: O.dual_encoder_forward(pp, x, fusion))
    tr = Trainer(cfg, m)
    for step in range(2):
        out = m(xs[step].to(dev))
        loss = tr.criterion(out, ys[step].to(dev))
        m.zero_grad(set_to_none=True)
        loss.backward()
        prog = m.backbone.__dict__["_engine"].program
        if kind == "unet":
            idxs = [prog.idx[l].view(prog.pooled[l].N, *prog.dims[l], prog.pooled[l].C) for l in range(1, prog.L)]
        else:
            idxs = [prog.idx[mm][l].view(prog.pooled[mm][l].N, *prog.dims[l], prog.pooled[mm][l].C)
                    for mm in range(prog.M) for l in range(1, prog.L)]
        res = {}
        for mode in ("free", "routed"):
            params = {n: p.detach().cpu().double().requires_grad_(True) for n, p in m.backbone.named_parameters()}
            if mode == "routed":
                pool, orig = routed_pool_factory(idxs)
                O.F.max_pool3d = pool
            try:
                rl = O.dice_ce_loss(fwd(params, xs[step].double()), ys[step])
                rl.backward()
            finally:
                if mode == "routed":
                    O.F.max_pool3d = orig
            res[mode] = params
        worst = []
        for n, p in m.backbone.named_parameters():
            if n.endswith(("conv1.bias", "conv2.bias")):
                continue
            worst.append((rel(p.grad, res["free"][n].grad), rel(p.grad, res["routed"][n].grad), n))
        worst.sort(reverse=True)
        print(f"step {step}: worst (err vs fp64 free-argmax, err vs fp64 engine-argmax, param):")
        for w in worst[:6]:
            print(f"   {w[0]:.3e}  {w[1]:.3e}  {w[2]}")
        tr.optimizer.step()


if __name__ == "__main__":
    main(*sys.argv[1:])
