"""Diagnostic: locate where engine and fp64 oracle gradients diverge inside a
DualEncoder(attention) step (teacher-forced at step 1)."""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mmseg_amd  # noqa: E402,F401
from oracle import mmseg_oracle as O  # noqa: E402
from tests.helpers import rel  # noqa: E402
from tests.test_model_gpu import _build, _inputs  # noqa: E402
from mmseg_amd.trainer.trainer import Trainer  # noqa: E402


FUSION = os.environ.get("DIAG_FUSION", "attention")


def block(p, pre, x, keep):
    x1 = F.conv3d(x, p[pre + "conv1.weight"], p[pre + "conv1.bias"], padding=1)
    x1.retain_grad()
    y1 = torch.relu(F.instance_norm(x1, eps=1e-5))
    x2 = F.conv3d(y1, p[pre + "conv2.weight"], p[pre + "conv2.bias"], padding=1)
    x2.retain_grad()
    y2 = torch.relu(F.instance_norm(x2, eps=1e-5))
    y2.retain_grad()
    keep[pre] = (x1, x2, y2)
    return y2


def oracle_fwd(p, x, keep):
    M = x.shape[1]
    per = []
    for m in range(M):
        f = block(p, f"encoders.{m}.init_conv.", x[:, m:m + 1], keep)
        fl = [f]
        for i in range(4):
            pl = F.max_pool3d(f, 2)
            pl.retain_grad()
            keep[("pooled", m, i + 1)] = pl
            f = block(p, f"encoders.{m}.blocks.{i}.conv.", pl, keep)
            fl.append(f)
        per.append(fl)
    fused = []
    keep["pooled_mean"], keep["w"] = [], []
    for l in range(5):
        st = torch.stack([pm[l] for pm in per], dim=1)
        if FUSION == "attention":
            B, Mm, Cc = st.shape[:3]
            pooled = st.reshape(B, Mm * Cc, -1).mean(dim=-1)
            pooled.retain_grad()
            pre = f"fusion_layers.{l}."
            h = torch.relu(F.linear(pooled, p[pre + "attention.2.weight"], p[pre + "attention.2.bias"]))
            w = torch.softmax(F.linear(h, p[pre + "attention.4.weight"], p[pre + "attention.4.bias"]), dim=1)
            fz = (st * w.view(B, Mm, 1, 1, 1, 1)).sum(dim=1)
            keep["pooled_mean"].append(pooled)
            keep["w"].append(w)
        else:
            fz = st.mean(dim=1)
        fz.retain_grad()
        fused.append(fz)
    keep["fused"] = fused
    keep["per"] = per
    y = fused[-1]
    for j, skip in enumerate(reversed(fused[:-1])):
        y = O.up_block(p, f"decoder.{j}.", y, skip)
    return F.conv3d(y, p["out_conv.weight"], p["out_conv.bias"])


def _gpu_dy(prog, m, l):
    """reconstruct the engine's effective dy of level output (m, l) from its buffers (mean fusion)"""
    dfused = prog.fused_out(l).to_ncdhw().double().cpu()
    dy = dfused / prog.M if FUSION != "attention" else torch.zeros_like(dfused)
    if FUSION == "attention":
        w = prog.gate_w[l].double().cpu()
        beta = prog.gate_beta[l].double().cpu()
        C = dfused.shape[1]
        dy = dfused * w[:, m].view(-1, 1, 1, 1, 1) + beta[:, m * C:(m + 1) * C].view(-1, C, 1, 1, 1)
    if l < prog.L - 1:
        dp = prog.pooled[m][l + 1].to_ncdhw().double().cpu()
        N, C, Do, Ho, Wo = dp.shape
        it = prog.idx[m][l + 1].view(N, Do, Ho, Wo, C).permute(0, 4, 1, 2, 3).long().cpu()
        for t in range(8):
            a, b, c = t >> 2, (t >> 1) & 1, t & 1
            dy[:, :, a::2, b::2, c::2] += (it == t).double() * dp
    return dy


def main():
    dev = torch.device("cuda", 0)
    cfg, m, g, M, C = _build("dual_tiny_attention" if FUSION == "attention" else "dual_tiny_cross_attention")
    xs, ys = _inputs(g, M, C)
    tr = Trainer(cfg, m)
    for step in range(2):
        out = m(xs[step].to(dev))
        loss = tr.criterion(out, ys[step].to(dev))
        m.zero_grad(set_to_none=True)
        loss.backward()
        prog = m.backbone.__dict__["_engine"].program
        keep = {}
        p = {n: q.detach().cpu().double().requires_grad_(True) for n, q in m.backbone.named_parameters()}
        ro = oracle_fwd(p, xs[step].double(), keep)
        O.dice_ce_loss(ro, ys[step]).backward()
        print(f"--- step {step}: logits {rel(out, ro):.2e}")
        for l in range(5):
            line = f" level {l}: dfused {rel(prog.fused_out(l).to_ncdhw(), keep['fused'][l].grad):.2e}"
            if FUSION == "attention":
                V = keep["per"][0][l][0, 0].numel()
                line += (f"  w {rel(prog.gate_w[l], keep['w'][l]):.2e}  beta {rel(prog.gate_beta[l] * V, keep['pooled_mean'][l].grad):.2e}"
                         f"  pooled {rel(prog.pooled_mean[l], keep['pooled_mean'][l]):.2e}")
            print(line)
        for mm in range(M):
            for l in range(5):
                pre = f"encoders.{mm}.init_conv." if l == 0 else f"encoders.{mm}.blocks.{l - 1}.conv."
                blk = prog.encs[mm][l]
                x1, x2, y2 = keep[pre]
                # after backward the engine holds g2 in x2's buffer and g1 in x1's buffer
                extra = ""
                if l >= 1:
                    extra = f"  dp {rel(prog.pooled[mm][l].to_ncdhw(), keep[('pooled', mm, l)].grad):.2e}"
                gdy = _gpu_dy(prog, mm, l)
                diff = (gdy - y2.grad).abs()
                nbad = int((diff > 1e-3 * y2.grad.abs().max()).sum())
                extra += f"  dy {rel(gdy, y2.grad):.2e} (bad elems {nbad}/{diff.numel()})"
                print(f"  m{mm} L{l}: g2 {rel(blk.x2.to_ncdhw(), x2.grad):.2e}  g1 {rel(blk.x1.to_ncdhw(), x1.grad):.2e}" + extra +
                      f"  dW2 {rel(m.backbone.get_parameter(pre + 'conv2.weight').grad, p[pre + 'conv2.weight'].grad):.2e}"
                      f"  dW1 {rel(m.backbone.get_parameter(pre + 'conv1.weight').grad, p[pre + 'conv1.weight'].grad):.2e}")
        tr.optimizer.step()


if __name__ == "__main__":
    main()
