"""Teacher-forced gradient diagnostics (GPU): per-parameter error of the engine
and of the fp32 oracle against the fp64 oracle, for a tiny golden config.

    python tools/diag_tf.py [tag] [steps]
Env knobs (MMSEG_*) select kernel variants, so two runs localise a kernel.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "unet_tiny"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    import mmseg_amd  # noqa: F401
    from mmseg_amd.trainer.trainer import Trainer
    from oracle import mmseg_oracle as O
    from tests.helpers import rel
    from tests.test_model_gpu import TINY, _build, _inputs

    cfg, m, g, M, C = _build(tag)
    xs, ys = _inputs(g, M, C)
    kind, _, _, fusion, lossname = TINY[tag]
    fwd = O.unet3d_forward if kind == "unet" else (lambda pp, x: O.dual_encoder_forward(pp, x, fusion))
    lossf = O.dice_ce_loss if lossname == "dice_ce" else O.tversky_loss
    tr = Trainer(cfg, m)
    dev = torch.device("cuda", 0)
    env = {k: v for k, v in os.environ.items() if k.startswith("MMSEG_")}
    print("env", env)
    for i in range(steps):
        refs = {}
        for dt in (torch.float32, torch.float64):
            params = {n: p.detach().cpu().to(dt).requires_grad_(True) for n, p in m.backbone.named_parameters()}
            ro = fwd(params, xs[i].to(dt))
            rl = lossf(ro, ys[i])
            rl.backward()
            refs[dt] = (ro, rl, params)
        out = m(xs[i].to(dev))
        loss = tr.criterion(out, ys[i].to(dev))
        m.zero_grad(set_to_none=True)
        loss.backward()
        r32, r64 = refs[torch.float32], refs[torch.float64]
        print(f"step {i}: logits {rel(out, r64[0]):.2e} (fp32 oracle {rel(r32[0], r64[0]):.2e}) "
              f"loss {loss.item():.6f} vs {r64[1].item():.6f}")
        for n, p in m.backbone.named_parameters():
            e = rel(p.grad, r64[2][n].grad)
            e32 = rel(r32[2][n].grad, r64[2][n].grad)
            flag = " <<<" if e > max(10 * e32, 1e-4) else ""
            print(f"  {n:45s} {tuple(p.shape)!s:22s} eng {e:.2e}  fp32 {e32:.2e}{flag}")
        tr.optimizer.step()


if __name__ == "__main__":
    main()
