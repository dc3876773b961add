"""Diagnostics: gradient differences of the bf16 c3 step between repeated runs and grouping modes
(MMSEG_GROUP_FORCE_R 1 / 0), optionally under extra env knobs given as KEY=VAL arguments per variant:
    python tools/diag_force.py [KEY=VAL,KEY=VAL ...]
Prints L2 differences d(1,1'), d(nf,nf'), d(1,nf) for each variant (a comma-joined knob list; '-' = none)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mmseg_amd  # noqa: F401,E402
from mmseg_amd.models.build import build_model  # noqa: E402
from mmseg_amd.trainer.trainer import Trainer  # noqa: E402
from tests.test_fullsize_gpu import CASES, _config, full_inputs  # noqa: E402


def grads(mode, x, y):
    os.environ["MMSEG_GROUP_FORCE_R"] = "0" if mode == "nf" else "1"
    model, mods, loss = CASES["fullgrad_dual_c3"]
    cfg = _config(model, mods, loss, "bfloat16")
    torch.manual_seed(3)
    m = build_model(cfg)
    tr = Trainer(cfg, m)
    m.train()
    lossv = tr._fused_loss(x, y)
    lossv.backward()
    g = torch.cat([p.grad.reshape(-1).float() for p in m.parameters()]).clone()
    names = [n for n, _ in m.named_parameters()]
    per = [p.grad.reshape(-1).float().clone() for p in m.parameters()]
    del m, tr
    return g, names, per


def main():
    dev = torch.device("cuda:0")
    x, y, _ = full_inputs(96, 2, 2, 6, 11)
    x, y = x.to(dev), y.to(dev)
    for var in (sys.argv[1:] or ["-"]):
        saved = {}
        if var != "-":
            for kv in var.split(","):
                k, v = kv.split("=")
                saved[k] = os.environ.get(k)
                os.environ[k] = v
        a, names, pa = grads("1", x, y)
        a2, _, _ = grads("1", x, y)
        b, _, pb = grads("nf", x, y)
        b2, _, _ = grads("nf", x, y)
        d = lambda u, v: float((u - v).norm() / v.norm())
        worst = sorted(((float((u - v).norm() / (v.norm() + 1e-30)), n) for u, v, n in zip(pa, pb, names)),
                       reverse=True)[:6]
        print(f"{var}: d(1,1') {d(a, a2):.2e}  d(nf,nf') {d(b, b2):.2e}  d(1,nf) {d(a, b):.2e}  worst {worst}",
              flush=True)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


if __name__ == "__main__":
    main()
