"""Where does the SwinUNETR dropout forward differ from the oracle?  Per-stage features (hs[0..4]) and logits,
engine (fp32) vs oracle (fp64) fed the engine's masks, for drop_rate 0 and 0.2."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import mmseg_amd  # noqa: F401
    from mmseg_amd.models.backbones.swin_unetr import SwinUNETR
    from oracle import swin_oracle as SO
    from tests.helpers import rel
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(21)
    x = torch.randn(2, 2, 64, 64, 64, generator=g)
    for p in (0.0, 0.2):
        torch.manual_seed(1)
        m = SwinUNETR(img_size=(64,) * 3, in_channels=2, out_channels=3, feature_size=24, drop_rate=p)
        with torch.no_grad():      # the tests' non-trivial LayerNorm affines and bias tables
            for name, prm in m.named_parameters():
                if "norm" in name or "relative_position_bias_table" in name:
                    prm.add_(0.1 * torch.randn_like(prm))
        m = m.to(dev)
        out, feats = m(x.to(dev), return_features=True)
        seeds = dict(m.__dict__["_engine"].program.drop_seeds)
        pr = {k: v.detach().cpu().double() for k, v in m.model.named_parameters()}
        drop = SO.make_drop(p, seeds) if p > 0 else None
        hs = SO.swin_transformer(pr, "swinViT.", x.double(), m.depths, m.num_heads, (7, 7, 7),
                                 SO.relative_position_index((7, 7, 7)), True, drop)
        ref = SO.swin_unetr_forward(pr, x.double(), m.depths, m.num_heads, drop=drop)
        print(f"p={p}: logits {rel(out, ref):.3e}; hs " + " ".join(f"{rel(f, h):.3e}" for f, h in zip(feats, hs)))


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def blocks():
    """Stage 1, block by block: engine's saved xm (after the attention residual) / block output vs the oracle."""
    import mmseg_amd  # noqa: F401
    from mmseg_amd.models.backbones.swin_unetr import SwinUNETR
    from oracle import swin_oracle as SO
    from tests.helpers import rel
    import torch.nn.functional as F
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(21)
    x = torch.randn(2, 2, 64, 64, 64, generator=g)
    for p in (0.0, 0.2):
        torch.manual_seed(1)
        m = SwinUNETR(img_size=(64,) * 3, in_channels=2, out_channels=3, feature_size=24, drop_rate=p)
        with torch.no_grad():
            for name, prm in m.named_parameters():
                if "norm" in name or "relative_position_bias_table" in name:
                    prm.add_(0.1 * torch.randn_like(prm))
        m = m.to(dev)
        m.train()
        out = m(x.to(dev))
        prog = m.__dict__["_engine"].program
        seeds = dict(prog.drop_seeds)
        pr = {k: v.detach().cpu().double() for k, v in m.model.named_parameters()}
        drop = SO.make_drop(p, seeds) if p > 0 else None
        x0 = F.conv3d(x.double(), pr["swinViT.patch_embed.proj.weight"], pr["swinViT.patch_embed.proj.bias"], stride=2)
        if drop:
            x0 = drop(x0, "pos")
        h = x0.permute(0, 2, 3, 4, 1)
        b, d, hh, w, c = h.shape
        window = (7, 7, 7)
        shift_full = (3, 3, 3)
        ws, ss = SO.get_window_size((d, hh, w), window, shift_full)
        dp, hp, wp = [-(-s // ws[i]) * ws[i] for i, s in enumerate((d, hh, w))]
        mask = SO.compute_mask((dp, hp, wp), ws, ss).double()
        index = SO.relative_position_index(window)
        st = prog.stages[0]
        for j in range(2):
            pre = f"swinViT.layers1.0.blocks.{j}."
            sv = st.saved[j]
            eng_in = sv["x"].float().cpu().view(b, d, hh, w, c)
            print(f"p={p} block {j}: input {rel(eng_in, h):.3e}", end=" ")
            shift = (0, 0, 0) if j == 0 else shift_full
            hn = SO.swin_block(pr, pre, h, mask, window, shift, 3, index, drop)
            # xm: engine after the attention residual
            eng_xm = sv["xm"].float().cpu().view(b, d, hh, w, c)
            hm = SO.swin_block(pr, pre, h, mask, window, shift, 3, index,
                               (lambda t, site: drop(t, site) if site.endswith("proj") else t * 0) if drop else None)
            if drop is None:
                hm = None
            if hm is not None:
                print(f"xm {rel(eng_xm, hm):.3e}", end=" ")
                zz = F.layer_norm(hm, (c,), pr[pre + "norm2.weight"], pr[pre + "norm2.bias"], 1e-5)
                zz = F.gelu(F.linear(zz, pr[pre + "mlp.linear1.weight"], pr[pre + "mlp.linear1.bias"]))
                gd = drop(zz, pre + "drop1")
                eg = sv["g"].float().cpu().view(gd.shape)
                diff = (eg.double() - gd).abs()
                print(f"g {rel(eg, gd):.3e} (n>1e-3: {(diff > 1e-3).sum().item()}, zero-pattern mismatches: "
                      f"{((eg == 0) != (gd == 0)).sum().item()})", end=" ")
            h = hn
        cat = st.msaved[0].float().cpu()
        hc = h
        if d % 2 or hh % 2 or w % 2:
            hc = F.pad(hc, (0, 0, 0, w % 2, 0, hh % 2, 0, d % 2))
        ocat = torch.cat([hc[:, i::2, j::2, k::2, :] for i, j, k in SO.MERGE_ORDER], -1).reshape(cat.shape)
        print(f"merge cat {rel(cat, ocat):.3e}", end=" ")
        y = prog.xs[1].float().cpu().view(b, d // 2, hh // 2, w // 2, 2 * c)
        oy = SO.patch_merging(pr, "swinViT.layers1.0.downsample.", h)
        print(f"stage out {rel(y, oy):.3e}")


if __name__ == "__main__" and len(sys.argv) > 1:
    blocks()
