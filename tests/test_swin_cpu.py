"""SwinUNETR host-side checks (CPU): MONAI module tree / state-dict names and parameter count of the
containers, the shifted-window mask plan against the oracle's compute_mask, the oracle's own shape
bookkeeping, and that the product model refuses a CPU input (no CPU fallback)."""
import numpy as np
import pytest
import torch

import mmseg_amd  # noqa: F401
from mmseg_amd.engine.swin import shift_mask, window_size_for
from mmseg_amd.models.backbones.swin_unetr import SwinUNETR
from mmseg_amd.models.build import build_model
from oracle import swin_oracle as SO


def test_state_dict_follows_monai_names():
    m = SwinUNETR(img_size=(128, 128, 128), in_channels=2, out_channels=6, feature_size=48)
    keys = set(m.state_dict())
    for k in ("model.swinViT.patch_embed.proj.weight", "model.swinViT.layers1.0.blocks.1.attn.qkv.weight",
              "model.swinViT.layers1.0.blocks.1.attn.relative_position_index",
              "model.swinViT.layers4.0.downsample.reduction.weight", "model.swinViT.layers2.0.downsample.norm.bias",
              "model.swinViT.layers3.0.blocks.0.mlp.linear2.bias", "model.encoder1.layer.conv3.conv.weight",
              "model.encoder10.layer.conv2.conv.weight", "model.decoder5.transp_conv.conv.weight",
              "model.decoder1.conv_block.conv3.conv.weight", "model.out.conv.conv.bias"):
        assert k in keys, k
    assert "model.encoder2.layer.conv3.conv.weight" not in keys         # same channels: identity residual
    assert sum(p.numel() for p in m.parameters()) == 62_188_632   # fs=48, 2 -> 6 (MONAI's is ~62.2 M)


def test_build_model_registry():
    cfg = {"model": {"name": "swin_unetr", "out_channels": 3, "backbone": {"img_size": [64, 64, 64],
                                                                        "feature_size": 24}},
           "data": {"modalities": ["CT", "PET"]}, "hardware": {"device": "cpu"}}
    model = build_model(cfg)
    assert cfg["model"]["in_channels"] == 2
    with pytest.raises(RuntimeError):
        model(torch.randn(1, 2, 64, 64, 64))


@pytest.mark.parametrize("dims,window", [((35, 35, 35), (7, 7, 7)), ((14, 14, 14), (7, 7, 7)),
                                         ((4, 4, 4), (7, 7, 7))])
def test_shift_mask_matches_oracle(dims, window):
    ws, ss = window_size_for(dims, window, (3, 3, 3))
    assert (ws, ss) == SO.get_window_size(dims, window, (3, 3, 3))
    if not any(ss):
        return
    got = shift_mask(dims, ws, ss)
    ref = SO.compute_mask(dims, ws, ss).numpy()
    assert np.array_equal(got, ref)


def test_oracle_shapes():
    torch.manual_seed(0)
    m = SwinUNETR(img_size=(64, 64, 64), in_channels=2, out_channels=3, feature_size=24)
    p = {k: v.detach() for k, v in m.model.named_parameters()}
    x = torch.randn(1, 2, 64, 64, 64)
    hs = SO.swin_transformer(p, "swinViT.", x, m.depths, m.num_heads, (7, 7, 7), SO.relative_position_index((7,) * 3))
    assert [h.shape[1:] for h in hs] == [(24, 32, 32, 32), (48, 16, 16, 16), (96, 8, 8, 8), (192, 4, 4, 4),
                                         (384, 2, 2, 2)]
    out = SO.swin_unetr_forward(p, x, m.depths, m.num_heads)
    assert out.shape == (1, 3, 64, 64, 64) and torch.isfinite(out).all()
