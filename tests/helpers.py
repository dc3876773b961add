"""Test helpers: NCDHW <-> NDHWC engine layout, golden fixture loading."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def to_ndhwc(x, dtype, ld=None, off=0):
    """NCDHW float tensor -> flat NDHWC device buffer (optionally inside a wider ld)."""
    N, C, D, H, W = x.shape
    ld = ld or C
    buf = torch.zeros(N, D, H, W, ld, dtype=dtype, device=x.device)
    buf[..., off:off + C] = x.permute(0, 2, 3, 4, 1).to(dtype)
    return buf.reshape(-1)


def from_ndhwc(buf, N, C, D, H, W, ld=None, off=0):
    ld = ld or C
    return buf.reshape(N, D, H, W, ld)[..., off:off + C].permute(0, 4, 1, 2, 3).float()


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    d = b.abs().max().item()
    return (a - b).abs().max().item() / (d if d > 0 else 1.0)
