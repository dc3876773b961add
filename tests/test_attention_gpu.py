"""CrossAttentionFusion on the HIP engine (reference attention_fusion.py:77-164):
the batched MFMA NT GEMM and transpose kernels against torch fp64, and the
module (forward + backward, every parameter gradient) against the golden
fixture the reference produced (tests/golden/cross_attention.npz) and against
the CPU oracle at a larger head_dim.  Tolerances: fp32 storage 1e-4
normwise (the north_star's logits bar is 1e-3); bf16 storage 3e-2 / 6e-2."""
import numpy as np
import pytest
import torch

import mmseg_amd  # noqa: F401
from mmseg_amd._lib import lib, ptr, stream_handle
from mmseg_amd.models.fusion import BidirectionalCrossAttention, CrossAttentionFusion
from oracle import mmseg_oracle as O
from tests.helpers import golden, rel

pytestmark = pytest.mark.gpu
CODE = {torch.float32: 0, torch.bfloat16: 1}


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("acc,bias,cf32", [(False, False, True), (True, True, True), (False, True, False)])
def test_bgemm_nt(dev, dtype, acc, bias, cf32):
    if dtype == torch.float32 and not cf32:
        pytest.skip("fp32 operands always produce fp32")
    g = torch.Generator().manual_seed(7)
    Bo, Bi, M, N, K = 2, 3, 70, 45, 40
    A = torch.randn(Bo, Bi, M, K + 8, generator=g)        # row stride K+8 (padding), K-contiguous
    Bm = torch.randn(Bo, Bi, N, K, generator=g)
    C0 = torch.randn(Bo, Bi, M, N + 3, generator=g)
    bv = torch.randn(N, generator=g)
    Ad, Bd = A.to(dtype).to(dev), Bm.to(dtype).to(dev)
    cdt = torch.float32 if cf32 else dtype
    Cd = C0.to(cdt).to(dev)
    alpha = 0.37
    lib().mmseg_bgemm_nt(ptr(Ad), Bi * M * (K + 8), M * (K + 8), K + 8, ptr(Bd), Bi * N * K, N * K, K, ptr(Cd),
                         Bi * M * (N + 3), M * (N + 3), N + 3, ptr(bv.to(dev)) if bias else None, Bo * Bi, Bi, M, N, K,
                         alpha, int(acc), 0 if cf32 else 1, CODE[dtype], stream_handle())
    ref = alpha * torch.einsum("abik,abjk->abij", A[..., :K].to(dtype).double(), Bm.to(dtype).double())
    if bias:
        ref = ref + bv.double()
    if acc:
        ref = ref + C0[..., :N].to(cdt).double()
    tol = 1e-5 if dtype == torch.float32 else (1e-2 if cf32 else 2e-2)
    assert rel(Cd[..., :N], ref) < tol
    assert torch.equal(Cd[..., N:].cpu(), C0[..., N:].to(cdt))     # padding columns untouched


@pytest.mark.parametrize("sdt,ddt", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_transpose(dev, sdt, ddt):
    tdt = {0: torch.float32, 1: torch.bfloat16}
    g = torch.Generator().manual_seed(8)
    x = torch.randn(2, 3, 37, 50, generator=g).to(tdt[sdt]).to(dev)
    y = torch.zeros(2, 3, 50, 40, dtype=tdt[ddt], device=dev)
    lib().mmseg_transpose(ptr(x), 3 * 37 * 50, 37 * 50, 50, sdt, ptr(y), 3 * 50 * 40, 50 * 40, 40, ddt, 6, 3, 37, 50,
                          stream_handle())
    ref = x.float().transpose(-1, -2).to(tdt[ddt])
    assert torch.equal(y[..., :37], ref)


def _load_golden_module(dtype, dev):
    gd = golden("cross_attention")
    m = CrossAttentionFusion(32, num_heads=4, engine_dtype=dtype)
    m.load_state_dict({k[2:]: torch.from_numpy(gd[k]) for k in gd.files if k.startswith("p_")})
    return m.to(dev), gd


@pytest.mark.parametrize("dtype,tol,gtol", [(torch.float32, 1e-4, 1e-4), (torch.bfloat16, 3e-2, 6e-2)])
def test_cross_attention_matches_reference_golden(dev, dtype, tol, gtol):
    m, gd = _load_golden_module(dtype, dev)
    q = torch.from_numpy(gd["q"]).to(dev).requires_grad_(True)
    kv = torch.from_numpy(gd["kv"]).to(dev).requires_grad_(True)
    out = m(q, kv)
    assert out.shape == q.shape and out.dtype == torch.float32
    assert rel(out, torch.from_numpy(gd["out"])) < tol
    (out * torch.from_numpy(gd["cot"]).to(dev)).sum().backward()
    assert rel(q.grad, torch.from_numpy(gd["dq"])) < gtol
    assert rel(kv.grad, torch.from_numpy(gd["dkv"])) < gtol
    _check_param_grads({n: p.grad for n, p in m.named_parameters()},
                       {n: torch.from_numpy(gd["g_" + n]) for n, _ in m.named_parameters()}, gtol)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 5e-2)])
def test_cross_attention_vs_oracle_hd16(dev, dtype, tol):
    """head_dim 16, 8^3 voxels (512 keys), 2 samples: forward and all gradients vs the CPU oracle."""
    torch.manual_seed(11)
    m = CrossAttentionFusion(64, num_heads=4, engine_dtype=dtype).to(dev)
    g = torch.Generator().manual_seed(12)
    q = torch.randn(2, 64, 8, 8, 8, generator=g)
    kv = torch.randn(2, 64, 8, 8, 8, generator=g)
    cot = torch.randn(2, 64, 8, 8, 8, generator=g)
    qd, kvd = q.to(dev).requires_grad_(True), kv.to(dev).requires_grad_(True)
    out = m(qd, kvd)
    (out * cot.to(dev)).sum().backward()
    p = {k: v.detach().cpu().double().requires_grad_(True) for k, v in m.named_parameters()}
    qr, kvr = q.double().requires_grad_(True), kv.double().requires_grad_(True)
    ref = O.cross_attention_fusion(p, "", qr, kvr, num_heads=4)
    (ref * cot.double()).sum().backward()
    assert rel(out, ref) < tol
    assert rel(qd.grad, qr.grad) < tol
    assert rel(kvd.grad, kvr.grad) < tol
    _check_param_grads({n: prm.grad for n, prm in m.named_parameters()}, {n: v.grad for n, v in p.items()}, 2 * tol)


@pytest.mark.parametrize("dtype,tol,gtol", [(torch.float32, 1e-4, 1e-4), (torch.bfloat16, 3e-2, 6e-2)])
def test_bidirectional_matches_reference_golden(dev, dtype, tol, gtol):
    gd = golden("bidirectional_attention")
    m = BidirectionalCrossAttention(32, num_heads=4, engine_dtype=dtype)
    m.load_state_dict({k[2:]: torch.from_numpy(gd[k]) for k in gd.files if k.startswith("p_")})
    m = m.to(dev)
    f1 = torch.from_numpy(gd["f1"]).to(dev).requires_grad_(True)
    f2 = torch.from_numpy(gd["f2"]).to(dev).requires_grad_(True)
    out = m(f1, f2)
    assert rel(out, torch.from_numpy(gd["out"])) < tol
    (out * torch.from_numpy(gd["cot"]).to(dev)).sum().backward()
    if dtype == torch.float32:
        assert rel(f1.grad, torch.from_numpy(gd["d1"])) < gtol
        assert rel(f2.grad, torch.from_numpy(gd["d2"])) < gtol
    else:   # bf16: ReLU-mask flips of near-zero normalised values move single voxels; bound the L2 error
        assert rel2(f1.grad, torch.from_numpy(gd["d1"])) < gtol
        assert rel2(f2.grad, torch.from_numpy(gd["d2"])) < gtol
    got = {n: p.grad for n, p in m.named_parameters()}
    ref = {n: torch.from_numpy(gd["g_" + n]) for n in got}
    cmp = rel if dtype == torch.float32 else rel2
    for pre in ("cross_attn_1to2.", "cross_attn_2to1."):
        _check_param_grads({k[len(pre):]: v for k, v in got.items() if k.startswith(pre)},
                           {k[len(pre):]: v for k, v in ref.items() if k.startswith(pre)}, gtol, cmp)
    assert cmp(got["fusion.0.weight"], ref["fusion.0.weight"]) < gtol
    scale = ref["fusion.0.weight"].abs().max().item()     # fusion.0.bias: a constant in front of the norm
    assert got["fusion.0.bias"].abs().max().item() <= (1e-4 if dtype == torch.float32 else 0.1) * scale


def rel2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm()).item()


def _check_param_grads(got, ref, tol, cmp=rel):
    """k_proj.bias shifts every score of a row by one constant (softmax cancels it); v_proj.bias and
    out_proj.bias add a per-channel constant in front of the InstanceNorm (which removes it).  Their
    gradients are zero in exact arithmetic and rounding noise in both implementations, so they are bounded
    against the scale of a non-zero gradient (q_proj.weight) instead of compared elementwise."""
    scale = ref["q_proj.weight"].abs().max().item()
    zero_tol = 1e-4 if tol < 1e-3 else 0.1
    for name in got:
        if name in ("k_proj.bias", "v_proj.bias", "out_proj.bias"):
            assert got[name].abs().max().item() <= zero_tol * scale, (name, got[name].abs().max().item(), scale)
            assert ref[name].abs().max().item() <= 1e-4 * scale
        else:
            assert cmp(got[name], ref[name]) < tol, name


def test_cross_attention_rejects_cpu():
    m = CrossAttentionFusion(32, num_heads=4)
    with pytest.raises(RuntimeError):
        m(torch.randn(1, 32, 2, 2, 2), torch.randn(1, 32, 2, 2, 2))
