"""Fused self-attention (kernels/attention.hip) against an fp32 PyTorch reference of the same op:
forward output and the packed dQKV gradient, with and without dropout (the dropout mask is read
back through the kernel itself with V = I, then applied to the fp32 reference)."""
import math

import pytest
import torch
import torch.nn.functional as F


def _ref(qkv, heads, mask=None, p=0.0):
    """fp32 softmax(Q K^T / sqrt(d)) (* mask / (1-p)) V from packed [B, S, 3*H*D]."""
    B, S, E = qkv.shape
    D = E // (3 * heads)
    q, k, v = qkv.view(B, S, 3, heads, D).permute(2, 0, 3, 1, 4).unbind(0)
    a = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(D), dim=-1)
    if mask is not None:
        a = a * mask / (1.0 - p)
    return (a @ v).transpose(1, 2).reshape(B, S, E // 3)


def test_attention_cpu_fallback_matches_reference():
    from parameter_server_distributed_amd.ops.attention import FusedSelfAttention

    torch.manual_seed(0)
    qkv = torch.randn(2, 16, 3 * 2 * 8)
    m = FusedSelfAttention(2, p=0.1).eval()
    torch.testing.assert_close(m(qkv), _ref(qkv, 2), atol=1e-5, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("B,S,H", [(2, 128, 3), (3, 64, 2), (2, 96, 1), (4, 32, 2)])
def test_fused_attention_matches_fp32(gpu, B, S, H):
    from parameter_server_distributed_amd.ops.attention import FusedSelfAttention

    torch.manual_seed(1)
    qkv = (torch.randn(B, S, 3 * H * 64, device=gpu) * 1.5).to(torch.bfloat16).requires_grad_(True)
    m = FusedSelfAttention(H, p=0.0).to(gpu)
    assert m._kernel_ok(qkv)
    o = m(qkv)
    g = torch.randn_like(o)
    o.backward(g)
    qr = qkv.detach().float().requires_grad_(True)
    orf = _ref(qr, H)
    orf.backward(g.float())
    torch.testing.assert_close(o.float(), orf, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(qkv.grad.float(), qr.grad, atol=3e-2, rtol=3e-2)


@pytest.mark.gpu
def test_fused_attention_dropout_mask_consistent(gpu):
    from parameter_server_distributed_amd import native

    C = native()
    torch.manual_seed(2)
    B, S, H, D, p = 2, 64, 2, 64, 0.2
    step = torch.tensor([5], device=gpu, dtype=torch.int64)
    qkv = (torch.randn(B, S, 3, H, D, device=gpu) * 0.5).to(torch.bfloat16)
    # V = I per head: O = dropout(P) V = dropout(P), so the kernel reveals its own mask
    probe = qkv.clone()
    probe[:, :, 2] = torch.eye(S, D, device=gpu, dtype=torch.bfloat16)[None, :, None, :].expand(B, S, H, D)
    po, _ = C.attn_fwd(probe.view(B, S, -1), H, p, 11, step)
    mask = (po.view(B, S, H, D).permute(0, 2, 1, 3) != 0).float()  # [B, H, q, key]
    keep = mask.mean().item()
    assert abs(keep - (1 - p)) < 0.02, keep
    # a different step draws a different mask
    po2, _ = C.attn_fwd(probe.view(B, S, -1), H, p, 11, step + 1)
    assert not torch.equal(po != 0, po2 != 0)

    x = qkv.view(B, S, -1).contiguous()
    o, lse = C.attn_fwd(x, H, p, 11, step)
    g = torch.randn_like(o)
    dqkv = C.attn_bwd(g, x, o, lse, H, p, 11, step)
    xr = x.float().requires_grad_(True)
    orf = _ref(xr, H, mask, p)
    orf.backward(g.float())
    torch.testing.assert_close(o.float(), orf, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(dqkv.float(), xr.grad, atol=3e-2, rtol=3e-2)


@pytest.mark.gpu
def test_bert_layer_uses_fused_attention(gpu):
    from parameter_server_distributed_amd.models.bert import BertLayer

    torch.manual_seed(3)
    layer = BertLayer(hidden=768, heads=12, ffn=3072, dropout=0.0).to(gpu).to(torch.bfloat16)
    x = torch.randn(2, 128, 768, device=gpu, dtype=torch.bfloat16, requires_grad=True)
    assert layer.attn._kernel_ok(layer.qkv(x))
    y = layer(x)
    y.float().sum().backward()
    # the same layer on the SDPA fallback (fp32 composite path for the attention only)
    qkv = layer.qkv(x.detach())
    B, S, E = qkv.shape
    q, k, v = qkv.float().view(B, S, 3, 12, 64).permute(2, 0, 3, 1, 4).unbind(0)
    a = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, S, 768)
    torch.testing.assert_close(layer.attn(qkv).float(), a, atol=2e-2, rtol=2e-2)
    assert torch.isfinite(x.grad).all()


@pytest.mark.gpu
def test_qkv_bias_grad_from_attention_matches_colsum(gpu):
    """The attention backward also sums dQKV's columns (per-sequence partials + one column reduce)
    and hands them to the QKV Linear as its bias gradient: every gradient matches the path where the
    Linear sums them itself."""
    from parameter_server_distributed_amd.ops.attention import FusedSelfAttention
    from parameter_server_distributed_amd.ops.linear import MfmaLinear

    torch.manual_seed(4)
    B, S, H = 8, 128, 4
    lin = MfmaLinear(256, 3 * H * 64).to(gpu).to(torch.bfloat16)
    att = FusedSelfAttention(H, p=0.0).to(gpu)
    x0 = torch.randn(B, S, 256, device=gpu).to(torch.bfloat16)
    g = torch.randn(B, S, H * 64, device=gpu).to(torch.bfloat16)

    def run(hand):
        lin.weight.grad = lin.bias.grad = None
        x = x0.clone().requires_grad_(True)
        qkv = lin(x)
        if not hand:
            qkv = qkv * 1  # untagged: the Linear sums its own bias gradient
        att(qkv).backward(g)
        return [t.float().clone() for t in (x.grad, lin.weight.grad, lin.bias.grad)]

    got, ref = run(True), run(False)
    assert lin._psd_bias_hand is None
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=1e-2, atol=1e-2 * float(b.abs().max()) + 1e-6)


def _np_mix32(h):
    import numpy as np

    h = h.astype(np.uint64) & 0xFFFFFFFF
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h


@pytest.mark.gpu
def test_attention_dropout_mask_is_the_documented_hash(gpu):
    """The forward's keep-mask equals common.h drop_keep over idx = ((b*H + h)*S + q)*S + key with
    the attention key (attention.hip attn_key), element for element: pins the one-hash-per-pair
    form (akeep2) to the per-element definition."""
    import numpy as np

    from parameter_server_distributed_amd import native

    C = native()
    B, S, H, D, p, seed, stepv = 2, 64, 2, 64, 0.2, 11, 5
    step = torch.tensor([stepv], device=gpu, dtype=torch.int64)
    qkv = (torch.randn(B, S, 3, H, D, device=gpu) * 0.5).to(torch.bfloat16)
    qkv[:, :, 2] = torch.eye(S, D, device=gpu, dtype=torch.bfloat16)[None, :, None, :].expand(B, S, H, D)
    po, _ = C.attn_fwd(qkv.view(B, S, -1), H, p, seed, step)
    got = (po.view(B, S, H, D).permute(0, 2, 1, 3) != 0).cpu().numpy()  # [B, H, q, key]

    key = int(_np_mix32(np.array([((seed * 0x27D4EB2F) ^ (stepv * 0x165667B1)) & 0xFFFFFFFF]))[0])
    idx = np.arange(B * H * S * S, dtype=np.uint64)
    pr = idx >> 1
    h = _np_mix32(np.uint64(key) ^ ((pr & 0xFFFFFFFF) * 0x9E3779B9 & 0xFFFFFFFF)
                  ^ (((pr >> 32) * 0x7F4A7C15) & 0xFFFFFFFF))
    bits = np.where(idx & 1, h >> 16, h & 0xFFFF)
    thresh = min(4294967295, int(np.floor(p * 4294967296.0)))
    want = (bits >= (thresh >> 16)).reshape(B, H, S, S)
    assert (got == want).all(), int((got != want).sum())
