"""Fused LayerNorm(x + dropout(h)) (kernels/layernorm.hip) against an fp32 composite with the same
dropout mask: forward, the residual and branch gradients, gamma/beta gradients; mask statistics and
per-step mask refresh through the device counter."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _mask(C, shape, p, seed, step, gpu):
    """The kernel's keep-mask for (seed, step): s = 0 + dropout(1) = mask / (1 - p)."""
    z = torch.zeros(shape, device=gpu, dtype=torch.bfloat16)
    one = torch.ones(shape, device=gpu, dtype=torch.bfloat16)
    H = shape[-1]
    g = torch.ones(H, device=gpu, dtype=torch.bfloat16)
    b = torch.zeros(H, device=gpu, dtype=torch.bfloat16)
    s = C.ln_fwd(z, one, g, b, 1e-12, p, seed, step)[1]
    return (s != 0).float()


@pytest.mark.parametrize("H,p", [(768, 0.0), (768, 0.1), (1024, 0.25)])
def test_fused_add_layernorm_matches_fp32(gpu, H, p):
    from parameter_server_distributed_amd import native
    from parameter_server_distributed_amd.ops.layernorm import FusedAddLayerNorm

    C = native()
    torch.manual_seed(0)
    shape = (4, 37, H)
    ln = FusedAddLayerNorm(H, eps=1e-12, p=p, seed=7).to(gpu)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.5, 0.5)
    ln.weight.data = ln.weight.data.to(torch.bfloat16)
    ln.bias.data = ln.bias.data.to(torch.bfloat16)
    step = torch.tensor([3], device=gpu, dtype=torch.int64)
    ln.step = step
    x = torch.randn(shape, device=gpu).to(torch.bfloat16).requires_grad_(True)
    h = torch.randn(shape, device=gpu).to(torch.bfloat16).requires_grad_(True)
    y = ln(x, h)
    g = torch.randn(shape, device=gpu).to(torch.bfloat16)
    y.backward(g)

    mask = _mask(C, shape, p, 7, step, gpu) if p > 0 else torch.ones(shape, device=gpu)
    if p > 0:
        keep = mask.mean().item()
        assert abs(keep - (1 - p)) < 0.02, keep
    xr = x.detach().float().requires_grad_(True)
    hr = h.detach().float().requires_grad_(True)
    wr = ln.weight.detach().float().requires_grad_(True)
    br = ln.bias.detach().float().requires_grad_(True)
    s = (xr + hr * mask / (1 - p)).to(torch.bfloat16).float()  # the kernel normalises the bf16 sum
    yr = F.layer_norm(s, (H,), wr, br, 1e-12)
    yr.backward(g.float())
    for a, b in ((y, yr), (x.grad, xr.grad), (h.grad, hr.grad), (ln.weight.grad, wr.grad), (ln.bias.grad, br.grad)):
        rel = ((a.float() - b).norm() / b.norm()).item()
        assert rel < 2e-2, rel


def test_dropout_mask_changes_with_device_step(gpu):
    from parameter_server_distributed_amd import native

    C = native()
    shape = (64, 768)
    s1 = torch.tensor([1], device=gpu, dtype=torch.int64)
    s2 = torch.tensor([2], device=gpu, dtype=torch.int64)
    m1 = _mask(C, shape, 0.1, 5, s1, gpu)
    m1b = _mask(C, shape, 0.1, 5, s1, gpu)
    m2 = _mask(C, shape, 0.1, 5, s2, gpu)
    m3 = _mask(C, shape, 0.1, 6, s1, gpu)
    assert torch.equal(m1, m1b)  # regenerable (backward reuses it)
    assert not torch.equal(m1, m2) and not torch.equal(m1, m3)


def test_residual_grad_handoff_matches_autograd_add(gpu, monkeypatch):
    """BertLayer with each residual LayerNorm handing x's gradient to the Linear that also reads x
    (accumulated by its bwd-data GEMM) vs the same layer with autograd adding the two gradients."""
    from parameter_server_distributed_amd.models.bert import BertLayer
    from parameter_server_distributed_amd.ops import layernorm as lnmod

    torch.manual_seed(1)
    layer = BertLayer(768, 12, 3072, dropout=0.0).to(gpu).to(torch.bfloat16)
    step = torch.tensor([1], device=gpu, dtype=torch.int64)
    for m in layer.modules():
        if hasattr(m, "step"):
            m.step = step
    x0 = torch.randn(4, 128, 768, device=gpu).to(torch.bfloat16)

    def run():
        layer.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        y = layer(x)
        y.float().pow(2).mean().backward()
        return x.grad.float(), {n: p.grad.float().clone() for n, p in layer.named_parameters()}

    gx, gp = run()
    assert not layer.qkv._psd_pending_dx and not layer.ffn1._psd_pending_dx
    orig = lnmod.FusedAddLayerNorm.forward
    monkeypatch.setattr(lnmod.FusedAddLayerNorm, "forward", lambda self, x, h, x_grad_to=None: orig(self, x, h))
    rx, rp = run()
    torch.testing.assert_close(gx, rx, rtol=2e-2, atol=2e-2 * float(rx.abs().max()))
    for n in rp:
        torch.testing.assert_close(gp[n], rp[n], rtol=2e-2, atol=2e-2 * float(rp[n].abs().max()) + 1e-6, msg=n)


@pytest.mark.gpu
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_branch_bias_grad_from_layernorm_matches_colsum(gpu, monkeypatch, p):
    """The residual LayerNorm's backward sums dh's columns (the branch Linear's bias gradient) and
    hands them to that Linear, which skips its column-sum kernels: every gradient matches the path
    without the hand-over (h detached from its producer's tag), and bias.grad matches dh's colsum."""
    from parameter_server_distributed_amd.ops.layernorm import FusedAddLayerNorm
    from parameter_server_distributed_amd.ops.linear import MfmaLinear

    torch.manual_seed(3)
    lin = MfmaLinear(3072, 768).to(gpu).to(torch.bfloat16)
    ln = FusedAddLayerNorm(768, p=p, seed=5).to(gpu).to(torch.bfloat16)
    ln.step = torch.tensor([2], device=gpu, dtype=torch.int64)
    x0 = torch.randn(2048, 768, device=gpu).to(torch.bfloat16)
    a0 = torch.randn(2048, 3072, device=gpu).to(torch.bfloat16)
    gy = torch.randn(2048, 768, device=gpu).to(torch.bfloat16)

    def run(hand):
        for t in (lin.weight, lin.bias, ln.weight, ln.bias):
            t.grad = None
        x, a = x0.clone().requires_grad_(True), a0.clone().requires_grad_(True)
        h = lin(a)
        if not hand:
            h = h * 1  # a fresh tensor without the producer tag
        ln(x, h).backward(gy)
        return [t.grad.float().clone() for t in (x, a, lin.weight, lin.bias, ln.weight, ln.bias)]

    got, ref = run(True), run(False)
    assert lin._psd_bias_hand is None  # consumed
    for g, r in zip(got, ref):
        torch.testing.assert_close(g, r, rtol=1e-2, atol=1e-2 * float(r.abs().max()) + 1e-6)
