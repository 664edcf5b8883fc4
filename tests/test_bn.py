"""Fused NHWC BatchNorm(+residual)(+ReLU) gfx950 kernels vs a plain PyTorch fp32 reference."""
import pytest
import torch
import torch.nn.functional as F

from parameter_server_distributed_amd.ops.bn import FusedBatchNorm2d

SHAPES = [(4, 64, 8, 8), (2, 256, 7, 7), (2, 2048, 3, 3), (3, 24, 5, 5), (8, 128, 14, 14)]


def _ref(x, w, b, rm, rv, res, relu, momentum=0.1, eps=1e-5):
    y = F.batch_norm(x, rm, rv, w, b, True, momentum, eps)
    if res is not None:
        y = y + res
    return F.relu(y) if relu else y


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("residual", [False, True])
def test_fused_bn_train_fwd_bwd(gpu, shape, relu, residual):
    torch.manual_seed(0)
    N, C, H, W = shape
    x = (torch.randn(shape) * 2 + 0.5).to(torch.bfloat16)
    r = torch.randn(shape).to(torch.bfloat16) if residual else None
    gy = torch.randn(shape).to(torch.bfloat16)
    m = FusedBatchNorm2d(C, relu=relu).to(gpu)
    with torch.no_grad():
        m.weight.copy_(torch.rand(C) + 0.5)
        m.bias.copy_(torch.randn(C) * 0.1)
        m.running_mean.copy_(torch.randn(C) * 0.1)
        m.running_var.copy_(torch.rand(C) + 0.5)
    m.weight.data = m.weight.data.to(torch.bfloat16)
    m.bias.data = m.bias.data.to(torch.bfloat16)
    rm0, rv0 = m.running_mean.cpu().clone(), m.running_var.cpu().clone()

    xd = x.to(gpu).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    rd = r.to(gpu).contiguous(memory_format=torch.channels_last).requires_grad_(True) if residual else None
    y = m(xd, rd)
    y.backward(gy.to(gpu).contiguous(memory_format=torch.channels_last))

    # fp32 reference on the same bf16-rounded inputs
    xr = x.float().requires_grad_(True)
    rr = r.float().requires_grad_(True) if residual else None
    wr = m.weight.detach().float().cpu().requires_grad_(True)
    br = m.bias.detach().float().cpu().requires_grad_(True)
    rm, rv = rm0.clone(), rv0.clone()
    yr = _ref(xr, wr, br, rm, rv, rr, relu)
    yr.backward(gy.float())

    torch.testing.assert_close(y.float().cpu(), yr.detach(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(m.running_mean.cpu(), rm, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(m.running_var.cpu(), rv, rtol=1e-3, atol=1e-3)
    assert int(m.num_batches_tracked.item()) == 1
    # gradients: bf16 outputs, relative to the gradient scale
    sc = xr.grad.abs().max().item() + 1e-6
    torch.testing.assert_close(xd.grad.float().cpu() / sc, xr.grad / sc, rtol=0, atol=2e-2)
    torch.testing.assert_close(m.weight.grad.float().cpu(), wr.grad, rtol=2e-2, atol=2e-2 * wr.grad.abs().max().item())
    torch.testing.assert_close(m.bias.grad.float().cpu(), br.grad, rtol=2e-2, atol=2e-2 * br.grad.abs().max().item())
    if residual:
        torch.testing.assert_close(rd.grad.float().cpu(), rr.grad, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_fused_bn_eval_matches_reference(gpu):
    torch.manual_seed(1)
    m = FusedBatchNorm2d(64, relu=True).to(gpu)
    m.running_mean.normal_()
    m.running_var.uniform_(0.5, 2.0)
    m.weight.data = (torch.rand(64, device=gpu) + 0.5).to(torch.bfloat16)
    m.bias.data = torch.randn(64, device=gpu).to(torch.bfloat16)
    m.eval()
    x = torch.randn(2, 64, 9, 9, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y = m(x)
        yr = m._reference(x)
    torch.testing.assert_close(y.float(), yr.float(), rtol=2e-2, atol=2e-2)


def test_fused_bn_cpu_reference_path():
    m = FusedBatchNorm2d(16, relu=True)
    x = torch.randn(2, 16, 4, 4)
    r = torch.randn(2, 16, 4, 4)
    y = m(x, r)
    ref = F.relu(F.batch_norm(x, None, None, None, None, True) + r)
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 64, 112, 112), (3, 16, 9, 7), (1, 8, 2, 2)], ids=str)
def test_maxpool3s2_matches_torch(gpu, shape):
    from parameter_server_distributed_amd.ops.pool import max_pool_3x3s2

    torch.manual_seed(0)
    x = torch.randn(shape).to(torch.bfloat16)
    xd = x.to(gpu).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = max_pool_3x3s2(xd)
    g = torch.randn(y.shape).to(torch.bfloat16)
    y.backward(g.to(gpu).contiguous(memory_format=torch.channels_last))
    xr = x.float().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    yr.backward(g.float())
    torch.testing.assert_close(y.float().cpu(), yr.detach(), rtol=0, atol=0)
    torch.testing.assert_close(xd.grad.float().cpu(), xr.grad, rtol=1e-2, atol=1e-2)


@pytest.mark.gpu
def test_resnet_residual_grad_fusion_matches_unfused(gpu, monkeypatch):
    """Identity-block residual gradients handed BN-to-BN inside the kernels == autograd's add.
    (Stored-output tails in both runs: the recomputing tails change the forward rounding -- pinned
    against fp32 in tests/test_tail.py -- and at batch 4 / 64x64, 16 samples per layer-4 BN channel,
    a forward perturbation of one bf16 ulp moves the stem's gradient by ~10 %.)"""
    from parameter_server_distributed_amd import models

    monkeypatch.setenv("PSD_FEATURES", "tail_recompute=0")
    torch.manual_seed(0)
    grads = []
    for fuse in (True, False):
        torch.manual_seed(0)
        spec = models.build("resnet50", gpu, torch.bfloat16, image_size=64, num_classes=10)
        m = spec.model
        for p in m.parameters():
            p.data = p.data.to(torch.bfloat16)
        for mod in m.modules():
            if hasattr(mod, "fuse_residual_grad"):
                mod.fuse_residual_grad = fuse
        x, y = spec.make_batch(4, gpu, seed=3)
        spec.loss(m(x), y).backward()
        grads.append({n: p.grad.float().clone() for n, p in m.named_parameters()})
    # relative-norm check: a wrong hand-over would be off by O(1); bf16 rounding differences (fp32
    # sums inside the kernels vs bf16 autograd adds) and the run-to-run noise of library GEMMs,
    # amplified through ReLU masks and bf16 ties in the stem pool, stay at a few percent
    for n in grads[0]:
        a, b = grads[0][n], grads[1][n]
        if b.norm() == 0:
            assert a.norm() == 0, n
            continue
        assert ((a - b).norm() / b.norm()).item() < 0.1, n


@pytest.mark.gpu
def test_maxpool3s2_second_gradient_is_summed(gpu):
    """dy2 (the first bottleneck's downsample-branch gradient) is added inside the gather kernel."""
    from parameter_server_distributed_amd import native

    torch.manual_seed(0)
    x = torch.randn(2, 16, 12, 10).to(torch.bfloat16).to(gpu).contiguous(memory_format=torch.channels_last)
    y, arg = native().maxpool3s2_fwd(x)
    g1 = torch.randn(y.shape).to(torch.bfloat16).to(gpu).contiguous(memory_format=torch.channels_last)
    g2 = torch.randn(y.shape).to(torch.bfloat16).to(gpu).contiguous(memory_format=torch.channels_last)
    both = native().maxpool3s2_bwd(g1, arg, 12, 10, g2)
    xr = x.float().cpu().requires_grad_(True)
    F.max_pool2d(xr, 3, 2, 1).backward(g1.float().cpu() + g2.float().cpu())
    torch.testing.assert_close(both.float().cpu(), xr.grad, rtol=1e-2, atol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(4, 2048, 7, 7), (3, 64, 5, 3), (2, 8, 1, 1)], ids=str)
def test_global_avg_pool_matches_torch(gpu, shape):
    from parameter_server_distributed_amd.ops.pool import global_avg_pool

    torch.manual_seed(0)
    x = torch.randn(shape).to(torch.bfloat16)
    xd = x.to(gpu).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = global_avg_pool(xd)
    assert y.shape == (shape[0], shape[1])
    g = torch.randn(y.shape).to(torch.bfloat16)
    y.backward(g.to(gpu))
    xr = x.float().requires_grad_(True)
    yr = torch.flatten(F.adaptive_avg_pool2d(xr, 1), 1)
    yr.backward(g.float())
    torch.testing.assert_close(y.float().cpu(), yr.detach(), rtol=1e-2, atol=1e-2)
    assert xd.grad.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(xd.grad.float().cpu(), xr.grad, rtol=1e-2, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("route", ["gemm", "miopen"])
def test_conv1x1_routes_match_fp32(gpu, route):
    """Both routes of the 1x1 conv (hipBLASLt GEMM / MIOpen) against an fp32 conv, fwd + both grads."""
    from parameter_server_distributed_amd.ops import conv as cv

    torch.manual_seed(0)
    m = cv.Conv1x1(64, 96).to(gpu).to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(3, 64, 10, 12).to(torch.bfloat16).to(gpu).contiguous(memory_format=torch.channels_last)
    xd = x.clone().requires_grad_(True)
    M = 3 * 10 * 12
    for kind in ("fwd", "dgrad"):
        cv.set_decision((kind, M, 64, 96), route)
    try:
        y = m(xd)
        g = torch.randn(y.shape).to(torch.bfloat16).to(gpu).contiguous(memory_format=torch.channels_last)
        y.backward(g)
    finally:
        for kind in ("fwd", "dgrad"):
            cv.set_decision((kind, M, 64, 96), None)
    xr = x.float().cpu().requires_grad_(True)
    wr = m.weight.detach().float().cpu().requires_grad_(True)
    yr = F.conv2d(xr, wr)
    yr.backward(g.float().cpu())
    assert y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float().cpu(), yr.detach(), rtol=2e-2, atol=5e-2)
    torch.testing.assert_close(xd.grad.float().cpu(), xr.grad, rtol=2e-2, atol=5e-2)
    torch.testing.assert_close(m.weight.grad.float().cpu(), wr.grad, rtol=2e-2, atol=2e-1)


@pytest.mark.gpu
def test_conv1x1_autotune_records_a_choice(gpu):
    from parameter_server_distributed_amd.ops import conv as cv

    m = cv.Conv1x1(32, 64).to(gpu).to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(2, 32, 8, 8, device=gpu, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    m(x.requires_grad_(True)).sum().backward()
    d = cv.decisions()
    assert d[("fwd", 128, 32, 64)] in ("gemm", "miopen", "psd") and d[("dgrad", 128, 32, 64)] in ("gemm", "miopen", "psd")


@pytest.mark.gpu
@pytest.mark.parametrize("shape,second", [((4, 64, 16, 12), False), ((2, 64, 112, 112), True), ((3, 16, 6, 10), True),
                                          ((1, 256, 8, 40), True)],
                         ids=str)
def test_stem_bn_relu_maxpool_fused_matches_composite(gpu, shape, second):
    """Fused stem (BN + ReLU + max-pool, pool gradient recomputed inside the BN backward) against
    the unfused gfx950 kernels (BN kernel, then pool kernel: same bf16 ties in the pool windows)
    for the output, running stats and every gradient, and the forward against fp32."""
    from parameter_server_distributed_amd.ops.bn import FusedBatchNorm2d, bn_relu_maxpool
    from parameter_server_distributed_amd.ops.pool import MaxPool3x3s2

    torch.manual_seed(0)
    C = shape[1]
    x = (torch.randn(shape) * 2 + 0.3).to(torch.bfloat16)
    g = torch.randn((shape[0], C, shape[2] // 2, shape[3] // 2)).to(torch.bfloat16)
    g2 = torch.randn(g.shape).to(torch.bfloat16) if second else None
    cl = dict(memory_format=torch.channels_last)
    res = []
    for fused in (True, False):
        torch.manual_seed(1)
        bn = FusedBatchNorm2d(C, relu=True).to(gpu)
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.5, 0.5)
        bn.weight.data = bn.weight.data.to(torch.bfloat16)
        bn.bias.data = bn.bias.data.to(torch.bfloat16)
        pool = MaxPool3x3s2()
        xd = x.to(gpu).contiguous(**cl).requires_grad_(True)
        if fused:
            y = bn_relu_maxpool(bn, pool, xd)
            if second:
                pool._psd_pending_dr.append(g2.to(gpu).contiguous(**cl))
            y.backward(g.to(gpu).contiguous(**cl))
            assert not pool._psd_pending_dr
        else:
            y = pool(bn(xd))
            y.backward((g + g2 if second else g).to(gpu).contiguous(**cl))
        res.append((y.float().cpu(), xd.grad.float().cpu(), bn.weight.grad.float().cpu(), bn.bias.grad.float().cpu(),
                    bn.running_mean.cpu(), bn.running_var.cpu(), bn.weight.detach().float().cpu(),
                    bn.bias.detach().float().cpu()))
    (y, dx, dw, db, rm, rv, w, b), (y0, dx0, dw0, db0, rm0, rv0, _, _) = res
    torch.testing.assert_close(y, y0, rtol=0, atol=0)
    torch.testing.assert_close(rm, rm0, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(rv, rv0, rtol=1e-6, atol=1e-6)
    # unfused rounds the pool gradient (and g + g2) to bf16 before the BN backward; fused keeps fp32
    torch.testing.assert_close(dx, dx0, rtol=2e-2, atol=2e-2 * dx0.abs().max().item())
    torch.testing.assert_close(dw, dw0, rtol=2e-2, atol=2e-2 * dw0.abs().max().item())
    torch.testing.assert_close(db, db0, rtol=2e-2, atol=2e-2 * db0.abs().max().item())
    yr = F.max_pool2d(F.relu(F.batch_norm(x.float(), None, None, w, b, True, 0.1, 1e-5)), 3, 2, 1)
    torch.testing.assert_close(y, yr, rtol=2e-2, atol=3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 3, 64, 64), (3, 3, 224, 224), (1, 3, 32, 96)], ids=str)
def test_stem_conv_fused_matches_unfused(gpu, shape):
    """gfx950 stem: (1) the implicit-GEMM conv output against an fp32 conv; (2) end to end against
    the stand-alone BN + pool kernels and MIOpen's weight gradient applied to the SAME conv output
    (so both sides see identical bf16 ties in the pool windows): output, running stats, gradients."""
    import torch.nn as nn

    from parameter_server_distributed_amd import native
    from parameter_server_distributed_amd.ops import conv as cv
    from parameter_server_distributed_amd.ops.bn import FusedBatchNorm2d
    from parameter_server_distributed_amd.ops.pool import MaxPool3x3s2

    torch.manual_seed(0)
    cl = dict(memory_format=torch.channels_last)
    x = torch.randn(shape).to(torch.bfloat16).to(gpu).contiguous(**cl)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(gpu).to(torch.bfloat16).to(**cl)
    w = conv.weight.detach()

    def make_bn():
        torch.manual_seed(1)
        bn = FusedBatchNorm2d(64, relu=True).to(gpu)
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.5, 0.5)
        bn.weight.data = bn.weight.data.to(torch.bfloat16)
        bn.bias.data = bn.bias.data.to(torch.bfloat16)
        return bn

    # (1) conv output
    bn = make_bn()
    conv_out = native().stem_fwd(x, w, bn.weight, bn.bias, bn.running_mean.clone(), bn.running_var.clone(), 0.1,
                                 1e-5)[5]
    ref = F.conv2d(x.float(), w.float(), stride=2, padding=3)
    torch.testing.assert_close(conv_out.float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())

    # (2) end to end
    bn, pool = make_bn(), MaxPool3x3s2()
    y = cv.stem_forward(conv, bn, pool, x)
    assert pool.native_last
    torch.manual_seed(2)
    g = torch.randn(y.shape, device=gpu).to(torch.bfloat16).contiguous(**cl)
    y.backward(g)
    bn0, pool0 = make_bn(), MaxPool3x3s2()
    c0 = conv_out.detach().clone().requires_grad_(True)
    y0 = pool0(bn0(c0))
    y0.backward(g)
    dw0 = torch.ops.aten.convolution_backward(c0.grad, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                              [False, True, False])[1]
    torch.testing.assert_close(y.float(), y0.float(), rtol=0, atol=0)
    torch.testing.assert_close(bn.running_mean, bn0.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn.running_var, bn0.running_var, rtol=1e-4, atol=1e-5)
    # the unfused side rounds the pool gradient to bf16 before the BN backward; the fused keeps fp32
    for a, b in ((conv.weight.grad, dw0), (bn.weight.grad, bn0.weight.grad), (bn.bias.grad, bn0.bias.grad)):
        a, b = a.float(), b.float()
        assert ((a - b).norm() / b.norm()).item() < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 3, 64, 64), (4, 3, 224, 224), (3, 3, 32, 96)], ids=str)
def test_stem_wgrad_matches_fp32(gpu, shape):
    """gfx950 stem weight gradient (MFMA reduction over all output pixels) against an fp32 conv."""
    from parameter_server_distributed_amd import native

    torch.manual_seed(0)
    cl = dict(memory_format=torch.channels_last)
    x = torch.randn(shape).to(torch.bfloat16)
    dy = torch.randn(shape[0], 64, shape[2] // 2, shape[3] // 2).to(torch.bfloat16)
    dw = native().stem_wgrad(x.to(gpu).contiguous(**cl), dy.to(gpu).contiguous(**cl))
    assert dw.shape == (64, 3, 7, 7) and dw.is_contiguous(memory_format=torch.channels_last)
    w = torch.zeros(64, 3, 7, 7, requires_grad=True)
    torch.nn.functional.conv2d(x.float(), w, stride=2, padding=3).backward(dy.float())
    ref = w.grad
    torch.testing.assert_close(dw.float().cpu(), ref, rtol=2e-2, atol=1e-2 * ref.abs().max().item())


@pytest.mark.gpu
def test_downsample_bn_applied_inside_bn3_matches_unfused(gpu):
    """Bottleneck with a stride-2 downsample branch: relu(bn3(conv3) + bn_ds(conv_ds)) on the fused
    path (the recomputing dual tail of ops/tail.py, or bn_add_bn_relu with the downsample BN inside
    bn3's apply pass) vs the unfused modules, both against an fp32 composite run of the same block:
    output, every gradient and both BNs' running statistics at the unfused path's bf16 error level
    (two bf16 paths that round in different places differ by a few % on near-cancelling BN
    gradient sums, so they are compared through fp32, not with each other)."""
    import copy

    import torch.nn as nn

    from parameter_server_distributed_amd.models.resnet import Bottleneck, _conv
    from parameter_server_distributed_amd.ops.bn import FusedBatchNorm2d

    torch.manual_seed(0)
    down = nn.Sequential(_conv(64, 256, 1, 2), FusedBatchNorm2d(256))
    blk = Bottleneck(64, 64, 2, 64, down).to(gpu).to(torch.bfloat16).to(memory_format=torch.channels_last)
    for m in blk.modules():
        if isinstance(m, FusedBatchNorm2d):
            m.running_mean.data = m.running_mean.data.float()
            m.running_var.data = m.running_var.data.float()
            with torch.no_grad():
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    ref = copy.deepcopy(blk)
    ref.fuse_residual_grad = False
    ref32 = copy.deepcopy(blk).float()
    x0 = torch.randn(8, 64, 28, 28, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    for m in (blk, ref, ref32):
        x = (x0.float() if m is ref32 else x0).clone().requires_grad_(True)
        y = m(x)
        y.float().pow(2).mean().backward()
        outs.append({"y": y.float(), "dx": x.grad.float(), **{n: p.grad.float() for n, p in m.named_parameters()},
                     **{n: b.float() for n, b in m.named_buffers() if b.is_floating_point()}})
    f, u, r = outs
    for n in r:
        e_f = ((f[n] - r[n]).norm() / r[n].norm().clamp_min(1e-6)).item()
        e_u = ((u[n] - r[n]).norm() / r[n].norm().clamp_min(1e-6)).item()
        assert e_f <= 1.5 * e_u + 1e-2, (n, e_f, e_u)

@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(64, 128, 128, 128), (64, 24, 256, 256)], ids=lambda s: "x".join(map(str, s)))
def test_fused_bn_streaming_launch_on_large_tensors(gpu, shape):
    """Tensors above 128 MB take the streaming (nontemporal) one-shot elementwise launch (C/8 | 256)
    or the streaming grid-stride one (C = 24): forward with residual + ReLU (bit-mask), backward,
    and the coefficient-only elementwise pass, against fp32 on the GPU."""
    from parameter_server_distributed_amd import native

    torch.manual_seed(0)
    N, C, H, W = shape
    x = (torch.randn(shape, device=gpu) * 2 + 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    r = torch.randn(shape, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(shape, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert x.numel() * 2 > 128 << 20
    m = FusedBatchNorm2d(C, relu=True).to(gpu)
    with torch.no_grad():
        m.weight.copy_(torch.rand(C) + 0.5)
        m.bias.copy_(torch.randn(C) * 0.1)
    m.weight.data = m.weight.data.to(torch.bfloat16)
    m.bias.data = m.bias.data.to(torch.bfloat16)
    xd, rd = x.clone().requires_grad_(True), r.clone().requires_grad_(True)
    y = m(xd, rd)
    y.backward(gy)

    xr, rr = x.float().requires_grad_(True), r.float().requires_grad_(True)
    wr = m.weight.detach().float().requires_grad_(True)
    br = m.bias.detach().float().requires_grad_(True)
    yr = F.relu(F.batch_norm(xr, None, None, wr, br, True, 0.1, 1e-5) + rr)
    yr.backward(gy.float())
    for name, a, b in (("y", y, yr), ("dx", xd.grad, xr.grad), ("dres", rd.grad, rr.grad)):
        rel = ((a.float() - b).norm() / b.norm()).item()
        assert rel < 1e-2, (name, rel)
    del y, yr, xd, rd, xr, rr

    g2 = gy.reshape(-1, C) if gy.is_contiguous() else gy.permute(0, 2, 3, 1).reshape(-1, C)
    x2 = x.permute(0, 2, 3, 1).reshape(-1, C)
    coef = torch.randn(3 * C, device=gpu)
    got = native().bn_elemt_coef(g2, x2, coef)
    want = coef[:C] * g2.float() + coef[C:2 * C] * x2.float() + coef[2 * C:]
    rel = ((got.float() - want).norm() / want.norm()).item()
    assert rel < 5e-3, rel
