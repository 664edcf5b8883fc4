"""The recomputing bottleneck tail (ops/tail.py): conv3's output is never stored.

Kernel level (small-integer operands: every product and sum is exact in bf16 / fp32, so the checks
are exact against fp32 PyTorch): the narrow kernel's statistics-only pass, its BN-apply epilogue
(bwd mode 8: relu(bf16(y) * scale + shift + residual) + ReLU bit-mask), the bwd-data epilogue
without the BN input (modes 2 / 5 with bx None) and the rowdot kernel that supplies the missing
sum g y. Model level: ResNet-50 with the tail on vs off -- loss, every gradient, running stats."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from parameter_server_distributed_amd import native

pytestmark = pytest.mark.gpu


def _ints(shape, lo, hi, g):
    return torch.randint(lo, hi + 1, shape, generator=g).float()


@pytest.mark.parametrize("Nb,H,cin,cout", [(2, 14, 64, 256), (3, 7, 128, 512), (1, 9, 256, 1024)])
def test_convn_stats_only_and_apply_epilogue_exact(gpu, Nb, H, cin, cout):
    C = native()
    g = torch.Generator().manual_seed(3)
    x = _ints((Nb, cin, H, H), -1, 1, g)
    w = _ints((cout, cin), -1, 1, g)
    M = Nb * H * H
    y = (x.permute(0, 2, 3, 1).reshape(M, cin).double() @ w.double().t())  # exact
    sc = _ints((cout,), 1, 2, g)
    sh = _ints((cout,), -3, 3, g) + 0.5
    res = _ints((M, cout), -4, 4, g)
    o = torch.relu(y * sc.double() + sh.double() + res.double())
    want_out = o.float().bfloat16().float()
    want_bits = (o > 0).view(M * cout // 8, 8)
    xd = x.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wd = w.to(gpu, torch.bfloat16)
    shift = torch.zeros(cout, device=gpu)
    nv = 0
    for v in range(C.convn_variants(cout)):
        if C.convn_variant_kind(cout, v) not in (0, 3, 4) or not C.convn_variant_ok(cout, v, 1, 1, 1, 0, H):
            continue
        nv += 1
        rows_alloc = max(C.convn_stats_rows(M), C.convn_part_rows(M, cout, v, H, H, 1))
        part = torch.full((rows_alloc, 2, cout), float("nan"), device=gpu)
        rows = C.convn_(xd, wd, part, 1, 1, 1, 0, part=part, shift=shift, variant=v, no_store=True)
        assert rows > 0
        got = part[:rows].double().sum(0).cpu()
        torch.testing.assert_close(got[0], y.sum(0), rtol=0, atol=1e-3, msg=lambda m: f"v{v} sum: {m}")
        torch.testing.assert_close(got[1], (y * y).sum(0), rtol=1e-7, atol=1e-3, msg=lambda m: f"v{v} sumsq: {m}")
        out = torch.full((M, cout), 7.0, device=gpu, dtype=torch.bfloat16)
        mb = torch.zeros(M * cout // 8, device=gpu, dtype=torch.uint8)
        ss = torch.cat([sc, sh]).to(gpu)
        assert C.convn_(xd, wd, out, 1, 1, 1, 0, variant=v, apply_ss=ss, apply_res=res.to(gpu, torch.bfloat16),
                        apply_mask=mb) == 1
        torch.testing.assert_close(out.float().cpu(), want_out, rtol=0, atol=0, msg=lambda m: f"v{v} out: {m}")
        bits = ((mb.cpu()[:, None] >> torch.arange(8, dtype=torch.uint8)) & 1).bool()
        assert torch.equal(bits, want_bits), v
    assert nv >= 3  # two gathered + the persistent 1x1


@pytest.mark.parametrize("mode", [2, 5])
def test_convn_bwd_epilogue_without_bn_input(gpu, mode):
    """Modes 2 / 5 with bx None: g as with bx, the second partial is sum g (0 - mean)."""
    C = native()
    Nb, H, K, N = 2, 12, 64, 128
    g = torch.Generator().manual_seed(9)
    dy = _ints((Nb, K, H, H), -1, 1, g)
    w2 = _ints((N, K), -1, 1, g)
    M = Nb * H * H
    out_ref = dy.permute(0, 2, 3, 1).reshape(M, K).double() @ w2.double().t()
    mean = _ints((N,), -2, 2, g)
    bits = torch.randint(0, 2, (M, N), generator=g).bool()
    packed = (bits.view(M * N // 8, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)).sum(1).to(torch.uint8)
    if mode == 2:
        dr = _ints((M, N), -2, 2, g)
        add = dr.double()
        bdr = dr.to(gpu, torch.bfloat16)
    else:
        dr4 = _ints((Nb, N, H // 2, H // 2), -2, 2, g)
        full = torch.zeros(Nb, N, H, H)
        full[:, :, ::2, ::2] = dr4
        add = full.permute(0, 2, 3, 1).reshape(M, N).double()
        bdr = dr4.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gref = torch.where(bits, out_ref + add, torch.zeros_like(out_ref))
    s1 = gref.sum(0)
    dyd = dy.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    for v in range(C.convn_variants(N)):
        if C.convn_variant_kind(N, v) not in (0, 3, 4):
            continue
        out = torch.full((M, N), 7.0, device=gpu, dtype=torch.bfloat16)
        part = torch.full((max(C.convn_stats_rows(M), C.convn_part_rows(M, N, v, H, H, 1)), 2, N), float("nan"),
                          device=gpu)
        rows = C.convn_bwd_(dyd, w2.to(gpu, torch.bfloat16), out, 1, 1, 1, 0, part, v, mode, None, mean.to(gpu),
                            bdr=bdr, bmbits=packed.to(gpu))
        assert rows > 0
        torch.testing.assert_close(out.double().cpu(), gref, rtol=0, atol=0)
        got = part[:rows].double().cpu().sum(0)
        torch.testing.assert_close(got[0], s1, rtol=0, atol=1e-6)
        torch.testing.assert_close(got[1], -mean.double() * s1, rtol=0, atol=1e-6)


def test_bnfold_rowdot(gpu):
    C = native()
    g = torch.Generator().manual_seed(4)
    cout, cin = 256, 64
    P = torch.randn(cout + cin + 1, cin, generator=g)
    w = torch.randn(cout, cin, generator=g).bfloat16()
    row = torch.full((2, cout), float("nan"), device=gpu)
    C.bnfold_rowdot(P.to(gpu), w.to(gpu), row)
    want = (w.double() * P[:cout].double()).sum(1)
    assert torch.equal(row[0].cpu(), torch.zeros(cout))
    torch.testing.assert_close(row[1].double().cpu(), want, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("Nb,H,cin,cout", [(2, 14, 64, 256), (3, 7, 128, 512), (1, 9, 256, 1024)])
def test_bnfold_gram_stats_exact(gpu, Nb, H, cin, cout, variant):
    """Gram statistics: the Gram launch gives G = x^T x and s = 1^T x from one read of x; then per
    channel (sum y - M k, sum y^2 - 2 k sum y + M k^2) = shifted sums of y = x W^T, never formed."""
    C = native()
    assert C.convw_gram_rows(cin) > 0
    g = torch.Generator().manual_seed(5)
    x = _ints((Nb, cin, H, H), -1, 1, g)
    w = _ints((cout, cin), -1, 1, g)
    k = _ints((cout,), -2, 2, g)
    M = Nb * H * H
    y = x.permute(0, 2, 3, 1).reshape(M, cin).double() @ w.double().t()
    d = y - k.double()
    xd = x.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    P = torch.full((C.convw_gram_rows(cin), cin), float("nan"), device=gpu)
    assert C.convw_gram_(xd, P, variant=variant)
    xm = x.permute(0, 2, 3, 1).reshape(M, cin).double()
    torch.testing.assert_close(P[:cin].double().cpu(), xm.t() @ xm, rtol=0, atol=0)
    torch.testing.assert_close(P[cin].double().cpu(), xm.sum(0), rtol=0, atol=0)
    row = torch.full((2, cout), float("nan"), device=gpu)
    C.bnfold_gram_stats(P, w.to(gpu, torch.bfloat16), k.to(gpu), M, row)
    got = row.double().cpu()
    torch.testing.assert_close(got[0], d.sum(0), rtol=0, atol=0)
    torch.testing.assert_close(got[1], (d * d).sum(0), rtol=0, atol=0)


def test_resnet_tail_matches_unfused(gpu, monkeypatch):
    """ResNet-50 (64x64 images, batch 8, non-zero bn3 scales) with the recomputing tail on vs off,
    each against an fp32 run of the same weights (PyTorch composite ops): every parameter gradient
    and running statistic of the tail run must be as close to the fp32 reference as the unfused
    run's is (within 1.5x + 2 %), and the loss within the unfused run's distance from fp32 + 0.5 %.

    bn3 scales are drawn from [0.1, 0.3]: with [0.5, 1.5] this network is chaotic at batch 8 --
    the fp32 model's own loss moves by 4 % under relative 2^-9 (one bf16 ulp) noise on its input
    (tools/probes/tail_chaos_probe.py, profiles/r5/tail_chaos_probe.txt), so no bf16 path can be
    compared to fp32 there; at [0.1, 0.3] that spread is 0.05 %, unfused 0.02 % and the tail 0.06 %
    from fp32."""
    import copy
    import json

    from parameter_server_distributed_amd import models
    from parameter_server_distributed_amd.models.resnet import Bottleneck
    from parameter_server_distributed_amd.ops import autotune, tail

    torch.manual_seed(0)
    spec = models.build("resnet50", gpu, torch.bfloat16, image_size=64, num_classes=10)
    for mod in spec.model.modules():  # non-zero bn3 scales: the tail's gradients are then not trivially 0
        if isinstance(mod, Bottleneck):
            nn.init.uniform_(mod.bn3.weight, 0.1, 0.3)
    for p in spec.model.parameters():
        p.data = p.data.to(torch.bfloat16)
    init = copy.deepcopy(spec.model.state_dict())
    x, y = spec.make_batch(8, gpu, seed=3)

    def run(tail_on: bool, fp32: bool = False, keep=None):
        monkeypatch.setenv("PSD_FEATURES", f"tail_recompute={int(tail_on)}")
        autotune._DECISIONS.clear()
        autotune._DECISIONS.update(keep or {})
        for k in tail.TAIL_CALLS:
            tail.TAIL_CALLS[k] = 0
        m = spec.model
        m.load_state_dict(init)
        m.zero_grad(set_to_none=True)
        if fp32:
            m = copy.deepcopy(m).float()
        loss = spec.loss(m(x.float() if fp32 else x), y)
        loss.backward()
        return (float(loss), {n: p.grad.float().clone() for n, p in m.named_parameters()},
                {n: b.float().clone() for n, b in m.named_buffers() if "running" in n}, dict(tail.TAIL_CALLS))

    ref32 = run(False, fp32=True)
    autotune._DECISIONS.clear()
    off = run(False)
    # the tail run keeps every decision the unfused run made (the shared convolutions run the same
    # kernels; only the tail's own keys are timed): re-autotuned kernels alone moved the b8 loss by
    # ~2 % between bf16 runs (tools/probes/tail_stats_probe.py)
    keep = dict(autotune._DECISIONS)
    on = run(True, keep=keep)
    autotune._DECISIONS.clear()
    calls = on[3]
    # ResNet-50's identity blocks whose conv3 shape the fold takes (layer1-3: 10 of 12); each
    # backward either fused (the next conv1's epilogue) or recomputed (no fused consumer)
    assert calls["fwd"] >= 10, calls
    assert calls["bwd_fused"] + calls["bwd_recompute"] == calls["fwd"] and calls["bwd_fused"] >= 9, calls
    # layers 1-2 downsample blocks: the recomputing dual tail, its backward fused into the next conv1
    assert calls["dual_fwd"] == 2 and calls["dual_bwd_fused"] == 2, calls
    # the loss: within the unfused run's distance from the fp32 run + 0.5 % (the
    # per-layer statistics themselves are pinned against fp64 by test_tail_statistics_match_fp64)
    print("loss fp32 %.4f tail %.4f unfused %.4f" % (ref32[0], on[0], off[0]))
    assert abs(on[0] - ref32[0]) <= abs(off[0] - ref32[0]) + 0.005 * abs(ref32[0]), (on[0], off[0], ref32[0])

    def rel(a, b):
        return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()

    bad = {}
    for n, b in ref32[1].items():
        if b.norm() == 0:
            continue
        e_on, e_off = rel(on[1][n], b), rel(off[1][n], b)
        if e_on > 1.5 * e_off + 0.02:
            bad[n] = (round(e_on, 4), round(e_off, 4))
    for n, b in ref32[2].items():  # running statistics: the same rule against the fp32 run
        e_on, e_off = rel(on[2][n], b), rel(off[2][n], b)
        if e_on > 1.5 * e_off + 0.02:
            bad[n] = (round(e_on, 4), round(e_off, 4))
    assert not bad, json.dumps(bad)


def test_tail_recompute_fallback_matches_unfused(gpu, monkeypatch):
    """A tail whose output has no fused consumer (here: a weighted sum, as before the pooling):
    the backward recomputes y3 once and runs the ordinary BN backward + fold. Gradients of a2, W3,
    gamma, beta and the residual vs the unfused conv3 -> bn3 module pair."""
    from parameter_server_distributed_amd.ops import autotune, tail
    from parameter_server_distributed_amd.ops.bn import FusedBatchNorm2d
    from parameter_server_distributed_amd.ops.conv import Conv1x1

    torch.manual_seed(1)
    n, cin, cout, h = 4, 64, 256, 14
    conv = Conv1x1(cin, cout).to(gpu).to(memory_format=torch.channels_last)
    conv.weight.data = conv.weight.data.bfloat16()
    bn = FusedBatchNorm2d(cout, relu=True).to(gpu)
    nn.init.uniform_(bn.weight, 0.5, 1.5)
    nn.init.uniform_(bn.bias, -0.2, 0.2)
    bn.weight.data, bn.bias.data = bn.weight.data.bfloat16(), bn.bias.data.bfloat16()
    a2 = torch.randn(n, cin, h, h, device=gpu).relu().bfloat16().contiguous(memory_format=torch.channels_last)
    idt = torch.randn(n, cout, h, h, device=gpu).bfloat16().contiguous(memory_format=torch.channels_last)
    r = torch.randn(n, cout, h, h, device=gpu).bfloat16()
    res = []
    # fp32 composite reference of the same math (conv -> batch-norm (batch statistics) -> + idt -> relu)
    x32 = a2.float().requires_grad_(True)
    i32 = idt.float().requires_grad_(True)
    w32 = conv.weight.detach().float().requires_grad_(True)
    g32 = bn.weight.detach().float().requires_grad_(True)
    b32 = bn.bias.detach().float().requires_grad_(True)
    rm, rv = torch.zeros(cout, device=gpu), torch.ones(cout, device=gpu)
    y32 = torch.relu(F.batch_norm(F.conv2d(x32, w32), rm, rv, g32, b32, True, bn.momentum, bn.eps) + i32)
    (y32 * r.float()).sum().backward()
    ref = [y32.detach(), x32.grad, i32.grad, w32.grad, g32.grad, b32.grad, rm, rv]
    for on in (True, False):
        monkeypatch.setenv("PSD_FEATURES", f"tail_recompute={int(on)}")
        autotune._DECISIONS.clear()
        for k in tail.TAIL_CALLS:
            tail.TAIL_CALLS[k] = 0
        for p in (conv.weight, bn.weight, bn.bias):
            p.grad = None
        bn.running_mean.zero_()
        bn.running_var.fill_(1)
        x = a2.clone().requires_grad_(True)
        i = idt.clone().requires_grad_(True)
        if on:
            assert tail.tail_ok(conv, bn, x, i)
            y = tail.conv_bn_tail(conv, bn, x, i)
        else:
            y = bn(conv(x), i)
        (y.float() * r.float()).sum().backward()
        res.append([t.float().clone() for t in (y, x.grad, i.grad, conv.weight.grad, bn.weight.grad, bn.bias.grad,
                                                 bn.running_mean, bn.running_var)])
        if on:
            calls = {k: v for k, v in tail.TAIL_CALLS.items() if not k.startswith("dual")}
            assert calls == {"fwd": 1, "bwd_fused": 0, "bwd_recompute": 1}, tail.TAIL_CALLS
    autotune._DECISIONS.clear()
    names = ("y", "da2", "didt", "dW3", "dgamma", "dbeta", "running_mean", "running_var")
    for nm, a, b, f in zip(names, res[0], res[1], ref):
        e_on = ((a - f).norm() / f.norm().clamp_min(1e-6)).item()
        e_off = ((b - f).norm() / f.norm().clamp_min(1e-6)).item()
        # the tail normalises the fp32 product, the unfused path the bf16-rounded one: each within the
        # other's error level of the fp32 reference (a random upstream gradient makes near-cancelling
        # BN-backward sums, so single-block bf16 gradients sit a few % from fp32)
        assert e_on <= 1.5 * e_off + 1e-2, (nm, e_on, e_off)


def test_tail_statistics_match_fp64(gpu, monkeypatch):
    """the recomputing tail's BN statistics per identity block of ResNet-50
    (64x64, batch 8, the test above), both routes -- the Gram moments (sum y = W s, sum y^2 =
    W^T G W: convw_gram_ + bnfold_gram_stats) and the narrow kernel's statistics-only pass -- against
    the fp64 mean / biased variance of y = a2 W^T from the same bf16 operands. No cancellation: the
    Gram variance is within 1e-5 of fp64 where the inputs are post-ReLU (mean / std ~ 0.5)."""
    from parameter_server_distributed_amd import models, native
    from parameter_server_distributed_amd.models import resnet as R
    from parameter_server_distributed_amd.models.resnet import Bottleneck
    from parameter_server_distributed_amd.ops import autotune, tail

    C = native()
    torch.manual_seed(0)
    spec = models.build("resnet50", gpu, torch.bfloat16, image_size=64, num_classes=10)
    for mod in spec.model.modules():
        if isinstance(mod, Bottleneck):
            nn.init.uniform_(mod.bn3.weight, 0.5, 1.5)
    for p in spec.model.parameters():
        p.data = p.data.to(torch.bfloat16)
    x, y = spec.make_batch(8, gpu, seed=3)
    caps = []
    orig = R.conv_bn_tail

    def cap(conv, bn, a2, idt, resid_to=None):
        caps.append((a2.detach().clone(), conv.weight.detach().clone()))
        return orig(conv, bn, a2, idt, resid_to)

    monkeypatch.setenv("PSD_FEATURES", "tail_recompute=1")
    monkeypatch.setattr(R, "conv_bn_tail", cap)
    autotune._DECISIONS.clear()
    spec.loss(spec.model(x), y).backward()
    autotune._DECISIONS.clear()
    assert len(caps) >= 10
    for li, (a2, w) in enumerate(caps):
        n, cin, h, wd = a2.shape
        cout = w.shape[0]
        M = n * h * wd
        w2 = w.reshape(cout, cin).contiguous()
        y64 = a2.permute(0, 2, 3, 1).reshape(M, cin).double() @ w2.double().t()
        mu, var = y64.mean(0), y64.var(0, unbiased=False)
        shift = torch.zeros(cout, device=gpu)
        got = {}
        P = torch.empty(C.convw_gram_rows(cin), cin, device=gpu, dtype=torch.float32)
        assert C.convw_gram_(a2, P)
        row = torch.empty(2, cout, device=gpu, dtype=torch.float32)
        C.bnfold_gram_stats(P, w2, shift, M, row)
        got["gram"] = row.double()
        for v in range(C.convn_variants(cout)):
            if C.convn_variant_kind(cout, v) in (0, 3, 4) and C.convn_variant_ok(cout, v, 1, 1, 1, 0, wd):
                part = torch.empty(tail._part_rows(M, cout, v, h, wd, 1), 2, cout, device=gpu, dtype=torch.float32)
                rows = C.convn_(a2, w2, part, 1, 1, 1, 0, part=part, shift=shift, variant=v, no_store=True)
                assert rows > 0
                got[f"pass{v}"] = part[:rows].double().sum(0)
        assert len(got) >= 2
        for k, (s1, s2) in got.items():
            m_k = s1 / M
            v_k = s2 / M - m_k * m_k
            dm = float(((m_k - mu).abs() / var.sqrt()).max())
            dv = float(((v_k - var).abs() / var).max())
            assert dm < 1e-5 and dv < 1e-5, (li, k, dm, dv)


@pytest.mark.parametrize("stride,c3,cd,cout", [(1, 64, 64, 256), (2, 128, 256, 512)])
def test_dual_tail_fallback_matches_unfused_and_fp32(gpu, monkeypatch, stride, c3, cd, cout):
    """The recomputing dual tail relu(bn3(conv3(a2)) + bnd(convd(x))) of a downsample block with a
    stride-1 (layer 1) or stride-2 (layer 2: on the quarter grid) 1x1 downsample convolution
    (ops/tail.py _DualTailFn) whose output has no fused consumer (a weighted sum): forward output,
    running statistics and every gradient against an fp32 composite reference, within the unfused
    path's error level (the dual tail ratio-scales one branch's weights before its one bf16
    rounding; the unfused path rounds y3 / yd)."""
    from parameter_server_distributed_amd.ops import autotune, tail
    from parameter_server_distributed_amd.ops.bn import FusedBatchNorm2d, bn_add_bn_relu
    from parameter_server_distributed_amd.ops.conv import Conv1x1, ConvNHWC

    torch.manual_seed(5)
    n, h = 4, 14
    conv3 = Conv1x1(c3, cout).to(gpu).to(memory_format=torch.channels_last)
    convd = (Conv1x1(cd, cout) if stride == 1 else ConvNHWC(cd, cout, 1, 2)).to(gpu).to(
        memory_format=torch.channels_last)
    for cv in (conv3, convd):
        cv.weight.data = cv.weight.data.bfloat16()
    bn3 = FusedBatchNorm2d(cout, relu=True).to(gpu)
    bnd = FusedBatchNorm2d(cout).to(gpu)
    for bn in (bn3, bnd):
        nn.init.uniform_(bn.weight, 0.5, 1.5)
        nn.init.uniform_(bn.bias, -0.2, 0.2)
        bn.weight.data, bn.bias.data = bn.weight.data.bfloat16(), bn.bias.data.bfloat16()
    a2 = torch.randn(n, c3, h, h, device=gpu).relu().bfloat16().contiguous(memory_format=torch.channels_last)
    xin = torch.randn(n, cd, h * stride, h * stride, device=gpu).relu().bfloat16().contiguous(
        memory_format=torch.channels_last)
    r = torch.randn(n, cout, h, h, device=gpu).bfloat16()
    params = (conv3.weight, convd.weight, bn3.weight, bn3.bias, bnd.weight, bnd.bias)

    # fp32 composite reference
    t = [p.detach().float().requires_grad_(True) for p in params]
    a32, x32 = a2.float().requires_grad_(True), xin.float().requires_grad_(True)
    rms = [torch.zeros(cout, device=gpu), torch.ones(cout, device=gpu), torch.zeros(cout, device=gpu),
           torch.ones(cout, device=gpu)]
    y32 = torch.relu(F.batch_norm(F.conv2d(a32, t[0]), rms[0], rms[1], t[2], t[3], True, 0.1, bn3.eps)
                     + F.batch_norm(F.conv2d(x32, t[1], stride=stride), rms[2], rms[3], t[4], t[5], True, 0.1,
                                    bnd.eps))
    (y32 * r.float()).sum().backward()
    ref = [y32.detach(), a32.grad, x32.grad] + [p.grad for p in t] + rms

    res = []
    for on in (True, False):
        monkeypatch.setenv("PSD_FEATURES", f"dual_recompute={int(on)}")
        autotune._DECISIONS.clear()
        for k in tail.TAIL_CALLS:
            tail.TAIL_CALLS[k] = 0
        for p in params:
            p.grad = None
        for bn in (bn3, bnd):
            bn.running_mean.zero_()
            bn.running_var.fill_(1)
        a = a2.clone().requires_grad_(True)
        x = xin.clone().requires_grad_(True)
        if on:
            assert tail.dual_tail_ok(conv3, bn3, a, convd, bnd, x)
            y = tail.conv_bn_dual_tail(conv3, bn3, a, convd, bnd, x)
        else:
            y = bn_add_bn_relu(bn3, conv3(a), bnd, convd(x))
        (y.float() * r.float()).sum().backward()
        res.append([y.float(), a.grad.float(), x.grad.float()] + [p.grad.float() for p in params]
                   + [bn3.running_mean.clone(), bn3.running_var.clone(), bnd.running_mean.clone(),
                      bnd.running_var.clone()])
        if on:
            assert tail.TAIL_CALLS["dual_fwd"] == 1 and tail.TAIL_CALLS["dual_bwd_recompute"] == 1, tail.TAIL_CALLS
    autotune._DECISIONS.clear()
    names = ("y", "da2", "dx", "dW3", "dWd", "dg3", "db3", "dgd", "dbd", "rm3", "rv3", "rmd", "rvd")
    for nm, a, b, f in zip(names, res[0], res[1], ref):
        e_on = ((a - f.float()).norm() / f.float().norm().clamp_min(1e-6)).item()
        e_off = ((b - f.float()).norm() / f.float().norm().clamp_min(1e-6)).item()
        assert e_on <= 1.5 * e_off + 1e-2, (nm, e_on, e_off)


@pytest.mark.parametrize("shape", [(2, 256, 56, 56), (3, 64, 14, 10)])
def test_subsample2_exact(gpu, shape):
    """kernels/pool.hip subsample2: the quarter-grid input of a stride-2 1x1 downsample, bitwise."""
    x = torch.randn(*shape, device=gpu).bfloat16().contiguous(memory_format=torch.channels_last)
    y = native().subsample2(x)
    assert y.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(y, x[:, :, ::2, ::2])


@pytest.mark.parametrize("cout,c3,cd", [(256, 64, 64), (512, 128, 256)])
def test_dual_weights_kernel_matches_torch(gpu, cout, c3, cd):
    """kernels/bnfold.hip bnfold_dual_weights (the dual tail's apply operands, one launch) == the
    torch-op formula ops/tail.dual_weights_reference, bitwise: ratio-scaled weights of the smaller-
    scale branch, s_big and the summed shift -- incl. ties, zero scales (zero-init gamma) and signs."""
    from parameter_server_distributed_amd.ops.tail import dual_weights_reference

    torch.manual_seed(0)
    w3 = torch.randn(cout, c3, device=gpu).bfloat16()
    wd = torch.randn(cout, cd, device=gpu).bfloat16()
    ss3 = torch.randn(2 * cout, device=gpu)
    ssd = torch.randn(2 * cout, device=gpu)
    ss3[:8] = 0.0  # s3 = 0 (zero-init bn3 gamma)
    ssd[4:12] = 0.0  # both zero on 4..7, sd = 0 on 8..11
    ssd[16:24] = ss3[16:24]  # ties
    ssd[24:32] = -ss3[24:32]  # |ties| with opposite signs
    wcat, ss = native().bnfold_dual_weights(w3, wd, ss3, ssd)
    wref, sref = dual_weights_reference(w3, wd, ss3, ssd)
    assert torch.equal(wcat, wref)
    assert torch.equal(ss, sref)
