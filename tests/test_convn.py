"""Narrow-output implicit-GEMM convolution (kernels/convn.hip) vs PyTorch fp32 ``F.conv2d``, and
the BatchNorm statistics it reduces in its epilogue vs the fp32 reference statistics of the
stored output.

Operands are small integers (exact in bf16 and in the fp32 accumulator), so a wrong gathered pixel,
a missed zero pad, a swapped (r, s) or a misplaced output column is a hard mismatch."""
import pytest
import torch
import torch.nn.functional as F

from parameter_server_distributed_amd import native

pytestmark = pytest.mark.gpu

CASES = [  # Nb, C, H, W, Cout, R, stride, pad
    (4, 64, 14, 14, 64, 3, 1, 1),      # layer1 conv2 shape family (BN = 64)
    (3, 128, 14, 14, 128, 3, 1, 1),    # layer2 conv2 (BN = 128), ragged M (588 rows)
    (4, 128, 28, 28, 128, 3, 2, 1),    # strided 3x3
    (2, 256, 15, 17, 64, 1, 1, 0),     # 1x1 256 -> 64, odd image, ragged M
    (2, 64, 14, 14, 256, 1, 1, 0),     # 1x1 K = 64 -> 256 (layer1 conv3: one K-tile)
    (2, 128, 7, 9, 512, 1, 1, 0),      # 1x1 -> 512: two 256-wide column tiles
    (2, 256, 14, 14, 512, 1, 2, 0),    # strided 1x1 (downsample)
    (1, 64, 5, 5, 64, 3, 1, 1),        # M = 25 < one tile
]


def _w2(w):
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1).contiguous()


def _case(case, gpu, seed=7):
    Nb, C, H, W, Cout, R, stride, pad = case
    g = torch.Generator().manual_seed(seed)
    x = torch.randint(-2, 3, (Nb, C, H, W), generator=g).float()
    w = torch.randint(-2, 3, (Cout, C, R, R), generator=g).float()
    ref = F.conv2d(x, w, stride=stride, padding=pad)
    xd = x.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    return x, w, ref, xd


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_convn_exact(gpu, case):
    """Every tile variant of the output width, exact against fp32 F.conv2d."""
    Nb, C, H, W, Cout, R, stride, pad = case
    x, w, ref, xd = _case(case, gpu)
    Ho, Wo = ref.shape[2], ref.shape[3]
    want = ref.permute(0, 2, 3, 1).reshape(-1, Cout).bfloat16().float()
    w2 = _w2(w.to(gpu, torch.bfloat16))
    nv = native().convn_variants(Cout)
    assert nv >= 2
    for v in range(nv):
        if not native().convn_variant_ok(Cout, v, R, R, stride, pad, Wo):
            continue
        out = torch.full((Nb * Ho * Wo, Cout), 7.0, device=gpu, dtype=torch.bfloat16)
        assert native().convn_(xd, w2, out, R, R, stride, pad, variant=v) == 1
        torch.testing.assert_close(out.float().cpu(), want, rtol=0, atol=0, msg=lambda m: f"variant {v}: {m}")


@pytest.mark.parametrize("case", CASES[:5], ids=lambda c: "x".join(map(str, c)))
def test_convn_stats_partials(gpu, case):
    """Summed over the partial rows, the epilogue's shifted sums equal the fp32 sums of the stored
    bf16 output (exact-integer data: every partial is an exact fp32 integer sum)."""
    Nb, C, H, W, Cout, R, stride, pad = case
    x, w, ref, xd = _case(case, gpu, seed=11)
    M = ref.numel() // Cout
    shift = torch.randint(-3, 4, (Cout,)).float().to(gpu)
    Ho, Wo = ref.shape[2], ref.shape[3]
    for v in range(native().convn_variants(Cout)):
        if not native().convn_variant_ok(Cout, v, R, R, stride, pad, Wo):
            continue
        nrow = max(native().convn_stats_rows(M), native().convn_part_rows(M, Cout, v, Ho, Wo, R))
        part = torch.full((nrow, 2, Cout), float("nan"), device=gpu)
        out = torch.empty(M, Cout, device=gpu, dtype=torch.bfloat16)
        rows = native().convn_(xd, _w2(w.to(gpu, torch.bfloat16)), out, R, R, stride, pad, part=part, shift=shift,
                               variant=v)
        assert 1 <= rows <= part.shape[0]
        y = out.double().cpu()
        d = y - shift.double().cpu()
        got = part[:rows].double().cpu().sum(0)
        assert torch.isfinite(got).all(), v
        torch.testing.assert_close(got[0], d.sum(0), rtol=1e-6, atol=1e-3)
        torch.testing.assert_close(got[1], (d * d).sum(0), rtol=1e-6, atol=1e-3)


def test_convn_declines_unsupported(gpu):
    x = torch.zeros(2, 96, 8, 8, device=gpu, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out = torch.empty(2 * 64, 64, device=gpu, dtype=torch.bfloat16)
    assert native().convn_(x, torch.zeros(64, 9 * 96, device=gpu, dtype=torch.bfloat16), out, 3, 3, 1, 1) == 0
    x = torch.zeros(2, 64, 8, 8, device=gpu, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out = torch.empty(2 * 64, 96, device=gpu, dtype=torch.bfloat16)  # 96 output channels: no tile
    assert native().convn_(x, torch.zeros(96, 9 * 64, device=gpu, dtype=torch.bfloat16), out, 3, 3, 1, 1) == 0


@pytest.mark.parametrize("relu", [False, True])
def test_bn_fwd_from_conv_partials_matches_fp32(gpu, relu):
    """BN forward fed with the convolution's statistics partials (fold + finalize, no reduce pass)
    vs fp32 F.batch_norm on the same bf16 conv output: output, batch statistics, running stats."""
    torch.manual_seed(5)
    Nb, C, H, W, Cout = 8, 64, 28, 28, 64  # M = 6272 -> 98 partial rows
    x = torch.randn(Nb, C, H, W, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, C, 3, 3, device=gpu) * 0.05).to(torch.bfloat16)
    M = Nb * H * W
    rm = torch.randn(Cout, device=gpu) * 0.1
    rv = torch.rand(Cout, device=gpu) + 0.5
    gamma = (torch.rand(Cout, device=gpu) + 0.5).to(torch.bfloat16)
    beta = (torch.randn(Cout, device=gpu) * 0.1).to(torch.bfloat16)
    part = torch.empty(native().convn_stats_rows(M), 2, Cout, device=gpu)
    out = torch.empty(M, Cout, device=gpu, dtype=torch.bfloat16)
    rows = native().convn_(x, _w2(w), out, 3, 3, 1, 1, part=part, shift=rm)
    assert rows > 0
    y4 = out.view(Nb, H, W, Cout).permute(0, 3, 1, 2)
    rm1, rv1 = rm.clone(), rv.clone()
    cnt = torch.zeros((), dtype=torch.int64, device=gpu)
    yb, mean, invstd, _, _ = native().bn_fwd(y4, gamma, beta, rm1, rv1, None, relu, True, 0.1, 1e-5, cnt, None,
                                             part_in=part, part_rows=rows)
    rm2, rv2 = rm.clone(), rv.clone()
    ref = F.batch_norm(y4.float(), rm2, rv2, gamma.float(), beta.float(), True, 0.1, 1e-5)
    if relu:
        ref = F.relu(ref)
    yf = y4.float()
    torch.testing.assert_close(mean, yf.mean((0, 2, 3)), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(invstd, torch.rsqrt(yf.var((0, 2, 3), unbiased=False) + 1e-5), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rm1, rm2, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rv1, rv2, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(yb.float(), ref, rtol=1e-2, atol=2e-2)
    assert int(cnt) == 1


@pytest.mark.parametrize("k,cin,cout,stride", [(3, 64, 64, 1), (1, 256, 64, 1), (1, 64, 256, 1), (3, 128, 128, 2)])
def test_conv_bn_module_psdn_route_matches_fp32(gpu, monkeypatch, k, cin, cout, stride):
    """The model-level route: ConvNHWC / Conv1x1 forced onto the narrow kernel (forward, stride-1
    bwd-data) with the consumer FusedBatchNorm2d's statistics reduced in the conv epilogue, vs an
    fp32 nn.Conv2d + F.batch_norm (+ ReLU) on the same bf16 operands: output, running stats and the
    input / weight / BN gradients."""
    from parameter_server_distributed_amd.ops.bn import FusedBatchNorm2d
    from parameter_server_distributed_amd.ops.conv import Conv1x1, ConvNHWC

    monkeypatch.setenv("PSD_AUTOTUNE_FORCE", "psdn0")
    torch.manual_seed(3)
    conv = (Conv1x1(cin, cout) if k == 1 and stride == 1 else ConvNHWC(cin, cout, k, stride))
    conv = conv.to(gpu, torch.bfloat16).to(memory_format=torch.channels_last)
    bn = FusedBatchNorm2d(cout, relu=True).to(gpu)
    bn.weight.data = bn.weight.data.to(torch.bfloat16)
    bn.bias.data = bn.bias.data.to(torch.bfloat16)
    object.__setattr__(conv, "_psd_bn", bn)
    ref = torch.nn.Conv2d(cin, cout, k, stride=stride, padding=k // 2, bias=False).to(gpu)
    ref.weight.data.copy_(conv.weight.float())
    x = torch.randn(8, cin, 16, 16, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    xr = x.detach().float().clone().requires_grad_(True)
    rm, rv = bn.running_mean.clone(), bn.running_var.clone()
    gw = bn.weight.detach().float().clone().requires_grad_(True)
    gb = bn.bias.detach().float().clone().requires_grad_(True)
    y = bn(conv(x))
    assert bn._psd_stats_pending is None  # handed over and consumed
    yr = F.relu(F.batch_norm(ref(xr), rm, rv, gw, gb, True, 0.1, 1e-5))
    torch.testing.assert_close(y.float(), yr.detach(), rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(bn.running_mean, rm, rtol=1e-2, atol=1e-3)
    torch.testing.assert_close(bn.running_var, rv, rtol=1e-2, atol=1e-3)
    g = torch.randn_like(yr)
    y.backward(g.to(torch.bfloat16))
    yr.backward(g)
    for got, want in ((x.grad, xr.grad), (conv.weight.grad, ref.weight.grad), (bn.weight.grad, gw.grad),
                      (bn.bias.grad, gb.grad)):
        err = float((got.float() - want).abs().max())
        assert err < 0.05 * float(want.abs().max()) + 1e-3, (err, float(want.abs().max()))


def test_resnet_convn_fusions_match_library_path(gpu, monkeypatch):
    """ResNet-50 end to end with the narrow kernel forced wherever it applies -- forward with the
    consumer BN's statistics in the epilogue, bwd-data with the producing BN's backward reduction
    in the epilogue (bn1 / bn2 from x and scale/shift; identity-block bn3 with the residual
    gradient added under the bit-mask) -- vs the same model with the kernel off (library
    convolutions, separate BN passes): loss and every parameter gradient. The recomputing tails
    (ops/tail.py, pinned against fp32 in test_tail.py) are off on both sides: 16 bottlenecks at
    batch 8 amplify their forward rounding differences past this bf16-vs-bf16 bound."""
    from parameter_server_distributed_amd import models
    from parameter_server_distributed_amd.ops import autotune

    res = []
    for on in (True, False):
        monkeypatch.setenv("PSD_FEATURES", f"convn={int(on)},tail_recompute=0")
        monkeypatch.setenv("PSD_AUTOTUNE_FORCE", "psdnb0,psdn0" if on else "miopen")
        autotune._DECISIONS.clear()
        torch.manual_seed(0)
        spec = models.build("resnet50", gpu, torch.bfloat16, image_size=64, num_classes=10)
        m = spec.model
        for p in m.parameters():  # bf16 parameters (the PS data plane's working copy)
            p.data = p.data.to(torch.bfloat16)
        x, y = spec.make_batch(8, gpu, seed=3)
        loss = spec.loss(m(x), y)
        loss.backward()
        res.append((float(loss), {n: p.grad.float().clone() for n, p in m.named_parameters()},
                    {n: b.clone() for n, b in m.named_buffers() if "running" in n}))
        if on:  # the fused paths actually ran
            picks = autotune.decisions()
            assert any(v == "psdnb0" for v in picks.values()), picks
            assert any(v == "psdn0" for k, v in picks.items() if "bnstats" in k), picks
    autotune._DECISIONS.clear()
    assert abs(res[0][0] - res[1][0]) < 0.02 * abs(res[1][0]) + 1e-3, (res[0][0], res[1][0])
    for n in res[1][1]:
        a, b = res[0][1][n], res[1][1][n]
        if b.norm() == 0:
            assert a.norm() < 1e-3, n
            continue
        assert ((a - b).norm() / b.norm()).item() < 0.1, n
    for n in res[1][2]:
        torch.testing.assert_close(res[0][2][n], res[1][2][n], rtol=2e-2, atol=2e-3, msg=n)


HALO_CASES = [  # Nb, C, H(=W), Cout: the persistent HALO kernel's shapes (C = N = 64, stride-1 3x3)
    (2, 64, 56, 64), (3, 64, 30, 64), (4, 64, 9, 64),
]


@pytest.mark.parametrize("case", HALO_CASES, ids=lambda c: "x".join(map(str, c)))
def test_convn_halo_exact_with_stats(gpu, case):
    """The persistent HALO variant (convh_kernel: input window staged once, taps read as shifted
    rows): exact against fp32 F.conv2d, and its statistics partials sum to the fp32 sums of the
    stored output."""
    Nb, C, H, Cout = case
    x, w, ref, xd = _case((Nb, C, H, H, Cout, 3, 1, 1), gpu)
    M = Nb * H * H
    want = ref.permute(0, 2, 3, 1).reshape(-1, Cout).bfloat16().float()
    w2 = _w2(w.to(gpu, torch.bfloat16))
    C_ = native()
    halo = [v for v in range(C_.convn_variants(Cout)) if C_.convn_variant_kind(Cout, v) == 2]
    assert halo and all(C_.convn_variant_ok(Cout, v, 3, 3, 1, 1, H) for v in halo)
    shift = torch.zeros(Cout, device=gpu)
    for v in halo:
        out = torch.full((M, Cout), 7.0, device=gpu, dtype=torch.bfloat16)
        assert C_.convn_(xd, w2, out, 3, 3, 1, 1, variant=v) == 1
        torch.testing.assert_close(out.float().cpu(), want, rtol=0, atol=0, msg=lambda m: f"variant {v}: {m}")
        rows_alloc = max(C_.convn_stats_rows(M), C_.convn_part_rows(M, Cout, v, H, H, 3))
        part = torch.full((rows_alloc, 2, Cout), float("nan"), device=gpu)
        rows = C_.convn_(xd, w2, out, 3, 3, 1, 1, part=part, shift=shift, variant=v)
        assert rows == C_.convn_part_rows(M, Cout, v, H, H, 3)
        s1 = part[:rows, 0].double().sum(0).cpu()
        s2 = part[:rows, 1].double().sum(0).cpu()
        o = out.double().cpu()
        torch.testing.assert_close(s1, o.sum(0), rtol=1e-6, atol=1e-3)
        torch.testing.assert_close(s2, (o * o).sum(0), rtol=1e-6, atol=1e-3)


def test_convn_halo_declines_where_it_cannot_tile(gpu):
    C_ = native()
    hv = 4  # first HALO variant of a 64-wide output
    assert not C_.convn_variant_ok(64, hv, 3, 3, 2, 1, 28)   # strided
    assert not C_.convn_variant_ok(64, hv, 1, 1, 1, 0, 56)   # 1x1
    assert not C_.convn_variant_ok(64, hv, 3, 3, 1, 1, 63)   # Wo + 2 > 64
    assert C_.convn_variant_ok(64, hv, 3, 3, 1, 1, 62)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,N,H", [(1, 256, 14), (2, 256, 14), (5, 256, 14), (2, 128, 10), (5, 64, 12), (1, 64, 9)])
def test_convn_bwd_epilogue_exact(gpu, mode, N, H):
    """The bwd-data epilogue of a 1x1 convolution (out = dY . W^T, K = 64) against an fp64 reference:
    mode 1 g = (x * scale + shift > 0) ? out : 0; mode 2 g = bit ? out + dr : 0; mode 5 as 2 with dr
    on the stride-2 quarter grid (added at even (h, w) only); partials sum g and sum g (x - mean) per
    channel, every tile variant. Small-integer operands: every value is exact in bf16 and fp32."""
    Nb, K = 3, 64
    g = torch.Generator().manual_seed(21)
    dy = torch.randint(-1, 2, (Nb, K, H, H), generator=g).float()
    w2 = torch.randint(-1, 2, (N, K), generator=g).float()
    M = Nb * H * H
    out_ref = dy.permute(0, 2, 3, 1).reshape(M, K).double() @ w2.double().t()
    bx = torch.randint(-3, 4, (M, N), generator=g).float()
    mean = torch.randint(-2, 3, (N,), generator=g).float()
    C_ = native()
    args = {}
    if mode == 1:
        scale = torch.randint(1, 3, (N,), generator=g).float()
        shift = torch.randint(-3, 4, (N,), generator=g).float() + 0.5  # never exactly zero
        keep = (bx * scale + shift) > 0
        gref = torch.where(keep, out_ref, torch.zeros_like(out_ref))
        args["bss"] = torch.cat([scale, shift]).to(gpu)
    else:
        bits = torch.randint(0, 2, (M, N), generator=g).bool()
        packed = (bits.view(M * N // 8, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)).sum(1).to(torch.uint8)
        args["bmbits"] = packed.to(gpu)
        if mode == 2:
            dr = torch.randint(-2, 3, (M, N), generator=g).float()
            add = dr.double()
            args["bdr"] = dr.to(gpu, torch.bfloat16)
        else:
            dr4 = torch.randint(-2, 3, (Nb, N, H // 2, H // 2), generator=g).float()
            full = torch.zeros(Nb, N, H, H)
            full[:, :, ::2, ::2] = dr4
            add = full.permute(0, 2, 3, 1).reshape(M, N).double()
            args["bdr"] = dr4.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
        gref = torch.where(bits, out_ref + add, torch.zeros_like(out_ref))
    s1 = gref.sum(0)
    s2 = (gref * (bx.double() - mean.double())).sum(0)
    dyd = dy.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w2d = w2.to(gpu, torch.bfloat16)
    nvar = 0
    for v in range(C_.convn_variants(N)):
        if not C_.convn_variant_ok(N, v, 1, 1, 1, 0, H):
            continue
        nvar += 1
        out = torch.full((M, N), 7.0, device=gpu, dtype=torch.bfloat16)
        part = torch.full((max(C_.convn_stats_rows(M), C_.convn_part_rows(M, N, v, H, H, 1)), 2, N), float("nan"),
                          device=gpu)
        rows = C_.convn_bwd_(dyd, w2d, out, 1, 1, 1, 0, part, v, mode, bx.to(gpu, torch.bfloat16), mean.to(gpu),
                             **args)
        assert rows > 0, v
        torch.testing.assert_close(out.double().cpu(), gref, rtol=0, atol=0, msg=lambda m: f"variant {v}: {m}")
        got = part[:rows].double().cpu().sum(0)
        torch.testing.assert_close(got[0], s1, rtol=0, atol=1e-6, msg=lambda m: f"variant {v} sum g: {m}")
        torch.testing.assert_close(got[1], s2, rtol=0, atol=1e-6, msg=lambda m: f"variant {v} sum g(x-mean): {m}")
    assert nvar >= 2


@pytest.mark.parametrize("Nb,H", [(2, 56), (3, 13), (1, 62), (2, 2)])
@pytest.mark.parametrize("mode", [1, 2])
def test_convn_persistent_bwd_matches_gathered(gpu, Nb, H, mode):
    """The persistent HALO variant (kind 2: C = N = 64 3x3, resident weights, double-buffered
    windows) as a stride-1 bwd-data with the producing BN's backward reduction in the epilogue
    (mode 1: ReLU mask from x and scale/shift; mode 2: bit-mask + handed-over residual gradient):
    output and summed partials equal the gathered variant's exactly (small-integer operands: every
    value and sum is exact). Odd and tiny images: partial last tiles, one-row images."""
    C_ = native()
    g = torch.Generator().manual_seed(5)
    dy = torch.randint(-1, 2, (Nb, 64, H, H), generator=g).float()
    w = torch.randint(-1, 2, (64, 64, 3, 3), generator=g).float()
    M = Nb * H * H
    bx = torch.randint(-3, 4, (M, 64), generator=g).to(gpu, torch.bfloat16)
    mean = torch.randint(-2, 3, (64,), generator=g).float().to(gpu)
    args = {}
    if mode == 1:
        args["bss"] = torch.cat([torch.randint(1, 3, (64,), generator=g).float(),
                                 torch.randint(-3, 4, (64,), generator=g).float() + 0.5]).to(gpu)
    else:
        bits = torch.randint(0, 2, (M * 64,), generator=g).bool().view(-1, 8)
        args["bmbits"] = (bits.to(torch.uint8) << torch.arange(8, dtype=torch.uint8)).sum(1).to(torch.uint8).to(gpu)
        args["bdr"] = torch.randint(-2, 3, (M, 64), generator=g).to(gpu, torch.bfloat16)
    dyd = dy.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wf = _w2(w.flip(2, 3).permute(1, 0, 2, 3).contiguous().to(gpu, torch.bfloat16))
    pv = [v for v in range(C_.convn_variants(64)) if C_.convn_variant_kind(64, v) == 2]
    assert len(pv) == 1 and C_.convn_variant_ok(64, pv[0], 3, 3, 1, 1, H)
    res = {}
    for v in (0, pv[0]):
        out = torch.full((M, 64), 7.0, device=gpu, dtype=torch.bfloat16)
        part = torch.full((max(C_.convn_stats_rows(M), C_.convn_part_rows(M, 64, v, H, H, 3)), 2, 64), float("nan"),
                          device=gpu)
        rows = C_.convn_bwd_(dyd, wf, out, 3, 3, 1, 1, part, v, mode, bx, mean, **args)
        assert rows == C_.convn_part_rows(M, 64, v, H, H, 3) > 0
        res[v] = (out.float().cpu(), part[:rows].double().sum(0).cpu())
    ref = F.conv_transpose2d(dy, w, padding=1)  # dX of conv(x, w): the bwd-data the kernel computes
    o0, p0 = res[0]
    assert torch.isfinite(p0).all()
    o1, p1 = res[pv[0]]
    torch.testing.assert_close(o1, o0, rtol=0, atol=0)
    torch.testing.assert_close(p1, p0, rtol=0, atol=1e-6)
    raw = ref.permute(0, 2, 3, 1).reshape(M, 64)
    assert ((o0 == 0) | (o0 == raw) | (mode == 2)).all()  # mode 1: masked copy of dX


S2_CASES = [  # Nb, Cin (= dX channels), H (= 2 Ho), Cout (= dY channels)
    (2, 128, 56, 128),   # layer2's first conv2 (BN = 128)
    (3, 256, 14, 256),   # layer3 family, ragged M (3 x 7 x 7 = 147 rows per phase)
    (2, 512, 14, 512),   # layer4: two 256-wide column tiles
    (2, 64, 28, 128),    # Cin 64 (BN = 64)
]


@pytest.mark.parametrize("nb,cin,H,cout", S2_CASES)
def test_dgrad_s2_phases_exact(gpu, nb, cin, H, cout):
    """Stride-2 3x3 bwd-data as four output-parity phase launches (convn_dgrad_s2_, kernels/convn.hip
    ophase) == fp32 conv2d_input on small-integer operands (exact), every gathered variant; the
    fused mode-1 epilogue: g = dX * relu'(bx * scale + shift) and the partials sum g, sum g (bx - mean)
    vs fp32 references."""
    from parameter_server_distributed_amd.ops.conv import _s2_phase_weights

    C = native()
    g = torch.Generator().manual_seed(0)
    w = torch.randint(-2, 3, (cout, cin, 3, 3), generator=g).float()
    dy = torch.randint(-2, 3, (nb, cout, H // 2, H // 2), generator=g).float()
    ref = torch.nn.grad.conv2d_input((nb, cin, H, H), w, dy, stride=2, padding=1)
    wb = w.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dyb = dy.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wph = _s2_phase_weights(wb)
    ref_cl = ref.permute(0, 2, 3, 1).reshape(-1, cin).to(gpu)
    vs = [v for v in range(C.convn_variants(cin)) if C.convn_variant_kind(cin, v) == 0]
    assert vs
    bx = torch.randn(nb, cin, H, H, generator=g).to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    mean = torch.randn(cin, generator=g).to(gpu)
    ss = torch.cat([torch.rand(cin, generator=g) + 0.5, 0.3 * torch.randn(cin, generator=g)]).to(gpu)
    bx2 = bx.permute(0, 2, 3, 1).reshape(-1, cin).float()
    mask = (bx2 * ss[:cin] + ss[cin:]) > 0
    g_ref = torch.where(mask, ref_cl, torch.zeros_like(ref_cl))
    for v in vs:
        out = torch.full((nb * H * H, cin), float("nan"), device=gpu, dtype=torch.bfloat16)
        assert C.convn_dgrad_s2_(dyb, wph, out, v) == 1
        # exact up to the bf16 rounding of the stored output (|dX| > 256 rounds; and every pixel written)
        torch.testing.assert_close(out.float(), ref_cl, rtol=1 / 128, atol=0)
        part = torch.empty(C.convn_dgrad_s2_rows(nb, H // 2, H // 2, cin, v), 2, cin, device=gpu)
        out2 = torch.full_like(out, float("nan"))
        rows = C.convn_dgrad_s2_(dyb, wph, out2, v, part=part, bx=bx, bmean=mean, bss=ss)
        assert 0 < rows <= part.shape[0]
        torch.testing.assert_close(out2.float(), g_ref, rtol=1 / 128, atol=0)
        s1 = part[:rows, 0].double().sum(0)
        s2 = part[:rows, 1].double().sum(0)
        e1 = g_ref.double().sum(0)
        # (the kernel sums the bf16-stored g)
        gq = out2.float().double()
        torch.testing.assert_close(s1, gq.sum(0), rtol=1e-5, atol=1e-2)
        torch.testing.assert_close(s2, (gq * (bx2.double() - mean.double())).sum(0), rtol=1e-4, atol=1e-1)
        torch.testing.assert_close(s1, e1, rtol=1e-2, atol=1.0)


def test_dgrad_s2_in_resnet_block_matches_miopen(gpu, monkeypatch):
    """A stride-2 bottleneck's conv2 bwd-data on the phase kernels (forced, plain and with bn1's
    reduction fused) vs MIOpen, all three against an fp32 composite run of the same block: block
    input gradient and every parameter gradient at MIOpen's bf16 error level (the BN weight
    gradients are near-cancelling sums: two bf16 paths differ by several % on them, so each is
    compared through fp32)."""
    import copy

    import torch.nn as nn

    from parameter_server_distributed_amd.models.resnet import Bottleneck, _conv
    from parameter_server_distributed_amd.ops import autotune
    from parameter_server_distributed_amd.ops.bn import FusedBatchNorm2d

    torch.manual_seed(0)
    blk0 = Bottleneck(256, 128, 2, 64, nn.Sequential(_conv(256, 512, 1, 2), FusedBatchNorm2d(512)))
    blk0 = blk0.to(gpu).to(memory_format=torch.channels_last)
    for p in blk0.parameters():
        p.data = p.data.to(torch.bfloat16)
    x0 = torch.randn(4, 256, 28, 28, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    def run(blk, x):
        x = x.clone().requires_grad_(True)
        blk(x).float().pow(2).mean().backward()
        return {"dx": x.grad.float(), **{n: p.grad.float() for n, p in blk.named_parameters()}}

    monkeypatch.setenv("PSD_FEATURES", "tail_recompute=0")
    res = {}
    s2 = lambda k: k[:2] == ("conv", "dgrad") and k[8] == 2  # noqa: E731 (the stride-2 bwd-data key)
    others = None
    for force in ("miopen", "psdnbs0", "psdns0"):
        monkeypatch.setenv("PSD_AUTOTUNE_FORCE", force)
        autotune._DECISIONS.clear()
        if others is not None:
            # every other op of the block on the MIOpen run's picks: only the stride-2 bwd-data differs
            # between the runs (per-run autotune picks elsewhere moved the near-cancelling BN weight
            # gradients by up to ~9 % and made the comparison flaky)
            autotune._DECISIONS.update(others)
        res[force] = run(copy.deepcopy(blk0), x0)
        picks = autotune.decisions()
        got = [v for k, v in picks.items() if s2(k)]
        assert got == [force], picks
        if others is None:
            others = {k: v for k, v in picks.items() if not s2(k)}
    autotune._DECISIONS.clear()
    ref = run(copy.deepcopy(blk0).float(), x0.float())

    def err(g, n):
        return ((g[n] - ref[n]).norm() / ref[n].norm().clamp_min(1e-6)).item()

    for force in ("psdnbs0", "psdns0"):
        for n in ref:
            assert err(res[force], n) <= 1.5 * err(res["miopen"], n) + 1e-2, (force, n, err(res[force], n),
                                                                              err(res["miopen"], n))
