"""BatchNorm statistics in the 8-phase GEMM epilogue (kernels/gemm.hip ST): the shifted per-channel
sums of the stored bf16 output, as partial rows for the consumer BN's finalize, on every launch path
that feeds a BN -- the bf16 GEMM (1x1 convolutions), the implicit-GEMM convolution, and their fp8
forms (per-tensor and MX block scales) -- vs fp64 sums of the output read back; and the module route
(the BN consumes the partials and skips its reduce) vs an fp32 reference.

Operands are small integers: every product, the fp32 accumulators and the fp32 partial sums are
exact, so the partials (taken from the accumulators, before the bf16 rounding of the store) must
match the fp64 sums of the exact product to rounding of the final fp64 comparison only."""
import pytest
import torch
import torch.nn.functional as F

from parameter_server_distributed_amd import native

pytestmark = pytest.mark.gpu
CL = torch.channels_last


def _ints(shape, gen, lo=-2, hi=3):
    return torch.randint(lo, hi, shape, generator=gen).float()


def _check(exact2d, part, rows, shift):
    assert rows > 0
    y = exact2d.double().cpu()
    d = y - shift.double().cpu()
    got = part[:rows].double().cpu().sum(0)
    assert torch.isfinite(got).all()
    torch.testing.assert_close(got[0], d.sum(0), rtol=1e-6, atol=1e-3)
    torch.testing.assert_close(got[1], (d * d).sum(0), rtol=1e-6, atol=1e-3)


@pytest.mark.parametrize("M,N,K", [(4000, 512, 256), (16384, 256, 512), (3000, 1024, 256)])
def test_gemm_stats_bf16(gpu, M, N, K):
    g = torch.Generator().manual_seed(1)
    A, B = _ints((M, K), g).to(gpu, torch.bfloat16), _ints((N, K), g).to(gpu, torch.bfloat16)
    shift = _ints((N,), g, -3, 4).to(gpu)
    out = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    part = torch.full((native().gemm_stats_rows(M), 2, N), float("nan"), device=gpu)
    rows = native().gemm_(A, B, True, True, out, part=part, shift=shift)
    exact = A.double().cpu() @ B.double().cpu().t()
    torch.testing.assert_close(out.float().cpu(), exact.float().bfloat16().float(), rtol=0, atol=0)
    _check(exact, part, rows, shift)


def test_gemm_stats_declines_small(gpu):
    """Too few tiles for the 8-phase kernel: nothing launched, 0 returned (the caller's BN reduces)."""
    A = torch.zeros(256, 256, device=gpu, dtype=torch.bfloat16)
    B = torch.zeros(256, 256, device=gpu, dtype=torch.bfloat16)
    out = torch.full((256, 256), 7.0, device=gpu, dtype=torch.bfloat16)
    part = torch.empty(native().gemm_stats_rows(256), 2, 256, device=gpu)
    assert native().gemm_(A, B, True, True, out, part=part, shift=torch.zeros(256, device=gpu)) == 0
    assert bool((out.float() == 7.0).all())


@pytest.mark.parametrize("mx", [False, True])
def test_gemm_fp8_stats(gpu, mx):
    M, N, K = 4000, 512, 256
    g = torch.Generator().manual_seed(2)
    A, B = _ints((M, K), g), _ints((N, K), g)
    Aq, Bq = A.to(gpu).to(torch.float8_e4m3fn), B.to(gpu).to(torch.float8_e4m3fn)
    if mx:  # E8M0 127 = 2^0
        sa = torch.full((M, K // 32), 127, device=gpu, dtype=torch.uint8)
        sb = torch.full((N, K // 32), 127, device=gpu, dtype=torch.uint8)
    else:
        sa, sb = torch.ones(1, device=gpu), torch.ones(1, device=gpu)
    shift = _ints((N,), g, -3, 4).to(gpu)
    out = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    part = torch.full((native().gemm_stats_rows(M), 2, N), float("nan"), device=gpu)
    rows = native().gemm_fp8_(Aq, Bq, sa, sb, out, part=part, shift=shift)
    exact = A.double() @ B.double().t()
    torch.testing.assert_close(out.float().cpu(), exact.float().bfloat16().float(), rtol=0, atol=0)
    _check(exact, part, rows, shift)


@pytest.mark.parametrize("fp8", [None, "tensor", "mx"])
def test_conv_fwd_stats(gpu, fp8):
    g = torch.Generator().manual_seed(3)
    C = 64 if fp8 is None else 128
    Nb, H, Cout = 4, 12, 256
    x, w = _ints((Nb, C, H, H), g), _ints((Cout, C, 3, 3), g)
    ref = F.conv2d(x, w, padding=1).permute(0, 2, 3, 1).reshape(-1, Cout)
    M = ref.shape[0]
    w2 = w.permute(0, 2, 3, 1).reshape(Cout, -1).contiguous()
    shift = _ints((Cout,), g, -3, 4).to(gpu)
    out = torch.empty(M, Cout, device=gpu, dtype=torch.bfloat16)
    part = torch.full((native().gemm_stats_rows(M), 2, Cout), float("nan"), device=gpu)
    if fp8 is None:
        rows = native().conv_fwd_(x.to(gpu, torch.bfloat16).contiguous(memory_format=CL), w2.to(gpu, torch.bfloat16),
                                  out, 3, 3, 1, 1, part=part, shift=shift)
    else:
        xq = x.to(gpu).permute(0, 2, 3, 1).contiguous().to(torch.float8_e4m3fn).permute(0, 3, 1, 2)
        wq = w2.to(gpu).to(torch.float8_e4m3fn)
        if fp8 == "mx":
            sx = torch.full((x.numel() // 32,), 127, device=gpu, dtype=torch.uint8)
            sw = torch.full((w2.numel() // 32,), 127, device=gpu, dtype=torch.uint8)
        else:
            sx, sw = torch.ones(1, device=gpu), torch.ones(1, device=gpu)
        rows = native().conv_fwd_fp8_(xq, wq, sx, sw, out, 3, 3, 1, 1, part=part, shift=shift)
    torch.testing.assert_close(out.float().cpu(), ref.bfloat16().float(), rtol=0, atol=0)
    _check(ref, part, rows, shift)


@pytest.mark.parametrize("k,cin,cout,force", [(1, 256, 256, "psds"), (3, 64, 256, "psds_igemm")])
def test_module_route_with_gemm_stats_matches_fp32(gpu, monkeypatch, k, cin, cout, force):
    """Conv1x1 / ConvNHWC forced onto the statistics-epilogue GEMM, its FusedBatchNorm2d consuming the
    partials (no reduce pass), vs fp32 nn.Conv2d + F.batch_norm + ReLU: output and running stats."""
    from parameter_server_distributed_amd.ops import autotune
    from parameter_server_distributed_amd.ops.bn import FusedBatchNorm2d
    from parameter_server_distributed_amd.ops.conv import Conv1x1, ConvNHWC

    monkeypatch.setenv("PSD_AUTOTUNE_FORCE", force)
    autotune._DECISIONS.clear()
    torch.manual_seed(4)
    conv = Conv1x1(cin, cout) if k == 1 else ConvNHWC(cin, cout, k, 1)
    conv = conv.to(gpu, torch.bfloat16).to(memory_format=CL)
    bn = FusedBatchNorm2d(cout, relu=True).to(gpu)
    bn.weight.data = bn.weight.data.to(torch.bfloat16)
    bn.bias.data = bn.bias.data.to(torch.bfloat16)
    object.__setattr__(conv, "_psd_bn", bn)
    ref = torch.nn.Conv2d(cin, cout, k, padding=k // 2, bias=False).to(gpu)
    ref.weight.data.copy_(conv.weight.float())
    x = torch.randn(16, cin, 32, 32, device=gpu).to(torch.bfloat16).contiguous(memory_format=CL)
    x.requires_grad_(True)
    rm, rv = bn.running_mean.clone(), bn.running_var.clone()
    y = bn(conv(x))
    assert bn._psd_stats_pending is None
    assert force in autotune.decisions().values(), autotune.decisions()
    yr = F.relu(F.batch_norm(ref(x.detach().float()), rm, rv, bn.weight.float(), bn.bias.float(), True, 0.1, 1e-5))
    torch.testing.assert_close(y.float(), yr, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(bn.running_mean, rm, rtol=1e-2, atol=1e-3)
    torch.testing.assert_close(bn.running_var, rv, rtol=1e-2, atol=1e-3)
    autotune._DECISIONS.clear()


def test_fp8_conv_bn_stats_handover_matches_reduce(gpu, monkeypatch):
    """An fp8 Conv1x1 + BN with the statistics from the fp8 GEMM epilogue vs the same with the BN's
    own reduce pass (feature gemm_stats off): identical conv output, so BN output and running stats agree
    to fp32 summation order."""
    from parameter_server_distributed_amd.ops.bn import FusedBatchNorm2d
    from parameter_server_distributed_amd.ops.conv import Conv1x1

    res = []
    for on in ("1", "0"):
        monkeypatch.setenv("PSD_FEATURES", f"gemm_stats={on}")
        torch.manual_seed(5)
        conv = Conv1x1(256, 512, fp8=True).to(gpu, torch.bfloat16).to(memory_format=CL)
        bn = FusedBatchNorm2d(512, relu=True).to(gpu)
        bn.weight.data = bn.weight.data.to(torch.bfloat16)
        bn.bias.data = bn.bias.data.to(torch.bfloat16)
        object.__setattr__(conv, "_psd_bn", bn)
        x = torch.randn(16, 256, 32, 32, device=gpu).to(torch.bfloat16).contiguous(memory_format=CL)
        x.requires_grad_(True)
        y = bn(conv(x))
        res.append((y.float(), bn.running_mean.clone(), bn.running_var.clone()))
    torch.testing.assert_close(res[0][0], res[1][0], rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(res[0][1], res[1][1], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(res[0][2], res[1][2], rtol=1e-4, atol=1e-5)
