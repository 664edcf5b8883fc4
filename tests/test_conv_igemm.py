"""Implicit-GEMM NHWC convolution forward (kernels/gemm.hip, GA mode of the 8-phase kernel) vs
PyTorch fp32 ``F.conv2d``: small-integer operands (exact in bf16 and in the fp32 accumulator) so a
wrong gathered pixel, a missed zero-pad or a swapped (r, s) shows up as a hard mismatch."""
import pytest
import torch
import torch.nn.functional as F

from parameter_server_distributed_amd import native

pytestmark = pytest.mark.gpu

CASES = [  # Nb, C, H, W, Cout, R, stride, pad
    (4, 64, 14, 14, 256, 3, 1, 1),
    (8, 128, 28, 28, 256, 3, 2, 1),
    (8, 256, 28, 28, 512, 1, 2, 0),
    (256, 256, 14, 14, 512, 3, 1, 1),  # 392 tiles: several per persistent workgroup
    (3, 512, 7, 7, 256, 3, 1, 1),      # ragged M (147 rows)
    (16, 64, 15, 17, 264, 3, 2, 1),    # odd image, ragged N
]


def _w2(w):
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1).contiguous()


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_conv_fwd_exact(gpu, case):
    Nb, C, H, W, Cout, R, stride, pad = case
    g = torch.Generator().manual_seed(7)
    x = torch.randint(-2, 3, (Nb, C, H, W), generator=g).float()
    w = torch.randint(-2, 3, (Cout, C, R, R), generator=g).float()
    ref = F.conv2d(x, w, stride=stride, padding=pad)
    Ho, Wo = ref.shape[2], ref.shape[3]
    xd = x.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out = torch.empty(Nb * Ho * Wo, Cout, device=gpu, dtype=torch.bfloat16)
    assert native().conv_fwd_(xd, _w2(w.to(gpu, torch.bfloat16)), out, R, R, stride, pad)
    want = ref.permute(0, 2, 3, 1).reshape(-1, Cout).bfloat16().float()
    torch.testing.assert_close(out.float().cpu(), want, rtol=0, atol=0)


def test_conv_fwd_declines_unsupported(gpu):
    x = torch.zeros(2, 96, 8, 8, device=gpu, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w2 = torch.zeros(256, 9 * 96, device=gpu, dtype=torch.bfloat16)
    out = torch.empty(2 * 64, 256, device=gpu, dtype=torch.bfloat16)
    assert not native().conv_fwd_(x, w2, out, 3, 3, 1, 1)  # C not a power of two


@pytest.mark.parametrize("stride", [1, 2])
def test_convnhwc_module_matches_fp32(gpu, monkeypatch, stride):
    """ConvNHWC forward (implicit GEMM) and backward (stride 1: bwd-data on the same kernel with the
    flipped weights) vs an fp32 nn.Conv2d on the same bf16-rounded operands."""
    from parameter_server_distributed_amd.ops.conv import ConvNHWC

    monkeypatch.setenv("PSD_AUTOTUNE_FORCE", "igemm")
    torch.manual_seed(3)
    conv = ConvNHWC(256, 256, 3, stride).to(gpu, torch.bfloat16).to(memory_format=torch.channels_last)
    ref = torch.nn.Conv2d(256, 256, 3, stride=stride, padding=1, bias=False).to(gpu)
    ref.weight.data.copy_(conv.weight.float())
    x = torch.randn(8, 256, 14, 14, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xr = x.float().clone().requires_grad_(True)
    x.requires_grad_(True)
    y = conv(x)
    yr = ref(xr)
    torch.testing.assert_close(y.float(), yr.detach(), rtol=2e-2, atol=2e-2 * float(yr.abs().max()))
    gy = torch.randn_like(yr)
    y.backward(gy.to(torch.bfloat16))
    yr.backward(gy)
    gerr = (x.grad.float() - xr.grad).abs()
    gscale = float(xr.grad.abs().max())
    assert float(gerr.max()) < 0.1 * gscale, (float(gerr.max()), gscale)
    assert float(gerr.mean()) < 0.015 * gscale
    torch.testing.assert_close(conv.weight.grad.float(), ref.weight.grad, rtol=2e-2,
                               atol=2e-2 * float(ref.weight.grad.abs().max()))


def test_conv1x1_psd_route_matches_fp32(gpu, monkeypatch):
    """Conv1x1 with every route forced to the MFMA GEMM (fwd NT, dgrad NN, split-K wgrad TN)."""
    from parameter_server_distributed_amd.ops.conv import Conv1x1

    monkeypatch.setenv("PSD_AUTOTUNE_FORCE", "psd")
    torch.manual_seed(4)
    conv = Conv1x1(256, 512).to(gpu, torch.bfloat16).to(memory_format=torch.channels_last)
    ref = torch.nn.Conv2d(256, 512, 1, bias=False).to(gpu)
    ref.weight.data.copy_(conv.weight.float())
    x = torch.randn(16, 256, 14, 14, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xr = x.float().clone().requires_grad_(True)
    x.requires_grad_(True)
    y = conv(x)
    yr = ref(xr)
    torch.testing.assert_close(y.float(), yr.detach(), rtol=2e-2, atol=2e-2 * float(yr.abs().max()))
    gy = torch.randn_like(yr)
    y.backward(gy.to(torch.bfloat16))
    yr.backward(gy)
    gerr = (x.grad.float() - xr.grad).abs()
    gscale = float(xr.grad.abs().max())
    assert float(gerr.max()) < 0.1 * gscale, (float(gerr.max()), gscale)
    assert float(gerr.mean()) < 0.015 * gscale
    torch.testing.assert_close(conv.weight.grad.float(), ref.weight.grad, rtol=2e-2,
                               atol=2e-2 * float(ref.weight.grad.abs().max()))


# ---------------------------------------------------------------- fp8 (e4m3) implicit GEMM
F8_CASES = [  # Nb, C, H, W, Cout, R, stride, pad
    (4, 128, 14, 14, 256, 3, 1, 1),
    (8, 256, 28, 28, 512, 1, 2, 0),
    (64, 256, 14, 14, 256, 3, 1, 1),   # several tiles per persistent workgroup
    (9, 512, 7, 7, 264, 3, 2, 1),      # ragged M (144 rows) and N
]


@pytest.mark.parametrize("afmt", ["e4m3", "e5m2"])
@pytest.mark.parametrize("case", F8_CASES, ids=lambda c: "x".join(map(str, c)))
def test_conv_fwd_fp8_exact(gpu, case, afmt):
    """fp8 operands holding small integers (exact in e4m3 and e5m2, products exact in the fp32 MFMA
    accumulator) and power-of-two dequant scales: the kernel must equal the fp32 convolution. The
    e5m2 input is the bwd-data form (dY gathered by the implicit GEMM)."""
    Nb, C, H, W, Cout, R, stride, pad = case
    g = torch.Generator().manual_seed(11)
    x = torch.randint(-3, 4, (Nb, C, H, W), generator=g).float()
    w = torch.randint(-3, 4, (Cout, C, R, R), generator=g).float()
    ref = F.conv2d(x, w, stride=stride, padding=pad) * 0.25
    Ho, Wo = ref.shape[2], ref.shape[3]
    xq = x.to(gpu).contiguous(memory_format=torch.channels_last).to(
        torch.float8_e5m2 if afmt == "e5m2" else torch.float8_e4m3fn)
    wq = _w2(w.to(gpu)).to(torch.float8_e4m3fn)
    sx = torch.tensor([0.5], device=gpu)
    sw = torch.tensor([0.5], device=gpu)
    out = torch.empty(Nb * Ho * Wo, Cout, device=gpu, dtype=torch.bfloat16)
    assert xq.is_contiguous(memory_format=torch.channels_last)
    assert native().conv_fwd_fp8_(xq, wq, sx, sw, out, R, R, stride, pad)
    want = ref.permute(0, 2, 3, 1).reshape(-1, Cout).bfloat16().float()
    torch.testing.assert_close(out.float().cpu(), want, rtol=0, atol=0)


def test_conv_fwd_fp8_declines_small_c(gpu):
    xq = torch.zeros(2, 64, 8, 8, device=gpu).contiguous(memory_format=torch.channels_last).to(torch.float8_e4m3fn)
    wq = torch.zeros(256, 9 * 64, device=gpu).to(torch.float8_e4m3fn)
    one = torch.ones(1, device=gpu)
    out = torch.empty(2 * 64, 256, device=gpu, dtype=torch.bfloat16)
    assert not native().conv_fwd_fp8_(xq, wq, one, one, out, 3, 3, 1, 1)  # C < 128


@pytest.mark.parametrize("kind", ["3x3", "3x3s2", "1x1"])
def test_fp8_conv_modules_match_fp32(gpu, kind):
    """fp8 modules vs fp32 nn.Conv2d: forward (e4m3) and, for the stride-1 shapes, bwd-data (e5m2 dY
    x e4m3 W) within fp8 error (per-tensor scales); the weight gradient stays bf16 (as tight as the
    bf16 path)."""
    from parameter_server_distributed_amd.ops.conv import Conv1x1, ConvNHWC

    torch.manual_seed(5)
    k, stride = (1, 1) if kind == "1x1" else (3, 2 if kind.endswith("s2") else 1)
    conv = (Conv1x1(256, 512, fp8=True) if kind == "1x1" else ConvNHWC(256, 256, 3, stride, fp8=True))
    conv = conv.to(gpu, torch.bfloat16).to(memory_format=torch.channels_last)
    ref = torch.nn.Conv2d(256, conv.out_channels, k, stride=stride, padding=k // 2, bias=False).to(gpu)
    ref.weight.data.copy_(conv.weight.float())
    x = torch.randn(8, 256, 14, 14, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xr = x.float().clone().requires_grad_(True)
    x.requires_grad_(True)
    y = conv(x)
    yr = ref(xr)
    err = (y.float() - yr.detach()).abs()
    scale = float(yr.abs().max())
    assert float(err.max()) < 0.08 * scale, (float(err.max()), scale)
    assert float(err.mean()) < 0.01 * scale
    gy = torch.randn_like(yr)
    y.backward(gy.to(torch.bfloat16))
    yr.backward(gy)
    gerr = (x.grad.float() - xr.grad).abs()
    gscale = float(xr.grad.abs().max())
    assert float(gerr.max()) < 0.1 * gscale, (float(gerr.max()), gscale)
    assert float(gerr.mean()) < 0.015 * gscale
    torch.testing.assert_close(conv.weight.grad.float(), ref.weight.grad, rtol=2e-2,
                               atol=2e-2 * float(ref.weight.grad.abs().max()))


# ---------------------------------------------------------------- implicit-GEMM weight gradient
WG_CASES = [  # Nb, C, H, W, Cout, R, stride, pad
    (4, 64, 16, 16, 256, 3, 1, 1),
    (8, 128, 14, 14, 256, 3, 2, 1),
    (16, 256, 8, 8, 512, 1, 2, 0),
    (32, 256, 14, 14, 256, 3, 1, 1),   # long pixel reduction: several K-tiles per split
    (2, 128, 12, 12, 264, 3, 1, 1),    # ragged Cout
]


@pytest.mark.parametrize("case", WG_CASES, ids=lambda c: "x".join(map(str, c)))
def test_conv_wgrad_exact(gpu, case):
    """dW = dY^T . im2col(x) on the gathered-B split-K kernel vs the fp32 weight gradient, small
    integers (exact products, exact fp32 sums below 2^24)."""
    Nb, C, H, W, Cout, R, stride, pad = case
    g = torch.Generator().manual_seed(13)
    x = torch.randint(-2, 3, (Nb, C, H, W), generator=g).float()
    wt = torch.zeros(Cout, C, R, R, requires_grad=True)
    y = F.conv2d(x, wt, stride=stride, padding=pad)
    dy = torch.randint(-2, 3, y.shape, generator=g).float()
    y.backward(dy)
    ref = wt.grad.permute(0, 2, 3, 1).reshape(Cout, -1)  # OHWI
    out = torch.empty(Cout, R * R * C, device=gpu, dtype=torch.bfloat16)
    xd = x.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dyd = dy.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert native().conv_wgrad_(dyd, xd, out, R, R, stride, pad)
    torch.testing.assert_close(out.float().cpu(), ref.bfloat16().float(), rtol=0, atol=0)


def test_convnhwc_wgrad_route_matches_fp32(gpu, monkeypatch):
    """ConvNHWC with every route forced to the implicit-GEMM kernels, weight gradient included."""
    from parameter_server_distributed_amd.ops.conv import ConvNHWC

    monkeypatch.setenv("PSD_AUTOTUNE_FORCE", "igemm")
    torch.manual_seed(6)
    conv = ConvNHWC(128, 256, 3, 1).to(gpu, torch.bfloat16).to(memory_format=torch.channels_last)
    ref = torch.nn.Conv2d(128, 256, 3, padding=1, bias=False).to(gpu)
    ref.weight.data.copy_(conv.weight.float())
    x = torch.randn(8, 128, 14, 14, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xr = x.float().clone().requires_grad_(True)
    y = conv(x.requires_grad_(True))
    yr = ref(xr)
    gy = torch.randn_like(yr)
    y.backward(gy.to(torch.bfloat16))
    yr.backward(gy)
    assert conv.weight.grad.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(conv.weight.grad.float(), ref.weight.grad, rtol=2e-2,
                               atol=2e-2 * float(ref.weight.grad.abs().max()))
