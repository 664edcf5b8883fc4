"""Large-tensor correctness: the gfx950 kernels on NHWC activations past 2^31
bytes -- the range a b2048 ResNet-50 reaches in layer1 (3.3 GB per 256-channel activation) -- vs
a chunked fp32 PyTorch reference. The kernels address their operands through 32-bit buffer
descriptors and int offsets; these tensors exercise the top half of that range (the launchers
decline operands of 4 GiB and more: tests/test_convn.py, test_conv_igemm.py)."""
import pytest
import torch
import torch.nn.functional as F

from parameter_server_distributed_amd import native

pytestmark = pytest.mark.gpu

GB = 1 << 30


def _chunks(n, step):
    for i in range(0, n, step):
        yield i, min(n, i + step)


def test_bn_fwd_bwd_past_2gib(gpu):
    """BN forward (reduce + finalize + apply with ReLU) and backward (reduce + elementwise) on a
    [M, 128] bf16 activation of 2.2 GB, against fp64 statistics and an fp32 chunked reference."""
    torch.manual_seed(0)
    M, C = 8_650_752, 128  # 2.2e9 bytes
    x = torch.empty(M, C, device=gpu, dtype=torch.bfloat16)
    for a, b in _chunks(M, 1 << 20):
        x[a:b] = (torch.randn(b - a, C, device=gpu) * 0.5 + 0.25).to(torch.bfloat16)
    assert x.numel() * 2 > 2 * GB
    g = (torch.rand(C, device=gpu) + 0.5).to(torch.bfloat16)
    bt = (torch.randn(C, device=gpu) * 0.1).to(torch.bfloat16)
    rm, rv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    y, mean, invstd, ss, _ = native().bn_fwd(x, g, bt, rm, rv, None, True, True, 0.1, 1e-5, None, None)
    s1 = torch.zeros(C, dtype=torch.float64, device=gpu)
    s2 = torch.zeros(C, dtype=torch.float64, device=gpu)
    for a, b in _chunks(M, 1 << 20):
        xf = x[a:b].double()
        s1 += xf.sum(0)
        s2 += (xf * xf).sum(0)
    mu = s1 / M
    var = s2 / M - mu * mu
    torch.testing.assert_close(mean.double(), mu, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(invstd.double(), torch.rsqrt(var + 1e-5), rtol=1e-4, atol=1e-5)
    sc, sh = (g.double() * torch.rsqrt(var + 1e-5)), None
    sh = bt.double() - mu * sc
    for a, b in ((0, 1 << 16), (M // 2, M // 2 + (1 << 16)), (M - (1 << 16), M)):  # head, middle, tail
        ref = torch.relu(x[a:b].double() * sc + sh)
        torch.testing.assert_close(y[a:b].double(), ref, rtol=1e-2, atol=2e-2)
    del y
    dy = torch.empty_like(x)
    for a, b in _chunks(M, 1 << 20):
        dy[a:b] = torch.randn(b - a, C, device=gpu).to(torch.bfloat16)
    dx, _, dg, db = native().bn_bwd(dy, x, None, g, mean, invstd, True, False, None, None, None, ss, None)
    # reference: dz = dy * mask; dx = g*invstd*(dz - mean(dz) - xhat*mean(dz*xhat))
    sz = torch.zeros(C, dtype=torch.float64, device=gpu)
    szx = torch.zeros(C, dtype=torch.float64, device=gpu)
    inv = invstd.double()
    for a, b in _chunks(M, 1 << 20):
        xh = (x[a:b].double() - mean.double()) * inv
        z = dy[a:b].double() * ((x[a:b].double() * sc + sh) > 0)
        sz += z.sum(0)
        szx += (z * xh).sum(0)
    torch.testing.assert_close(db.double(), sz, rtol=2e-2, atol=1.0)
    torch.testing.assert_close(dg.double(), szx, rtol=2e-2, atol=1.0)
    for a, b in ((0, 1 << 16), (M - (1 << 16), M)):
        xh = (x[a:b].double() - mean.double()) * inv
        z = dy[a:b].double() * ((x[a:b].double() * sc + sh) > 0)
        ref = g.double() * inv * (z - sz / M - xh * szx / M)
        torch.testing.assert_close(dx[a:b].double(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("kernel", ["convn", "conv_fwd"])
def test_implicit_gemm_conv_input_past_2gib(gpu, kernel):
    """Implicit-GEMM convolution whose NHWC input is 2.2 GB (256 channels): the narrow kernel
    (1x1 -> 64) and the 8-phase kernel (3x3 -> 256), checked against F.conv2d on image chunks at
    the head, middle and tail of the batch (exact small-integer operands)."""
    Nb, C, H, W = 1056, 256, 64, 64  # 1056*64*64*256*2 = 2.2e9 bytes
    cout, k = (64, 1) if kernel == "convn" else (256, 3)
    x = torch.empty(Nb, C, H, W, device=gpu, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gen = torch.Generator(device=gpu).manual_seed(1)
    for a, b in _chunks(Nb, 64):
        x[a:b] = torch.randint(-2, 3, (b - a, C, H, W), device=gpu, generator=gen).to(torch.bfloat16)
    assert x.numel() * 2 > 2 * GB
    w = torch.randint(-1, 2, (cout, C, k, k), device=gpu, generator=gen).to(torch.bfloat16)
    w2 = w.permute(0, 2, 3, 1).reshape(cout, -1).contiguous()
    out = torch.empty(Nb * H * W, cout, device=gpu, dtype=torch.bfloat16)
    if kernel == "convn":
        assert native().convn_(x, w2, out, k, k, 1, k // 2) >= 1
    else:
        assert native().conv_fwd_(x, w2, out, k, k, 1, k // 2)
    o4 = out.view(Nb, H, W, cout)
    for a, b in ((0, 8), (Nb // 2, Nb // 2 + 8), (Nb - 8, Nb)):
        ref = F.conv2d(x[a:b].float(), w.float(), padding=k // 2)
        torch.testing.assert_close(o4[a:b].float(), ref.permute(0, 2, 3, 1).bfloat16().float(), rtol=0, atol=0)
