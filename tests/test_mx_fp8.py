"""MX (OCP microscaling) fp8 on gfx950: quantisation with one E8M0 scale per 32 contiguous elements
(kernels/fp8.hip quant_mx_kernel) and the block-scaled MFMA GEMM / implicit-GEMM convolution
(kernels/gemm.hip gemm8p_kernel<..., MX>), against fp32 PyTorch references of the same ops on the
dequantised operands (so only accumulation order differs). The lane map the kernel relies on is
pinned by tools/probes/mx_probe.hip."""
import pytest
import torch
import torch.nn.functional as F

from parameter_server_distributed_amd.ops import dequantize_mx_ref, quantize_mx, quantize_mx_ref

pytestmark = pytest.mark.gpu


def _blocky(shape, gen, device):
    """Random data whose 32-element blocks span ~2^-12 .. 2^12 in magnitude (per-tensor scaling
    would flush the small blocks; block scaling keeps every block at full e4m3 precision)."""
    x = torch.randn(*shape, generator=gen, device=device)
    flat = x.view(-1, 32)
    flat *= torch.exp2(torch.randint(-12, 13, (flat.shape[0], 1), generator=gen, device=device).float())
    return x


@pytest.mark.parametrize("e5m2", [False, True])
def test_quant_mx_matches_reference(gpu, e5m2):
    gen = torch.Generator(device=gpu).manual_seed(0)
    x = _blocky((4096, 256), gen, gpu).to(torch.bfloat16)
    q, s = quantize_mx(x, e5m2=e5m2)
    qr, sr = quantize_mx_ref(x, e5m2=e5m2)
    assert torch.equal(s, sr)
    assert (q.view(torch.uint8) != qr.view(torch.uint8)).float().mean().item() < 1e-4
    if not e5m2:
        back = torch.empty_like(x, dtype=torch.float32)
        from parameter_server_distributed_amd import native

        native().dequant_mx_(q, s, back)
        torch.testing.assert_close(back, dequantize_mx_ref(q, s), rtol=0, atol=0)
        # e4m3 (3 mantissa bits) in every block: |err| <= 2^-4 |x| + half a subnormal step of the block
        blk = torch.exp2(s.float() - 127.0).repeat_interleave(32).view(x.shape)
        err = (back - x.float()).abs()
        assert bool((err <= 2.0 ** -4 * x.float().abs() + 2.0 ** -10 * blk).all())


@pytest.mark.parametrize("M,N,K", [(512, 256, 256), (640, 512, 1024), (1000, 384, 512)])
@pytest.mark.parametrize("e5m2", [False, True])
def test_gemm_mx_matches_dequantised_reference(gpu, M, N, K, e5m2):
    from parameter_server_distributed_amd import native

    gen = torch.Generator(device=gpu).manual_seed(M + N + K)
    a = _blocky((M, K), gen, gpu).to(torch.bfloat16)
    b = _blocky((N, K), gen, gpu).to(torch.bfloat16)
    aq, asc = quantize_mx(a, e5m2=e5m2)
    bq, bsc = quantize_mx(b)
    out = torch.empty(M, N, device=gpu, dtype=torch.float32)
    native().gemm_fp8_(aq, bq, asc, bsc, out)
    ref = dequantize_mx_ref(aq, asc) @ dequantize_mx_ref(bq, bsc).t()
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4 * ref.abs().max().item())


def test_gemm_mx_bf16_out_relu(gpu):
    from parameter_server_distributed_amd import native

    gen = torch.Generator(device=gpu).manual_seed(3)
    M, N, K = 768, 512, 512
    a = torch.randn(M, K, generator=gen, device=gpu).to(torch.bfloat16)
    b = torch.randn(N, K, generator=gen, device=gpu).to(torch.bfloat16)
    aq, asc = quantize_mx(a)
    bq, bsc = quantize_mx(b)
    out = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    native().gemm_fp8_(aq, bq, asc, bsc, out, act=1)
    ref = torch.relu(dequantize_mx_ref(aq, asc) @ dequantize_mx_ref(bq, bsc).t())
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("k,stride,cin,cout", [(3, 1, 128, 256), (3, 2, 256, 256), (1, 1, 256, 512)])
def test_conv_mx_matches_dequantised_reference(gpu, k, stride, cin, cout):
    from parameter_server_distributed_amd import native

    gen = torch.Generator(device=gpu).manual_seed(k * 100 + cin)
    nb, h = 8, 14
    x = _blocky((nb, h, h, cin), gen, gpu).to(torch.bfloat16)  # NHWC storage
    w = (torch.randn(cout, k, k, cin, generator=gen, device=gpu) * 0.05).to(torch.bfloat16)  # OHWI
    xq, xs = quantize_mx(x)
    wq, ws = quantize_mx(w)
    pad = k // 2
    ho = (h + 2 * pad - k) // stride + 1
    out = torch.empty(nb * ho * ho, cout, device=gpu, dtype=torch.bfloat16)
    x4 = xq.permute(0, 3, 1, 2)  # channels_last view
    assert native().conv_fwd_fp8_(x4, wq.view(cout, -1), xs, ws, out, k, k, stride, pad)
    xd = dequantize_mx_ref(xq, xs).permute(0, 3, 1, 2)
    wd = dequantize_mx_ref(wq, ws).permute(0, 3, 1, 2)
    ref = F.conv2d(xd, wd, stride=stride, padding=pad).permute(0, 2, 3, 1).reshape(-1, cout)
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
