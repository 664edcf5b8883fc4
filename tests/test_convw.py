"""Narrow implicit-GEMM weight gradient (kernels/convw.hip) vs the PyTorch fp32 weight gradient of
``F.conv2d``.

Operands are small integers, so every per-split partial and the slab sum are exact fp32 integers
and the bf16 result must equal the rounded fp32 reference bit for bit: a wrong gathered pixel, a
missed zero pad, a swapped (r, s), a transposed fragment or a dropped split is a hard mismatch."""
import pytest
import torch
import torch.nn.functional as F

from parameter_server_distributed_amd import native

pytestmark = pytest.mark.gpu

CASES = [  # Nb, C, H, W, Cout, R, stride, pad
    (4, 256, 14, 14, 64, 1, 1, 0),     # layer1 conv1 family: 1x1 256 -> 64
    (3, 64, 15, 13, 256, 1, 1, 0),     # layer1 conv3: 1x1 64 -> 256, ragged M (585 px)
    (4, 64, 14, 14, 64, 3, 1, 1),      # layer1 conv2: 3x3 64 -> 64 (KK = 576: TKK 192 / 64)
    (3, 128, 14, 14, 128, 3, 1, 1),    # layer2 conv2
    (4, 128, 28, 28, 128, 3, 2, 1),    # strided 3x3
    (2, 512, 7, 9, 128, 1, 1, 0),      # 1x1 512 -> 128 (two column tiles)
    (2, 128, 7, 9, 512, 1, 1, 0),      # 1x1 128 -> 512 (two row tiles)
    (2, 256, 14, 14, 512, 1, 2, 0),    # strided 1x1 (downsample)
    (1, 64, 5, 5, 64, 3, 1, 1),        # M = 25 < one stage
]


def _case(case, gpu, seed=11):
    Nb, C, H, W, Cout, R, stride, pad = case
    g = torch.Generator().manual_seed(seed)
    x = torch.randint(-2, 3, (Nb, C, H, W), generator=g).float()
    Ho, Wo = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - R) // stride + 1
    dy = torch.randint(-2, 3, (Nb, Cout, Ho, Wo), generator=g).float()
    ref = torch.nn.grad.conv2d_weight(x, (Cout, C, R, R), dy, stride=stride, padding=pad)
    cl = torch.channels_last
    return (x.to(gpu, torch.bfloat16).contiguous(memory_format=cl), dy.to(gpu, torch.bfloat16).contiguous(memory_format=cl),
            ref)


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_convw_exact(gpu, case):
    """Every tile variant, exact against the fp32 weight gradient (OHWI result layout)."""
    Nb, C, H, W, Cout, R, stride, pad = case
    xd, dyd, ref = _case(case, gpu)
    want = ref.permute(0, 2, 3, 1).reshape(Cout, -1).bfloat16().float()
    nv = native().convw_variants(Cout, R * R * C)
    assert nv >= 1
    for v in range(nv):
        out = torch.full((Cout, R * R * C), 7.0, device=gpu, dtype=torch.bfloat16)
        assert native().convw_(dyd, xd, out, R, R, stride, pad, variant=v)
        torch.testing.assert_close(out.float().cpu(), want, rtol=0, atol=0, msg=lambda m: f"variant {v}: {m}")


def test_convw_accumulate(gpu):
    """accumulate=True adds the gradient to what the output held (the PS gradient sink)."""
    case = CASES[0]
    Nb, C, H, W, Cout, R, stride, pad = case
    xd, dyd, ref = _case(case, gpu)
    want = ref.permute(0, 2, 3, 1).reshape(Cout, -1) + 3.0
    out = torch.full((Cout, R * R * C), 3.0, device=gpu, dtype=torch.bfloat16)
    assert native().convw_(dyd, xd, out, R, R, stride, pad, accumulate=True)
    torch.testing.assert_close(out.float().cpu(), want.bfloat16().float(), rtol=0, atol=0)


def test_convw_random_bf16(gpu):
    """Gaussian bf16 operands at a layer1-like size: relative error of an fp32-accumulated bf16
    result against the fp32 reference."""
    torch.manual_seed(0)
    x = torch.randn(8, 64, 56, 56, device=gpu).bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn(8, 64, 56, 56, device=gpu).bfloat16().contiguous(memory_format=torch.channels_last)
    ref = torch.nn.grad.conv2d_weight(x.float(), (64, 64, 3, 3), dy.float(), padding=1)
    for v in range(native().convw_variants(64, 576)):  # incl. the persistent HALO variant (the last)
        out = torch.empty(64, 576, device=gpu, dtype=torch.bfloat16)
        assert native().convw_(dy, x, out, 3, 3, 1, 1, variant=v)
        got = out.float().view(64, 3, 3, 64).permute(0, 3, 1, 2)
        err = (got - ref).norm() / ref.norm()
        assert err < 4e-3, (v, err)


def test_convw_declines(gpu):
    """Shapes outside the contract return False (C not a power of two >= 64, Cout not 64/128/256k)."""
    x = torch.zeros(1, 48, 8, 8, device=gpu, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.zeros(1, 64, 8, 8, device=gpu, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert not native().convw_(dy, x, torch.empty(64, 48, device=gpu, dtype=torch.bfloat16), 1, 1, 1, 0)
    x = torch.zeros(1, 64, 8, 8, device=gpu, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.zeros(1, 96, 8, 8, device=gpu, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert not native().convw_(dy, x, torch.empty(96, 64, device=gpu, dtype=torch.bfloat16), 1, 1, 1, 0)
