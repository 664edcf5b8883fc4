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
    assert native().conv_fwd_(x, w2, out, 3, 3, 1, 1) is False  # C not a power of two
