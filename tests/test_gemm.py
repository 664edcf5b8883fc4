"""MFMA bf16 GEMM (kernels/gemm.hip) vs PyTorch fp32, every operand layout, epilogue and split-K.

Exact small-integer operands first (a swapped fragment/C-layout shows up as a hard mismatch, and
asymmetric data catches transposes -- cdna_hip_programming.md §3), then random-normal data.
"""
import pytest
import torch

from parameter_server_distributed_amd import native

pytestmark = pytest.mark.gpu

SHAPES = [(128, 128, 64), (256, 192, 128), (104, 72, 136), (64, 64, 64), (520, 40, 72), (48, 264, 2056)]


def _ops(M, N, K, a_k, b_k, dev, ints=True, seed=0):
    g = torch.Generator().manual_seed(seed)
    if ints:
        a = torch.randint(-3, 4, (M, K), generator=g).float()
        b = torch.randint(-3, 4, (K, N), generator=g).float()
    else:
        a = torch.randn(M, K, generator=g)
        b = torch.randn(K, N, generator=g)
    a16, b16 = a.to(torch.bfloat16), b.to(torch.bfloat16)
    A = (a16 if a_k else a16.t()).contiguous().to(dev)  # a_k: [M,K]; else [K,M]
    B = (b16.t() if b_k else b16).contiguous().to(dev)  # b_k: [N,K]; else [K,N]
    return A, B, a16.float() @ b16.float()


@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, False), (False, True)],
                         ids=["NT", "NN", "TN", "TT"])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_gemm_layouts_exact(gpu, a_k, b_k, shape):
    M, N, K = shape
    if (not a_k and M % 8) or (not b_k and N % 8):
        pytest.skip("MN-major operand needs a multiple of 8")
    A, B, ref = _ops(M, N, K, a_k, b_k, gpu)
    out = torch.empty(M, N, dtype=torch.float32, device=gpu)
    native().gemm_(A, B, a_k, b_k, out)
    torch.testing.assert_close(out.cpu(), ref, rtol=0, atol=0)


@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, False)], ids=["NT", "NN", "TN"])
@pytest.mark.parametrize("shape", [(64, 96, 4096), (256, 64, 12544), (136, 256, 520)], ids=str)
def test_gemm_splitk_exact(gpu, a_k, b_k, shape):
    M, N, K = shape
    A, B, ref = _ops(M, N, K, a_k, b_k, gpu, seed=3)
    out = torch.full((M, N), 5.0, dtype=torch.float32, device=gpu)
    native().gemm_splitk_(A, B, a_k, b_k, out, True, 1.0, 0)
    torch.testing.assert_close(out.cpu(), ref + 5.0, rtol=0, atol=0)
    outb = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    native().gemm_splitk_(A, B, a_k, b_k, outb, False, 0.5, 0)
    torch.testing.assert_close(outb.float().cpu(), (ref * 0.5).bfloat16().float(), rtol=0, atol=0)


@pytest.mark.parametrize("act", [0, 1, 2], ids=["none", "relu", "gelu"])
def test_gemm_bias_act_epilogue(gpu, act):
    M, N, K = 200, 136, 96
    A, B, ref = _ops(M, N, K, True, True, gpu, ints=False, seed=5)
    bias = torch.randn(N).to(torch.bfloat16)
    z = ref + bias.float()
    want = {0: z, 1: torch.relu(z), 2: torch.nn.functional.gelu(z, approximate="tanh")}[act]
    out = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=gpu) if act == 2 else None
    native().gemm_(A, B, True, True, out, bias.to(gpu), act, aux)
    torch.testing.assert_close(out.float().cpu(), want, rtol=2e-2, atol=2e-2)
    if aux is not None:
        torch.testing.assert_close(aux.float().cpu(), z, rtol=2e-2, atol=2e-2)


def test_colsum(gpu):
    x = torch.randn(1000, 136).to(torch.bfloat16)
    out = torch.ones(136, dtype=torch.bfloat16, device=gpu)
    native().colsum_(x.to(gpu), out, True)
    torch.testing.assert_close(out.float().cpu(), (x.float().sum(0) + 1).bfloat16().float(), rtol=1e-2, atol=5e-2)
    o32 = torch.zeros(136, device=gpu)
    native().colsum_(x.to(gpu), o32, False)
    torch.testing.assert_close(o32.cpu(), x.float().sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("shape", [(8192, 768), (8192, 3072), (8192, 4096), (37, 2056), (100000, 64)],
                         ids=lambda s: "x".join(map(str, s)))
def test_colsum_shapes_deterministic(gpu, shape):
    x = torch.randn(*shape, device=gpu).to(torch.bfloat16)
    o1 = torch.zeros(shape[1], device=gpu)
    o2 = torch.zeros(shape[1], device=gpu)
    native().colsum_(x, o1, False)
    native().colsum_(x, o2, False)
    assert torch.equal(o1, o2)
    torch.testing.assert_close(o1.cpu(), x.float().sum(0).cpu(), rtol=1e-4, atol=2e-3)


@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, False), (False, True)],
                         ids=["NT", "NN", "TN", "TT"])
@pytest.mark.parametrize("shape", [(2048, 2048, 256), (2000, 2120, 320), (2304, 4096, 768)],
                         ids=lambda s: "x".join(map(str, s)))
def test_gemm_256_tile_path_exact(gpu, a_k, b_k, shape):
    """Shapes large enough for the 256x256 global_load_lds kernel (incl. ragged M/N edges)."""
    M, N, K = shape
    A, B, ref = _ops(M, N, K, a_k, b_k, gpu, seed=11)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    native().gemm_(A, B, a_k, b_k, out)
    torch.testing.assert_close(out.float().cpu(), ref.bfloat16().float(), rtol=0, atol=0)


def test_gemm_256_splitk_exact(gpu):
    M, N, K = 2048, 2048, 16384
    A, B, ref = _ops(M, N, K, False, False, gpu, seed=12)
    out = torch.zeros(M, N, dtype=torch.float32, device=gpu)
    native().gemm_splitk_(A, B, False, False, out, False, 1.0, 0)
    torch.testing.assert_close(out.cpu(), ref, rtol=0, atol=0)
