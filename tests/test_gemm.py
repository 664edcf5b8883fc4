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
@pytest.mark.parametrize("shape", [(200, 136, 96), (2048, 2056, 512)], ids=["small", "big"])
def test_gemm_bias_act_epilogue(gpu, act, shape):
    M, N, K = shape
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
@pytest.mark.parametrize("shape", [(2048, 2048, 256), (2000, 2120, 320), (2304, 4096, 768), (8192, 768, 768),
                                   (3000, 1000, 512)],
                         ids=lambda s: "x".join(map(str, s)))
def test_gemm_256_tile_path_exact(gpu, a_k, b_k, shape):
    """Shapes large enough for the 8-phase kernel, 256x256 and 128x256 tiles (incl. ragged M/N)."""
    M, N, K = shape
    A, B, ref = _ops(M, N, K, a_k, b_k, gpu, seed=11)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    native().gemm_(A, B, a_k, b_k, out)
    torch.testing.assert_close(out.float().cpu(), ref.bfloat16().float(), rtol=0, atol=0)


@pytest.mark.parametrize("c_f32", [False, True], ids=["bf16", "f32"])
def test_gemm_256_long_k_exact(gpu, c_f32):
    """Many K-tiles through the 256x256 pipeline (staging wraps the LDS buffers many times)."""
    M, N, K = 2304, 2048, 4160
    A, B, ref = _ops(M, N, K, True, True, gpu, seed=13)
    out = torch.empty(M, N, dtype=torch.float32 if c_f32 else torch.bfloat16, device=gpu)
    native().gemm_(A, B, True, True, out)
    want = ref if c_f32 else ref.bfloat16().float()
    torch.testing.assert_close(out.float().cpu(), want, rtol=0, atol=0)


def test_gemm_256_splitk_exact(gpu):
    M, N, K = 2048, 2048, 16384
    A, B, ref = _ops(M, N, K, False, False, gpu, seed=12)
    out = torch.zeros(M, N, dtype=torch.float32, device=gpu)
    native().gemm_splitk_(A, B, False, False, out, False, 1.0, 0)
    torch.testing.assert_close(out.cpu(), ref, rtol=0, atol=0)


@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, False), (False, True)],
                         ids=["NT", "NN", "TN", "TT"])
@pytest.mark.parametrize("shape", [(8264, 2104, 320), (16384, 4096, 256), (4160, 8448, 576)],
                         ids=lambda s: "x".join(map(str, s)))
def test_gemm_persistent_multi_tile_exact(gpu, a_k, b_k, shape):
    """More tiles than CUs: each persistent workgroup runs several tiles back to back, the next tile's
    first K-tiles staged during the previous one (odd K-tile counts flip the LDS buffer parity at
    the seam; ragged M/N clamp rows of the NEXT tile's stages)."""
    M, N, K = shape
    A, B, ref = _ops(M, N, K, a_k, b_k, gpu, seed=17)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    native().gemm_(A, B, a_k, b_k, out)
    torch.testing.assert_close(out.float().cpu(), ref.bfloat16().float(), rtol=0, atol=0)


@pytest.mark.parametrize("act", [0, 1, 2], ids=["none", "relu", "gelu"])
def test_gemm_persistent_bias_act_epilogue(gpu, act):
    M, N, K = 8192, 3072, 256  # 384 tiles of 256x256: > 1 tile per workgroup
    A, B, ref = _ops(M, N, K, True, True, gpu, ints=False, seed=19)
    bias = torch.randn(N).to(torch.bfloat16)
    z = ref + bias.float()
    want = {0: z, 1: torch.relu(z), 2: torch.nn.functional.gelu(z, approximate="tanh")}[act]
    out = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=gpu) if act == 2 else None
    native().gemm_(A, B, True, True, out, bias.to(gpu), act, aux)
    torch.testing.assert_close(out.float().cpu(), want, rtol=2e-2, atol=2e-2)
    if aux is not None:
        torch.testing.assert_close(aux.float().cpu(), z, rtol=2e-2, atol=2e-2)


# ---------------------------------------------------------------- fp8 (OCP e4m3fn) forward GEMM
@pytest.mark.parametrize("shape", [(2048, 2048, 512), (300, 520, 256), (4096, 768, 3072), (8192, 8192, 256),
                                   (8320, 4352, 384)],
                         ids=lambda s: "x".join(map(str, s)))
def test_gemm_fp8_exact_small_ints(gpu, shape):
    """Small integers are exact in e4m3: the MX-scaled fp8 MFMA must reproduce the fp32 product."""
    M, N, K = shape
    g = torch.Generator().manual_seed(21)
    a = torch.randint(-3, 4, (M, K), generator=g).float()
    b = torch.randint(-3, 4, (N, K), generator=g).float()
    aq, bq = a.to(torch.float8_e4m3fn).to(gpu), b.to(torch.float8_e4m3fn).to(gpu)
    sa = torch.tensor([0.5], device=gpu)
    sb = torch.tensor([2.0], device=gpu)
    out = torch.empty(M, N, dtype=torch.float32, device=gpu)
    native().gemm_fp8_(aq, bq, sa, sb, out)
    torch.testing.assert_close(out.cpu(), a @ b.t(), rtol=0, atol=0)


@pytest.mark.parametrize("act", [0, 2], ids=["none", "gelu"])
def test_gemm_fp8_quantized_matches_dequant_reference(gpu, act):
    from parameter_server_distributed_amd.ops import quantize_fp8

    M, N, K = 1024, 1536, 768
    x = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    w = (torch.randn(N, K, device=gpu) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=gpu).to(torch.bfloat16)
    xq, sx = quantize_fp8(x)
    wq, sw = quantize_fp8(w)
    ref = (xq.float() * sx) @ (wq.float() * sw).t() + bias.float()
    if act == 2:
        ref = torch.nn.functional.gelu(ref, approximate="tanh")
    out = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    native().gemm_fp8_(xq, wq, sx, sw, out, bias, act)
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=1e-2)


def test_mfma_linear_fp8_forward_backward(gpu):
    from parameter_server_distributed_amd.ops.linear import MfmaLinear

    torch.manual_seed(0)
    lin = MfmaLinear(512, 384, act="gelu", fp8=True).to(gpu, torch.bfloat16)
    ref = torch.nn.Linear(512, 384).to(gpu)
    with torch.no_grad():
        ref.weight.copy_(lin.weight.float())
        ref.bias.copy_(lin.bias.float())
    x = torch.randn(256, 512, device=gpu)
    xb = x.to(torch.bfloat16).requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    y = lin(xb)
    yr = torch.nn.functional.gelu(ref(xr), approximate="tanh")
    rel = (y.float() - yr).norm() / yr.norm()
    assert rel < 0.06, rel  # e4m3 forward
    g = torch.randn_like(yr)
    y.backward(g.to(torch.bfloat16))
    yr.backward(g)
    relx = (xb.grad.float() - xr.grad).norm() / xr.grad.norm()
    relw = (lin.weight.grad.float() - ref.weight.grad).norm() / ref.weight.grad.norm()
    assert relx < 0.08 and relw < 0.08, (relx, relw)


@pytest.mark.parametrize("route", ["mfma", "mfma_ct", "blas"])
@pytest.mark.parametrize("act", [None, "relu", "gelu"])
def test_mfma_linear_routes_match_fp32(gpu, route, act):
    """Both per-shape routes of MfmaLinear (MFMA kernels / hipBLASLt + separate epilogue) against an
    fp32 nn.Linear: forward, dx, dW, db."""
    from parameter_server_distributed_amd.ops import autotune as at
    from parameter_server_distributed_amd.ops.linear import ACTS, MfmaLinear

    torch.manual_seed(0)
    M, K, N = 384, 256, 320
    lin = MfmaLinear(K, N, act=act).to(gpu, torch.bfloat16)
    ref = torch.nn.Linear(K, N).to(gpu)
    with torch.no_grad():
        ref.weight.copy_(lin.weight.float())
        ref.bias.copy_(lin.bias.float())
    keys = [("linear", "fwd", M, K, N, ACTS[act], True), ("linear", "dgrad", M, K, N), ("linear", "wgrad", M, K, N)]
    for k in keys:
        at.set_decision(k, route)
    try:
        x = torch.randn(M, K, device=gpu)
        xb = x.to(torch.bfloat16).requires_grad_(True)
        xr = x.to(torch.bfloat16).float().requires_grad_(True)
        y = lin(xb)
        yr = ref(xr)
        if act == "relu":
            yr = torch.relu(yr)
        elif act == "gelu":
            yr = torch.nn.functional.gelu(yr, approximate="tanh")
        g = torch.randn_like(yr)
        y.backward(g.to(torch.bfloat16))
        yr.backward(g.to(torch.bfloat16).float())
    finally:
        for k in keys:
            at.set_decision(k, None)
    for a, b in ((y, yr), (xb.grad, xr.grad), (lin.weight.grad, ref.weight.grad), (lin.bias.grad, ref.bias.grad)):
        rel = ((a.float() - b).norm() / b.norm()).item()
        assert rel < 2e-2, rel


def test_gelu_bwd_colsum_matches_torch(gpu):
    M, N = 3000, 776
    dy = torch.randn(M, N, device=gpu).to(torch.bfloat16)
    pre = (torch.randn(M, N, device=gpu) * 3).to(torch.bfloat16)
    dx = torch.empty_like(dy)
    db = torch.zeros(N, device=gpu)
    native().gelu_bwd_colsum_(dy, pre, dx, db, False)
    want = torch.ops.aten.gelu_backward(dy.float(), pre.float(), approximate="tanh")
    torch.testing.assert_close(dx.float(), want, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(db, dx.float().sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("b_k", [False, True], ids=["NN", "NT"])
@pytest.mark.parametrize("shape", [(2048, 3072, 768), (4000, 1024, 256)], ids=str)
def test_gemm_gelu_bwd_epilogue_matches_unfused(gpu, b_k, shape):
    """ACT 3: g = bf16(bf16(dY W) * gelu'(pre)) in the GEMM epilogue equals the GEMM followed by the
    separate GELU-backward + column-sum pass bit for bit; the bias gradient from the epilogue's
    per-tile partials matches that pass's column sums."""
    M, N, K = shape
    C = native()
    A, B, _ = _ops(M, N, K, True, b_k, gpu, ints=False, seed=3)
    pre = (torch.randn(M, N, device=gpu) * 2).to(torch.bfloat16)
    dx = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    C.gemm_(A, B, True, b_k, dx)
    g_ref = torch.empty_like(dx)
    db_ref = torch.zeros(N, device=gpu)
    C.gelu_bwd_colsum_(dx, pre, g_ref, db_ref, False)
    g = torch.full_like(dx, float("nan"))
    db = torch.full((N,), float("nan"), device=gpu)
    assert C.gemm_gelu_bwd_(A, B, True, b_k, pre, g, db)
    assert torch.equal(g, g_ref)
    # a shape off the 8-phase kernel (too few tiles) declines without launching
    small = torch.zeros(256, 256, dtype=torch.bfloat16, device=gpu)
    assert not C.gemm_gelu_bwd_(small, small, True, True, small, small.clone(), torch.zeros(256, device=gpu))
    torch.testing.assert_close(db, g.float().sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(db, db_ref, rtol=1e-5, atol=1e-3)


def test_ffn_gelu_handover_matches_unfused(gpu, monkeypatch):
    """BERT FFN pair with ffn2.psd_gelu_input_from(ffn1): ffn2's bwd-data GEMM returns d(pre) and
    ffn1's bias gradient; every gradient equals the unfused path (feature gelu_fuse off) and an fp32 reference."""
    from parameter_server_distributed_amd.ops import linear as L

    torch.manual_seed(1)
    M, H, F = 1024, 256, 1024
    f1 = L.MfmaLinear(H, F, act="gelu").to(gpu, torch.bfloat16)
    f2 = L.MfmaLinear(F, H).to(gpu, torch.bfloat16)
    f2.psd_gelu_input_from(f1)
    x0 = torch.randn(M, H, device=gpu).to(torch.bfloat16)
    gy = torch.randn(M, H, device=gpu).to(torch.bfloat16)
    calls = {"n": 0}
    real = L._gelu_dgrad

    def counted(*a, **k):
        calls["n"] += 1
        return real(*a, **k)

    monkeypatch.setattr(L, "_gelu_dgrad", counted)

    def run(fuse):
        monkeypatch.setenv("PSD_FEATURES", f"gelu_fuse={int(fuse)}")
        for p in list(f1.parameters()) + list(f2.parameters()):
            p.grad = None
        x = x0.clone().requires_grad_(True)
        f2(f1(x)).backward(gy)
        return [x.grad.clone()] + [p.grad.clone() for p in (f1.weight, f1.bias, f2.weight, f2.bias)]

    fused = run(True)
    assert calls["n"] == 1
    plain = run(False)
    assert calls["n"] == 1
    for a, b in zip(fused, plain):
        torch.testing.assert_close(a.float(), b.float(), rtol=1e-2, atol=1e-2)
    # fp32 reference
    xr = x0.float().requires_grad_(True)
    w1, b1, w2, b2 = (t.detach().float().requires_grad_(True) for t in (f1.weight, f1.bias, f2.weight, f2.bias))
    yr = torch.nn.functional.linear(torch.nn.functional.gelu(torch.nn.functional.linear(xr, w1, b1), approximate="tanh"), w2, b2)
    yr.backward(gy.float())
    for a, b in zip(fused, (xr.grad, w1.grad, b1.grad, w2.grad, b2.grad)):
        rel = ((a.float() - b).norm() / b.norm()).item()
        assert rel < 2e-2, rel


# ---------------------------------------------------------------- 192 x 256 tiles stored transposed
# (gemm_ct_: Y[N, M] = B A^T + bias[M]; the 768-wide BERT GEMMs as 512 tiles instead of 384 256-tiles)
CT_SHAPES = [(192, 256, 128), (200, 1000, 192), (768, 4096, 768), (2304, 2048, 256), (768, 520, 3072),
             (392, 33000, 128)]


@pytest.mark.parametrize("shape", CT_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_gemm_ct_exact(gpu, shape):
    """Small-integer operands: exact in fp32 out, every tile edge (M past 192-multiples, N past 256)."""
    M, N, K = shape
    g = torch.Generator().manual_seed(7)
    a = torch.randint(-3, 4, (M, K), generator=g).float().to(torch.bfloat16)
    b = torch.randint(-3, 4, (N, K), generator=g).float().to(torch.bfloat16)
    ref = b.float() @ a.float().t()
    out = torch.full((N, M), 7.0, dtype=torch.float32, device=gpu)
    assert native().gemm_ct_(a.to(gpu), b.to(gpu), out)
    torch.testing.assert_close(out.cpu(), ref, rtol=0, atol=0)


@pytest.mark.parametrize("act", [0, 1, 2], ids=["none", "relu", "gelu"])
@pytest.mark.parametrize("shape", [(768, 32768, 768), (2304, 4096, 768), (200, 1000, 192)], ids=str)
def test_gemm_ct_bias_act_vs_fp32(gpu, act, shape):
    """Random-normal operands: bias per output column of Y, ReLU / GELU and the GELU pre-activation,
    bf16 out, against the fp32 reference of the same op (F.linear)."""
    M, N, K = shape
    g = torch.Generator().manual_seed(11)
    w = torch.randn(M, K, generator=g).to(torch.bfloat16)
    x = torch.randn(N, K, generator=g).to(torch.bfloat16)
    bias = torch.randn(M, generator=g).to(torch.bfloat16)
    z = torch.nn.functional.linear(x.float(), w.float(), bias.float())
    want = {0: z, 1: torch.relu(z), 2: torch.nn.functional.gelu(z, approximate="tanh")}[act]
    out = torch.empty(N, M, dtype=torch.bfloat16, device=gpu)
    aux = torch.empty(N, M, dtype=torch.bfloat16, device=gpu) if act == 2 else None
    assert native().gemm_ct_(w.to(gpu), x.to(gpu), out, bias.to(gpu), act, aux)
    torch.testing.assert_close(out.float().cpu(), want, rtol=2e-2, atol=2e-2)
    if aux is not None:
        torch.testing.assert_close(aux.float().cpu(), z, rtol=2e-2, atol=2e-2)


def test_gemm_ct_declines_outside_contract(gpu):
    C = native()
    a = torch.zeros(100, 128, dtype=torch.bfloat16, device=gpu)  # M % 8 != 0
    b = torch.zeros(256, 128, dtype=torch.bfloat16, device=gpu)
    assert not C.gemm_ct_(a, b, torch.empty(256, 100, dtype=torch.bfloat16, device=gpu))
    a = torch.zeros(192, 96, dtype=torch.bfloat16, device=gpu)  # K % 64 != 0
    assert not C.gemm_ct_(a, torch.zeros(256, 96, dtype=torch.bfloat16, device=gpu),
                          torch.empty(256, 192, dtype=torch.bfloat16, device=gpu))


@pytest.mark.parametrize("shape", [(2304, 768, 8192), (768, 3072, 4096), (520, 1000, 2056)], ids=str)
def test_gemm_splitk_bcontig_bitwise(gpu, shape):
    """The split-K GEMM with an N-major B staged as contiguous 128-column halves against the
    quadrant-interleaved halves (default): the same K order per output, so bitwise equal; and exact
    against fp32 on small integers."""
    M, N, K = shape
    C = native()
    g = torch.Generator().manual_seed(13)
    a = torch.randint(-3, 4, (K, M), generator=g).float().to(torch.bfloat16).to(gpu)
    b = torch.randint(-3, 4, (K, N), generator=g).float().to(torch.bfloat16).to(gpu)
    outs = []
    for bc in (True, False):
        out = torch.empty(M, N, dtype=torch.float32, device=gpu)
        C.gemm_set_bcontig(bc)
        try:
            C.gemm_splitk_(a, b, False, False, out, False, 1.0, 0)
        finally:
            C.gemm_set_bcontig(False)
        outs.append(out.cpu())
    assert torch.equal(outs[0], outs[1])
    torch.testing.assert_close(outs[0], a.float().cpu().t() @ b.float().cpu(), rtol=0, atol=0)


@pytest.mark.parametrize("out_f32", [True, False], ids=["f32", "bf16"])
def test_gemm_splitk_single_split_direct(gpu, out_f32):
    """A split-K GEMM whose shape gets one split (192 256-tiles: the chip is full without splitting)
    runs as the single-split GEMM writing the output itself (no slab / reduce): exact on small
    integers in TN layout, and the accumulate path (slab + reduce) still adds."""
    M, N, K = 4096, 3072, 4096
    C = native()
    g = torch.Generator().manual_seed(23)
    a = torch.randint(-2, 3, (K, M), generator=g).float()
    b = torch.randint(-2, 3, (K, N), generator=g).float()
    ref = a.t() @ b
    dt = torch.float32 if out_f32 else torch.bfloat16
    out = torch.empty(M, N, dtype=dt, device=gpu)
    C.gemm_splitk_(a.to(torch.bfloat16).to(gpu), b.to(torch.bfloat16).to(gpu), False, False, out, False, 1.0, 0)
    torch.testing.assert_close(out.float().cpu(), ref if out_f32 else ref.bfloat16().float(), rtol=0, atol=0)
    acc = torch.full((M, N), 2.0, dtype=torch.float32, device=gpu)
    C.gemm_splitk_(a.to(torch.bfloat16).to(gpu), b.to(torch.bfloat16).to(gpu), False, False, acc, True, 1.0, 0)
    torch.testing.assert_close(acc.cpu(), ref + 2.0, rtol=0, atol=0)
