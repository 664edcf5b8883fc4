"""Numerics of the gfx950 kernels (GPU) and their C++ host twins (CPU) against plain PyTorch fp32.

Every kernel test runs twice: on the CPU path (always) and on cuda:0 (``-m gpu``, MI355X).
"""
import pytest
import torch

from parameter_server_distributed_amd.ops import (OptimConfig, OptimDyn, dequantize_fp8, fused_apply_,
                                                  multi_reduce_, pack_cast_, quantize_fp8)

DEVICES = [pytest.param("cpu", id="cpu"), pytest.param("cuda", id="gpu", marks=pytest.mark.gpu)]


def _dev(name):
    if name == "cuda":
        if not torch.cuda.is_available():
            pytest.fail("GPU test selected but no GPU visible")
        return torch.device("cuda", 0)
    return torch.device("cpu")


def _torch_opt(cfg: OptimConfig, p):
    if cfg.kind in ("sgd", "momentum"):
        return torch.optim.SGD([p], lr=cfg.lr, momentum=cfg.momentum if cfg.kind == "momentum" else 0.0,
                               dampening=cfg.dampening, nesterov=cfg.nesterov, weight_decay=cfg.weight_decay,
                               maximize=cfg.maximize)
    cls = torch.optim.Adam if cfg.kind == "adam" else torch.optim.AdamW
    return cls([p], lr=cfg.lr, betas=(cfg.beta1, cfg.beta2), eps=cfg.eps, weight_decay=cfg.weight_decay,
               maximize=cfg.maximize, foreach=False)


CFGS = [
    OptimConfig("sgd", lr=1.0, momentum=0.0),  # the reference's p -= g (src/parameter_server.cpp:87)
    OptimConfig("sgd", lr=0.1, momentum=0.0, weight_decay=1e-2),
    OptimConfig("momentum", lr=0.05, momentum=0.9),
    OptimConfig("momentum", lr=0.05, momentum=0.9, nesterov=True, weight_decay=1e-3),
    OptimConfig("momentum", lr=0.05, momentum=0.8, dampening=0.1),
    OptimConfig("adam", lr=1e-3, weight_decay=1e-2),
    OptimConfig("adamw", lr=1e-3, weight_decay=1e-2),
    OptimConfig("adam", lr=1e-3, maximize=True),
]


@pytest.mark.parametrize("devname", DEVICES)
@pytest.mark.parametrize("cfg", CFGS, ids=lambda c: f"{c.kind}-wd{c.weight_decay}-n{int(c.nesterov)}")
@pytest.mark.parametrize("gdtype", [torch.float32, torch.bfloat16], ids=["g32", "g16"])
@pytest.mark.parametrize("nsrc", [1, 3])
def test_fused_apply_matches_torch_optim(devname, cfg, gdtype, nsrc):
    dev = _dev(devname)
    g = torch.Generator().manual_seed(7)
    n = 4096 * 3 + 5  # exercises the 8-wide vector body and the scalar tail
    p0 = torch.randn(n, generator=g)
    ref = p0.clone().requires_grad_(True)
    opt = _torch_opt(cfg, ref)
    master = p0.clone().to(dev)
    s1 = torch.zeros(n, device=dev) if cfg.num_states >= 1 else None
    s2 = torch.zeros(n, device=dev) if cfg.num_states >= 2 else None
    shadow = torch.empty(n, dtype=torch.bfloat16, device=dev)
    dyn = OptimDyn(dev, lr=cfg.lr, grad_scale=1.0 / nsrc)
    for step in range(4):
        srcs = [torch.randn(n, generator=g).to(gdtype) for _ in range(nsrc)]
        gsum = sum(s.float() for s in srcs) * (1.0 / nsrc)
        ref.grad = gsum.clone()
        opt.step()
        fused_apply_(cfg, dyn, master, [s.to(dev) for s in srcs], s1, s2, shadow)
    tol = 2e-5 if cfg.kind in ("sgd", "momentum") else 1e-4
    torch.testing.assert_close(master.cpu(), ref.detach(), rtol=tol, atol=tol)
    torch.testing.assert_close(shadow.cpu(), master.cpu().to(torch.bfloat16), rtol=0, atol=0)
    assert dyn.step == 4


@pytest.mark.parametrize("devname", DEVICES)
@pytest.mark.parametrize("sd,od", [(torch.float32, torch.float32), (torch.bfloat16, torch.float32),
                                   (torch.bfloat16, torch.bfloat16), (torch.float32, torch.bfloat16)])
@pytest.mark.parametrize("k", [1, 2, 7, 16])
def test_multi_reduce(devname, sd, od, k):
    dev = _dev(devname)
    n = 10_007
    srcs = [torch.randn(n).to(sd) for _ in range(k)]
    want = (sum(s.float() for s in srcs) * 0.25).to(od)
    out = torch.empty(n, dtype=od, device=dev)
    multi_reduce_(out, [s.to(dev) for s in srcs], 0.25)
    tol = 1e-6 if od == torch.float32 else 1e-2
    torch.testing.assert_close(out.cpu().float(), want.float(), rtol=tol, atol=tol)


@pytest.mark.parametrize("devname", DEVICES)
@pytest.mark.parametrize("sd,dd", [(torch.float32, torch.bfloat16), (torch.bfloat16, torch.float32),
                                   (torch.float32, torch.float32)])
def test_pack_cast_many_tensors(devname, sd, dd):
    dev = _dev(devname)
    sizes = [1, 7, 8, 100, 8192, 8193, 20000, 3]
    srcs = [torch.randn(s).to(sd).to(dev) for s in sizes]
    flat = torch.zeros(sum(sizes) + 64, dtype=dd, device=dev)
    dsts, off = [], 0
    for s in sizes:
        dsts.append(flat.narrow(0, off, s))
        off += s
    pack_cast_(srcs, dsts)
    for s, d in zip(srcs, dsts):
        torch.testing.assert_close(d.cpu(), s.cpu().to(dd), rtol=0, atol=0)


@pytest.mark.parametrize("devname", DEVICES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,e5m2", [(4099, False), (3_000_017, False), (4099, True), (2_500_003, True)])
def test_fp8_roundtrip(devname, dtype, n, e5m2):
    """Per-tensor quantisation (on the GPU: amax partials + quantise) bit-equal to torch's cast of
    the scaled input, e4m3fn and e5m2, with odd tails and several amax blocks."""
    dev = _dev(devname)
    x = (torch.randn(n, generator=torch.Generator().manual_seed(n)) * 3).to(dtype)
    x[n // 3] = -17.5  # the amax sits in one block, negative
    x = x.to(dev)
    q, sinv = quantize_fp8(x, e5m2=e5m2)
    fmax, fdt = (57344.0, torch.float8_e5m2) if e5m2 else (448.0, torch.float8_e4m3fn)
    amax = x.float().abs().max()
    assert abs(sinv.item() - amax.item() / fmax) < 1e-6 * max(1.0, amax.item() / fmax * 448.0)
    # reference: torch's fp8 cast of the scaled input
    ref_q = (x.float().cpu() * (fmax / amax.cpu())).clamp(-fmax, fmax).to(fdt)
    assert q.dtype == fdt
    assert torch.equal(q.cpu().view(torch.uint8), ref_q.view(torch.uint8))
    if e5m2:
        return
    back = dequantize_fp8(q, sinv, torch.float32)
    torch.testing.assert_close(back.cpu(), ref_q.float() * sinv.cpu(), rtol=1e-6, atol=1e-6)
    rel = ((back.cpu() - x.float().cpu()).abs() / (x.float().cpu().abs() + 1e-3)).median()
    assert rel < 0.05


@pytest.mark.gpu
@pytest.mark.parametrize("e5m2", [False, True])
def test_fp8_delayed_scaling(e5m2):
    """DelayedScale: the first call scales just-in-time; later calls quantise with the amax the
    previous call recorded (in the same pass), so quantising the same tensor again is bit-equal to
    the just-in-time result, and a tensor with a larger amax saturates instead of rescaling."""
    from parameter_server_distributed_amd.ops.conv import DelayedScale

    dev = _dev("cuda")
    x = (torch.randn(1_000_003, generator=torch.Generator().manual_seed(3)) * 2).to(torch.bfloat16).to(dev)
    ds = DelayedScale(1.0)
    q0, s0 = ds.quantize(x, e5m2)
    qj, sj = quantize_fp8(x, e5m2=e5m2)
    assert torch.equal(q0.view(torch.uint8), qj.view(torch.uint8)) and torch.equal(s0, sj)
    q1, s1 = ds.quantize(x, e5m2)  # delayed: previous amax == this amax
    torch.cuda.synchronize()
    assert torch.equal(q1.view(torch.uint8), qj.view(torch.uint8))
    torch.testing.assert_close(s1, sj, rtol=1e-6, atol=0)
    amax = float(x.float().abs().max())
    assert abs(float(ds.hist[0]) - amax) <= 1e-6 * amax and float(ds.hist[1]) == 0.0
    y = x * 4  # amax grows 4x: quantised with the old scale (saturating), history follows
    q2, s2 = ds.quantize(y, e5m2)
    torch.cuda.synchronize()
    torch.testing.assert_close(s2, sj, rtol=1e-6, atol=0)
    fmax = 57344.0 if e5m2 else 448.0
    assert float(q2.float().abs().max()) == fmax
    assert abs(float(ds.hist[0]) - 4 * amax) <= 1e-5 * amax


@pytest.mark.gpu
@pytest.mark.parametrize("rows,V", [(4864, 30528), (1024, 1000), (37, 264), (8, 30522 + 6)])
def test_fused_cross_entropy_matches_fp32(rows, V):
    """Fused bf16 softmax cross-entropy (kernels/xent.hip) vs F.cross_entropy on the same values in
    fp32: loss, and the gradient (bf16-rounded), including ignored (-100) rows."""
    from parameter_server_distributed_amd.ops.loss import cross_entropy

    dev = _dev("cuda")
    g = torch.Generator().manual_seed(rows)
    x = (torch.randn(rows, V, generator=g) * 3).to(torch.bfloat16).to(dev)
    y = torch.randint(0, V, (rows,), generator=g)
    y[::7] = -100
    y = y.to(dev)
    xr = x.float().clone().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(xr, y)
    ref.backward()
    xk = x.clone().requires_grad_(True)
    loss = cross_entropy(xk, y)
    loss.backward()
    torch.testing.assert_close(loss.float(), ref.detach(), rtol=1e-5, atol=1e-5)
    assert xk.grad.dtype == torch.bfloat16
    torch.testing.assert_close(xk.grad.float(), xr.grad, rtol=1e-2, atol=1e-2 * float(xr.grad.abs().max()))
