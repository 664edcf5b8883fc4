"""fp8 weights through the PS (BASELINE config 5, "fp8 weights"): both data planes publish the MX
e4m3 copy of the fp32 masters (one E8M0 scale per 32 elements) and the fp8 convolutions consume the
pulled weights directly. Checked against the fp32 masters: the pulled e4m3 weights + scales are
bit-equal to quantising the owner's master, the bf16 working copy is their dequantisation, and the
fp8 convolutions read the published copy (no per-step weight quantisation)."""
import pytest
import torch

from parameter_server_distributed_amd import native
from parameter_server_distributed_amd.ops import quantize_mx
from parameter_server_distributed_amd.ops.optim import OptimConfig

pytestmark = pytest.mark.gpu


def _model(gpu):
    from parameter_server_distributed_amd.models import prepare
    from parameter_server_distributed_amd.models.resnet import ResNet

    torch.manual_seed(0)
    m = prepare(ResNet((1, 1, 1, 1), num_classes=10, width_per_group=128, fp8=True), gpu, torch.bfloat16,
                channels_last=True)
    for p in m.parameters():
        p.data = p.data.to(torch.bfloat16)
    return m.train()


def _batch(gpu):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(16, 3, 64, 64, generator=g).to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    return x, torch.randint(0, 10, (16,), generator=g).to(gpu)


def _check_published(model, qf, sf, pf, master):
    """Every fp8 module's published weight == MX(master slice); bf16 working copy == its dequant."""
    from parameter_server_distributed_amd.ops import conv as conv_ops

    n_checked = 0
    for m in model.modules():
        if not getattr(m, "fp8", False) or getattr(m, "_psd_w8", None) is None:
            continue
        w = m.weight
        w2 = w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)
        off = (w.data_ptr() - pf.data_ptr()) // 2
        q, s = m._psd_w8(w2)
        want_q, want_s = quantize_mx(master.narrow(0, off, w.numel()).contiguous())
        assert torch.equal(s, want_s)
        assert torch.equal(q.view(torch.uint8).flatten(), want_q.view(torch.uint8))
        back = torch.empty(w.numel(), device=w.device, dtype=torch.bfloat16)
        native().dequant_mx_(q.flatten(), s, back)
        assert torch.equal(back, w2.flatten())
        n_checked += 1
    assert n_checked >= 4
    return conv_ops


def test_async_plane_publishes_mx_weights(gpu):
    from parameter_server_distributed_amd.ops import conv as conv_ops
    from parameter_server_distributed_amd.parallel.async_ps import AsyncPS

    model = _model(gpu)
    ps = AsyncPS(model, OptimConfig("momentum", lr=0.05, momentum=0.9), staleness=0, bucket_mb=4, device=gpu,
                 pull_dtype="fp8")
    try:
        x, y = _batch(gpu)
        before = conv_ops.FP8_CALLS["ps_weights"]
        for _ in range(3):
            ps.begin_step()
            torch.nn.functional.cross_entropy(model(x).float(), y).backward()
            ps.finish_step()
        assert conv_ops.FP8_CALLS["ps_weights"] > before, "fp8 convolutions did not read the published weights"
        ps.drain()
        ps.begin_step()  # pull the final version
        torch.cuda.synchronize()
        assert ps.versions() == [4] or ps.versions() == [3], ps.versions()
        _check_published(model, ps.q8s[ps.cb], ps.sc8s[ps.cb], ps.pbufs[ps.cb], ps.master[0])
        assert bool(torch.isfinite(ps.pbufs[ps.cb].float()).all())
    finally:
        ps.close()


def test_collective_plane_publishes_mx_weights(gpu):
    from parameter_server_distributed_amd.parallel.collective_ps import CollectivePS
    from parameter_server_distributed_amd.runtime.trainer import Trainer

    model = _model(gpu)
    ps = CollectivePS(model, OptimConfig("momentum", lr=0.05, momentum=0.9), staleness=0, bucket_mb=4, device=gpu,
                      pull_dtype="fp8")
    assert ps.pull_mx
    x, y = _batch(gpu)
    tr = Trainer(model, lambda out, t: torch.nn.functional.cross_entropy(out.float(), t), ps, (x, y), use_graph=False)
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    _check_published(model, ps.p8, ps.p8_mx, ps.params_flat, ps.master)
