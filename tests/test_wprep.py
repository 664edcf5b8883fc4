"""Batched bwd-data weight operands (ops/wprep.py, kernels/wprep.hip).

The operands are permutations of the weight, so the GPU checks are bitwise against the torch
formulas they replace (``w.t()``, ``w.flip(2, 3).permute(1, 2, 3, 0)``, ``_s2_phase_weights``),
including a refresh after an in-place weight update; a ResNet block's gradients with the batched
operands match the per-convolution ones. The CPU test pins the tap geometry of each kind."""
import copy

import pytest
import torch
import torch.nn as nn

from parameter_server_distributed_amd.ops import wprep
from parameter_server_distributed_amd.ops.conv import _s2_phase_weights
from parameter_server_distributed_amd.utils.config import set_feature


def _apply_geo(w, g):
    """dst[ci][r'][s'][co] = w[co][ci][r0 + r' sr][s0 + s' ss] (torch reference of one job)."""
    rp, sp, r0, s0, sr, ss = g
    rows = [r0 + i * sr for i in range(rp)]
    cols = [s0 + j * ss for j in range(sp)]
    sub = w[:, :, rows][:, :, :, cols]
    return sub.permute(1, 2, 3, 0).reshape(w.shape[1], -1)


def _want(w, kind):
    cout, cin, k, _ = w.shape
    if kind == "t":
        return [w.reshape(cout, cin).t().contiguous()]
    if kind == "f":
        return [w.flip(2, 3).permute(1, 2, 3, 0).reshape(cin, k * k * cout).contiguous()]
    return _s2_phase_weights(w)


@pytest.mark.parametrize("kind,k", [("t", 1), ("f", 3), ("p", 3)])
def test_geometry_matches_torch_formulas(kind, k):
    w = torch.randn(16, 24, k, k)
    got = [_apply_geo(w, g) for g in wprep._geo(kind, k)]
    want = _want(w, kind)
    assert len(got) == len(want)
    for a, b in zip(got, want):
        assert torch.equal(a, b)


def test_cpu_weights_are_not_registered():
    wprep.REGISTRY.clear()
    m = nn.Conv2d(16, 16, 3, bias=False)
    wprep.note(m, m.weight.data, "f")
    assert wprep.get(m, m.weight.data, "f") is None
    assert not wprep.REGISTRY.entries


SHAPES = [  # cout, cin, k, kind
    (256, 64, 1, "t"),
    (64, 256, 1, "t"),
    (512, 128, 1, "t"),
    (64, 64, 3, "f"),
    (24, 40, 3, "f"),     # ragged 64-tiles in both dimensions
    (128, 128, 3, "p"),
    (72, 200, 3, "p"),
]


@pytest.mark.gpu
def test_batched_operands_bitwise(gpu):
    wprep.REGISTRY.clear()
    set_feature("wprep", True)
    try:
        torch.manual_seed(0)
        mods, ws = [], []
        for cout, cin, k, kind in SHAPES:
            m = nn.Module()
            w = torch.randn(cout, cin, k, k, device=gpu).to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            mods.append(m)
            ws.append(w)
            wprep.note(m, w, kind)
        for rnd in range(2):
            for m, w, (_, _, _, kind) in zip(mods, ws, SHAPES):
                got = wprep.get(m, w, kind)
                assert got is not None
                got = got if isinstance(got, list) else [got]
                want = _want(w, kind)
                assert len(got) == len(want)
                for a, b in zip(got, want):
                    assert a.shape == b.shape
                    assert torch.equal(a, b), (w.shape, kind, rnd)
            # an in-place update (the PS apply) and the next forward: the operands follow
            for m, w, (_, _, _, kind) in zip(mods, ws, SHAPES):
                w.mul_(-2.0).add_(0.5)
                wprep.note(m, w, kind)
        # a weight of another storage is not served from the table
        m, w, (_, _, _, kind) = mods[0], ws[0], SHAPES[0]
        assert wprep.get(m, w.clone(memory_format=torch.channels_last), kind) is None
        # a Parameter whose storage alternates between two buffers (the async PS's prefetch double
        # buffer, parallel/async_ps.py begin_step): each step serves the current buffer
        m = nn.Module()
        bufs = [torch.randn(128, 64, 3, 3, device=gpu).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last) for _ in range(2)]
        p = nn.Parameter(bufs[0].clone(memory_format=torch.channels_last))
        for step in range(5):
            p.data = bufs[step % 2]
            wprep.note(m, p, "f")
            got = wprep.get(m, p, "f")
            assert got is not None and torch.equal(got, _want(bufs[step % 2], "f")[0]), step
        assert len(wprep.REGISTRY.tables[p.device]) == 2  # one job table per buffer set
    finally:
        set_feature("wprep", None)
        wprep.REGISTRY.clear()


@pytest.mark.gpu
def test_resnet_blocks_match_unbatched(gpu, monkeypatch):
    """A stride-2 (1x1 transposes, stride-2 phases, strided downsample) and a stride-1 (tap flip)
    bottleneck: every gradient with the batched operands equals the per-convolution build."""
    from parameter_server_distributed_amd.models.resnet import Bottleneck, _conv
    from parameter_server_distributed_amd.ops import autotune
    from parameter_server_distributed_amd.ops.bn import FusedBatchNorm2d

    torch.manual_seed(0)
    net0 = nn.Sequential(
        Bottleneck(256, 128, 2, 64, nn.Sequential(_conv(256, 512, 1, 2), FusedBatchNorm2d(512))),
        Bottleneck(512, 128, 1, 64, None),
    ).to(gpu).to(memory_format=torch.channels_last)
    for p in net0.parameters():
        p.data = p.data.to(torch.bfloat16)
    x0 = torch.randn(4, 256, 28, 28, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    monkeypatch.setenv("PSD_FEATURES", "tail_recompute=0")

    def run(on):
        set_feature("wprep", on)
        wprep.REGISTRY.clear()
        net = copy.deepcopy(net0)
        out = {}
        for step in range(2):  # the second step refreshes the table built in the first
            x = x0.clone().requires_grad_(True)
            net.zero_grad(set_to_none=True)
            net(x).float().pow(2).mean().backward()
            out = {"dx": x.grad.float(), **{n: p.grad.float() for n, p in net.named_parameters()}}
            with torch.no_grad():
                for p in net.parameters():
                    p.add_(p.grad, alpha=-0.01)
        return out, len(wprep.REGISTRY.entries)

    calls = {"n": 0}
    real = wprep.REGISTRY._refresh

    def counted(dev):
        calls["n"] += 1
        real(dev)

    try:
        autotune._DECISIONS.clear()
        off, n_off = run(False)
        monkeypatch.setattr(wprep.REGISTRY, "_refresh", counted)
        on, n_on = run(True)  # the same autotune decisions (kept from the first run)
    finally:
        set_feature("wprep", None)
        wprep.REGISTRY.clear()
        autotune._DECISIONS.clear()
    assert n_off == 0 and n_on >= 6, (n_off, n_on)
    assert calls["n"] == 2, calls  # one refresh per step
    for n in off:
        err = ((on[n] - off[n]).norm() / off[n].norm().clamp_min(1e-6)).item()
        assert err <= 1e-2, (n, err)
