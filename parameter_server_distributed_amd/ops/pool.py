"""NHWC bf16 pooling on the gfx950 kernels of ``csrc/kernels/pool.hip``: the ResNet stem's 3x3 /
stride-2 / pad-1 max-pool and the head's global average pool. Other devices / dtypes / shapes use
``F.max_pool2d`` / ``F.adaptive_avg_pool2d`` (the numerics references of the tests)."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import native


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod):
        y, arg = native().maxpool3s2_fwd(x)
        ctx.save_for_backward(arg)
        ctx.hw = (x.shape[2], x.shape[3])
        ctx.mod = mod
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        # second consumer's gradient of the pool output (handed over by the first bottleneck's
        # _Fork): summed inside the gather kernel instead of by an autograd add over the output
        pend = getattr(ctx.mod, "_psd_pending_dr", None)
        dy2 = pend.pop() if pend else None
        return native().maxpool3s2_bwd(dy, arg, ctx.hw[0], ctx.hw[1], dy2), None


def _pool_kernel_ok(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0


def max_pool_3x3s2(x: torch.Tensor, mod: "MaxPool3x3s2 | None" = None) -> torch.Tensor:
    if _pool_kernel_ok(x):
        return _MaxPoolFn.apply(x, mod)
    return F.max_pool2d(x, 3, 2, 1)


class MaxPool3x3s2(nn.Module):
    """Stem max-pool. ``native_last`` tells the model whether the last forward ran the kernel, i.e.
    whether a consumer may hand it a second output gradient through ``_psd_pending_dr``."""

    def __init__(self):
        super().__init__()
        self._psd_pending_dr: list = []
        self.native_last = False

    def forward(self, x):
        self.native_last = _pool_kernel_ok(x)
        return max_pool_3x3s2(x, self)


class _GapFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[2], x.shape[3])
        return native().gap_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return native().gap_bwd(dy, ctx.hw[0], ctx.hw[1])


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] (channels_last) -> [N, C]."""
    if _pool_kernel_ok(x):
        return _GapFn.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
