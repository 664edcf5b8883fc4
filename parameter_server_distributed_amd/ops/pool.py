"""3x3 / stride-2 / pad-1 max-pool on NHWC bf16 (kernels/pool.hip); ``F.max_pool2d`` elsewhere."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import native


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y, arg = native().maxpool3s2_fwd(x)
        ctx.save_for_backward(arg)
        ctx.hw = (x.shape[2], x.shape[3])
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        return native().maxpool3s2_bwd(dy, arg, ctx.hw[0], ctx.hw[1])


def max_pool_3x3s2(x: torch.Tensor) -> torch.Tensor:
    if x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0:
        return _MaxPoolFn.apply(x)
    return F.max_pool2d(x, 3, 2, 1)
