"""Softmax cross-entropy on bf16 logits through the fused gfx950 kernels of ``csrc/kernels/xent.hip``.

Forward reads the logits once (per-row log-sum-exp kept for backward); backward writes the bf16
gradient ``(softmax - onehot) * dloss / count`` in one pass -- no fp32 copy of the logits, no
log-prob tensor (the MLM decoder's logits are 4864 x 30528 per BERT-base b256 step). Mean over the
rows whose label is not negative (``ignore_index=-100`` semantics). Host tensors, other dtypes or
column counts that are not a multiple of 8 use ``F.cross_entropy`` on fp32 logits -- the reference
the tests compare against.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import native


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        loss_row, lse = native().xent_fwd(logits, labels)
        count = (labels >= 0).sum().clamp_min(1).to(torch.float32)
        ctx.save_for_backward(logits, labels, lse, count)
        return loss_row.sum() / count

    @staticmethod
    def backward(ctx, g):
        logits, labels, lse, count = ctx.saved_tensors
        scale = (g.float() / count).reshape(1)
        return native().xent_bwd(logits, labels, lse, scale), None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Mean softmax cross-entropy of ``logits [rows, classes]`` against int64 ``labels [rows]``."""
    if (logits.is_cuda and logits.dtype == torch.bfloat16 and logits.dim() == 2 and logits.shape[1] % 8 == 0
            and logits.stride(1) == 1 and logits.stride(0) % 8 == 0 and logits.data_ptr() % 16 == 0
            and labels.dtype == torch.int64 and labels.dim() == 1):
        return _XentFn.apply(logits, labels.contiguous())
    return F.cross_entropy(logits.float(), labels)
