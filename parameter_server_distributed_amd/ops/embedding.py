"""Embedding with a deterministic gfx950 weight gradient (kernels/embed.hip).

forward   F.embedding (a gather)
backward  large vocabularies: stable sort of the ids; runs of equal ids are cut into segments of
          at most 64 sorted positions, one wave sums a segment's output-gradient rows (fp32), and
          the run's first wave adds the run's segment partials in order and writes the table row
          -- no atomics, so the gradient is bitwise reproducible, and a skewed batch (thousands of
          [PAD] tokens) costs no more than a uniform one;
          small vocabularies (<= 16 rows, e.g. BERT's token types): onehot(ids)^T . dy on the GEMM
          (a per-row sum over thousands of tokens is one long run, which the per-run kernel would
          sum serially)
CPU tensors, non-bf16 tables or widths off the kernel's grid (Hd % 256) use nn.Embedding's path.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import native

SMALL_VOCAB = 16


class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, mod):
        ctx.save_for_backward(ids)
        ctx.shape = weight.shape
        ctx.mod = mod
        return F.embedding(ids, weight)

    @staticmethod
    def backward(ctx, g):
        (ids,) = ctx.saved_tensors
        V, Hd = ctx.shape
        g2 = g.reshape(-1, Hd).contiguous()
        flat = ids.reshape(-1)
        # straight into the PS flat-gradient buffer when the data plane installed a sink (the table
        # gradient is then neither zeroed by the data plane nor accumulated into it)
        sink = getattr(ctx.mod, "_psd_grad_sink", None)
        dw = sink(ctx.mod.weight) if sink is not None else None
        if dw is None or not dw.is_contiguous():
            dw = torch.empty(V, Hd, dtype=g2.dtype, device=g2.device)
        if V <= SMALL_VOCAB:
            torch.mm(F.one_hot(flat, V).to(g2.dtype).t(), g2, out=dw)
            return None, dw, None
        s, perm = torch.sort(flat, stable=True)
        dw.zero_()
        native().embed_bwd_(s, perm, g2, dw)
        return None, dw, None


class FusedEmbedding(nn.Embedding):
    """``nn.Embedding`` (no padding_idx / max_norm / sparse) whose weight gradient runs on the
    deterministic gfx950 kernel for bf16 device tables."""

    def forward(self, ids):
        w = self.weight
        if (w.is_cuda and w.dtype == torch.bfloat16 and torch.is_grad_enabled() and w.requires_grad
                and self.padding_idx is None and self.max_norm is None and not self.sparse
                and (w.shape[0] <= SMALL_VOCAB or (w.shape[1] % 256 == 0 and w.shape[1] <= 2048))):
            return _EmbedFn.apply(ids, w, self)
        return super().forward(ids)

    def psd_direct_grad_params(self):
        return [self.weight]
