"""``LayerNorm(x + dropout(h))`` -- the transformer residual tail -- on the fused gfx950 kernels of
``csrc/kernels/layernorm.hip`` (one pass forward, one pass backward + a tiny gamma/beta finalize).

Dropout masks come from a counter-based hash of (per-site seed, device step counter, element), so
they are regenerated in backward instead of stored, and a replayed hipGraph draws fresh masks each
step: the owning model bumps the shared counter on the device at the start of every forward
(``bump_step``). gamma/beta gradients go straight into the PS flat-gradient buffer when the data
plane installed a grad sink (as the fused BN does).

CPU tensors, other dtypes or hidden sizes use the composite ``F.layer_norm(x + F.dropout(h))`` --
the reference the tests compare against.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import native


class _AddLNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, h, weight, bias, mod, p, x_grad_to=None):
        C = native()
        shp = x.shape
        y, s, mean, rstd = C.ln_fwd(x.contiguous(), h.contiguous(), weight, bias, mod.eps, p, mod.seed, mod.step)
        ctx.mod, ctx.p, ctx.x_grad_to = mod, p, x_grad_to
        ctx.tok = getattr(x_grad_to, "_psd_tok", None) if x_grad_to is not None else None
        # h straight from an MfmaLinear with a bias and no activation (ops/linear.py tags its
        # output): the backward sums dh's columns in its own pass -- that Linear's bias gradient --
        # and hands it over, so the Linear skips its column-sum kernels
        src = getattr(h, "_psd_src", None)
        ctx.h_src = src if (src is not None and src[0].bias is not None and src[0].act in (None, "none")
                            and src[0]._psd_tok == src[1]) else None
        ctx.save_for_backward(s, mean, rstd, weight)
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        s, mean, rstd, w = ctx.saved_tensors
        mod = ctx.mod
        sink = getattr(mod, "_psd_grad_sink", None)
        dgo = dbo = None
        if sink is not None:
            dgo, dbo = sink(mod.weight), sink(mod.bias)
        dhs = None
        if ctx.h_src is not None:
            lin = ctx.h_src[0]
            lsink = getattr(lin, "_psd_grad_sink", None)
            dhs = lsink(lin.bias) if lsink is not None else None
            if dhs is None:
                dhs = torch.empty_like(lin.bias)
        dx, dh, dg, db = native().ln_bwd(dy, s, mean, rstd, w, ctx.p, mod.seed, mod.step, dgo, dbo, dhs)
        if dhs is not None:
            ctx.h_src[0]._psd_bias_hand = (ctx.h_src[1], dh.data_ptr(), dhs)
        if ctx.x_grad_to is not None:
            # residual-branch gradient handed to the Linear that also consumes x: its dgrad GEMM
            # accumulates onto it (beta = 1) instead of autograd adding the two [M, H] gradients
            ctx.x_grad_to._psd_pending_dx.append((ctx.tok, dx))
            return None, dh.view(dy.shape), dg, db, None, None, None
        return dx.view(dy.shape), dh.view(dy.shape), dg, db, None, None, None


class FusedAddLayerNorm(nn.LayerNorm):
    """``nn.LayerNorm`` applied to ``x + dropout(h)`` in one fused kernel family on MI355X."""

    def __init__(self, hidden: int, eps: float = 1e-12, p: float = 0.1, seed: int = 0):
        super().__init__(hidden, eps=eps)
        self.p = p
        self.seed = int(seed) & 0x7FFFFFFF
        self.step = None  # device int64 counter, set by the owning model (dropout masks per step)

    def psd_direct_grad_params(self):
        return [self.weight, self.bias]

    def _kernel_ok(self, x, h) -> bool:
        return (x.is_cuda and x.dtype == torch.bfloat16 and h.dtype == torch.bfloat16 and x.shape == h.shape
                and x.shape[-1] in (768, 1024) and self.weight is not None and self.weight.dtype == torch.bfloat16)

    def forward(self, x, h, x_grad_to=None):
        """``x_grad_to``: the ``MfmaLinear`` that consumed ``x`` earlier in the forward (the block's
        first projection). The gradient of ``x`` through this LayerNorm is then handed to that
        Linear's backward, which folds it into its bwd-data GEMM (beta = 1): the residual-stream
        gradient add is gone. The caller guarantees ``x`` has no other consumer."""
        p = self.p if self.training else 0.0
        if self._kernel_ok(x, h):
            if (x_grad_to is not None and torch.is_grad_enabled() and x.requires_grad
                    and getattr(x_grad_to, "psd_takes_pending_dx", lambda _x: False)(x)):
                return _AddLNFn.apply(x.detach(), h, self.weight, self.bias, self, p, x_grad_to)
            return _AddLNFn.apply(x, h, self.weight, self.bias, self, p)
        return F.layer_norm(x + F.dropout(h, p, self.training), self.normalized_shape,
                            None if self.weight is None else self.weight.to(x.dtype),
                            None if self.bias is None else self.bias.to(x.dtype), self.eps)


def bump_step(model: nn.Module) -> None:
    """Advance the model's dropout step counter (a non-persistent int64 buffer ``_psd_rng_step``,
    moved with the model) and point every FusedAddLayerNorm / FusedSelfAttention / FusedBertEmbeddings at it. Called at the start of each
    training forward; the increment runs on the device, so a captured hipGraph replays it."""
    step = getattr(model, "_psd_rng_step", None)
    if step is None or not model.training:
        return
    from .attention import FusedSelfAttention
    from .embedding import FusedBertEmbeddings

    for m in model.modules():
        if isinstance(m, (FusedAddLayerNorm, FusedSelfAttention, FusedBertEmbeddings)):
            m.step = step
    step.add_(1)
