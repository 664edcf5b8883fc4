"""Multi-head self-attention on the fused gfx950 kernels of ``csrc/kernels/attention.hip``.

Input is the packed QKV projection output ``[B, S, 3*H*64]`` exactly as the QKV Linear writes it;
output is ``[B, S, H*64]`` exactly as the output projection reads it. Backward returns the packed
``dQKV``. Compared with ``F.scaled_dot_product_attention`` on q/k/v views this removes the
transpose copy of the output, the stack/cat of dq/dk/dv and the layout copy in backward, and runs
the whole head (S <= 128) out of LDS in one kernel per direction.

Attention dropout uses the counter hash shared with the fused LayerNorm (per-site seed + the
model's device step counter, see ``ops/layernorm.bump_step``): masks are regenerated in backward
and a replayed hipGraph draws fresh ones each step.

CPU tensors, other dtypes, head dims != 64 or S not in {32, 64, 96, 128} use SDPA -- the reference
the tests compare against.
"""
from __future__ import annotations


import torch
import torch.nn as nn
import torch.nn.functional as F

from ..utils.config import feature as _feat
from .. import native


class _AttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, mod, p):
        # qkv straight from an MfmaLinear with a bias (ops/linear.py tags its output): backward also
        # sums dqkv's columns -- that Linear's bias gradient -- and hands it over
        src = getattr(qkv, "_psd_src", None) if _feat("attn_bias") else None
        ctx.src = src if (src is not None and src[0].bias is not None and src[0].act in (None, "none")
                          and src[0]._psd_tok == src[1]) else None
        qkv = qkv.contiguous()
        o, lse = native().attn_fwd(qkv, mod.heads, p, mod.seed, mod.step)
        ctx.mod, ctx.p = mod, p
        ctx.save_for_backward(qkv, o, lse)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        mod = ctx.mod
        db = None
        if ctx.src is not None:
            lin = ctx.src[0]
            sink = getattr(lin, "_psd_grad_sink", None)
            db = sink(lin.bias) if sink is not None else None
            if db is None:
                db = torch.empty_like(lin.bias)
        dqkv = native().attn_bwd(do, qkv, o, lse, mod.heads, ctx.p, mod.seed, mod.step, db)
        if db is not None:
            ctx.src[0]._psd_bias_hand = (ctx.src[1], dqkv.data_ptr(), db)
        return dqkv, None, None


class FusedSelfAttention(nn.Module):
    """softmax(Q K^T / sqrt(d)) V with dropout on the probabilities, from the packed QKV tensor."""

    def __init__(self, heads: int, p: float = 0.1, seed: int = 0):
        super().__init__()
        self.heads = heads
        self.p = p
        self.seed = int(seed) & 0x7FFFFFFF
        self.step = None  # device int64 counter, set by the owning model (ops/layernorm.bump_step)

    def _kernel_ok(self, qkv) -> bool:
        B, S, E = qkv.shape
        return (qkv.is_cuda and qkv.dtype == torch.bfloat16 and E % (3 * self.heads) == 0
                and E // (3 * self.heads) == 64 and S % 32 == 0 and 32 <= S <= 128)

    def forward(self, qkv):
        p = self.p if self.training else 0.0
        if self._kernel_ok(qkv):
            return _AttnFn.apply(qkv, self, p)
        B, S, E = qkv.shape
        H = self.heads
        q, k, v = qkv.view(B, S, 3, H, E // (3 * H)).permute(2, 0, 3, 1, 4).unbind(0)
        a = F.scaled_dot_product_attention(q, k, v, dropout_p=p)
        return a.transpose(1, 2).reshape(B, S, E // 3)
