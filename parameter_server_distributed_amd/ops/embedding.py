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


def _bert_emb_kernel_ok(mod, ids, types) -> bool:
    w, p, t = mod.word.weight, mod.pos.weight, mod.tok_type.weight
    tabs = (w, p, t, mod.ln.weight, mod.ln.bias)
    return (ids.is_cuda and ids.dtype == torch.long and types is not None and types.dtype == torch.long
            and ids.dim() == 2 and types.shape == ids.shape and ids.shape[1] <= p.shape[0]
            and all(x is not None and x.dtype == torch.bfloat16 for x in tabs) and w.shape[1] == 768
            and mod.word.padding_idx is None and mod.tok_type.padding_idx is None and mod.pos.padding_idx is None
            and w.shape[0] > SMALL_VOCAB)


class _BertEmbLNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, types, w, pt, tt, gamma, beta, mod, p):
        B, S = ids.shape
        ids_f, types_f = ids.reshape(-1).contiguous(), types.reshape(-1).contiguous()
        y, mean, rstd = native().emb_ln_fwd(ids_f, types_f, w, pt, tt, gamma, beta, S, mod.ln.eps, p, mod.seed,
                                            mod.step)
        ctx.save_for_backward(ids_f, types_f, mean, rstd)
        ctx.mod, ctx.p, ctx.S = mod, p, S
        return y.view(B, S, -1)

    @staticmethod
    def backward(ctx, dy):
        ids, types, mean, rstd = ctx.saved_tensors
        mod = ctx.mod
        w, pt, tt = mod.word.weight, mod.pos.weight, mod.tok_type.weight
        sink = getattr(mod, "_psd_grad_sink", None)

        def out(param):  # the PS flat-gradient view (direct), else a fresh tensor
            v = sink(param) if sink is not None else None
            return v if v is not None and v.is_contiguous() else torch.empty_like(param)

        dgo, dbo = out(mod.ln.weight), out(mod.ln.bias)
        dT = out(tt) if tt.shape[0] <= 2 else None
        H = w.shape[1]
        dx, dg, db, dT = native().emb_ln_bwd(dy.reshape(-1, H), ids, types, w, pt, tt, mod.ln.weight, mean, rstd,
                                             ctx.S, ctx.p, mod.seed, mod.step, dgo, dbo, dT)
        if dT is None:  # > 2 token types: one-hot GEMM as FusedEmbedding's small-vocabulary path
            dT = out(tt)
            torch.mm(F.one_hot(types, tt.shape[0]).to(dx.dtype).t(), dx, out=dT)
        # word table: the deterministic sorted scatter of dx (kernels/embed.hip, as _EmbedFn)
        dW = out(w)
        s, perm = torch.sort(ids, stable=True)
        dW.zero_()
        native().embed_bwd_(s, perm, dx, dW)
        # position table: rows [0, S) take the batch sum, the rest none
        dP = out(pt)
        S = ctx.S
        dP[:S].copy_(torch.sum(dx.view(-1, S, H), 0, dtype=torch.float32))
        if S < dP.shape[0]:
            dP[S:].zero_()
        return None, None, dW, dP, dT, dg, db, None, None


class FusedBertEmbeddings(nn.Module):
    """BERT's embedding block ``dropout(LayerNorm(word[ids] + pos[s] + type[types]))`` on one fused
    gfx950 kernel each way (kernels/layernorm.hip emb_ln_*): the rows are gathered straight from the
    tables, the backward re-gathers them (only the row statistics are saved) and writes the
    embedding-sum gradient once for the word table's deterministic sorted scatter, the position
    table's batch sum and -- in the same pass -- the type rows' and LayerNorm's parameter gradients.
    Off-GPU / off-shape: the composite of nn.Embedding, nn.LayerNorm and F.dropout (the tests'
    reference). ``step``: the owning model's device dropout counter (layernorm.bump_step)."""

    def __init__(self, vocab: int, hidden: int, max_pos: int = 512, type_vocab: int = 2, eps: float = 1e-12,
                 p: float = 0.1, seed: int = 0):
        super().__init__()
        self.word = FusedEmbedding(vocab, hidden)
        self.pos = nn.Embedding(max_pos, hidden)
        self.tok_type = FusedEmbedding(type_vocab, hidden)
        self.ln = nn.LayerNorm(hidden, eps=eps)
        self.p = p
        self.seed = int(seed) & 0x7FFFFFFF
        self.step = None

    def psd_direct_grad_params(self):
        return [self.word.weight, self.pos.weight, self.tok_type.weight, self.ln.weight, self.ln.bias]

    def forward(self, ids, types):
        p = self.p if self.training else 0.0
        if (torch.is_grad_enabled() and any(x.requires_grad for x in self.parameters())
                and _bert_emb_kernel_ok(self, ids, types)):
            return _BertEmbLNFn.apply(ids, types, self.word.weight, self.pos.weight, self.tok_type.weight,
                                      self.ln.weight, self.ln.bias, self, p)
        S = ids.shape[1]
        pos = torch.arange(S, device=ids.device)
        x = self.word(ids) + self.pos(pos)[None] + self.tok_type(types)
        return F.dropout(self.ln(x), p, self.training)
