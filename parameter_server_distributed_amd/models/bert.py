"""BERT-base (12 layers, hidden 768, 12 heads, FFN 3072) with the masked-LM head, for BASELINE.json
config 4 (BERT-base with the Adam update kernel). Random init, synthetic token batches.

Every Linear is an ``MfmaLinear`` (hand-written gfx950 MFMA GEMM forward + both backward GEMMs,
bias/GELU fused); attention is the fused gfx950 kernel of ``ops/attention.py`` (SDPA off-GPU).
Deviations from the original BERT, both standard in large-scale training and stated here: the
vocabulary is padded to 30528 (a multiple of 64, for the GEMM tiles) and the MLM decoder weight is
untied from the word embedding (the PS data plane overlaps each bucket's update with the rest of
backward, which requires every weight to be consumed by exactly one autograd node).
"""
from __future__ import annotations


import torch
import torch.nn as nn

from ..ops.attention import FusedSelfAttention
from ..ops.embedding import FusedBertEmbeddings
from ..ops.layernorm import FusedAddLayerNorm, bump_step
from ..ops.linear import MfmaLinear
from ..ops.loss import cross_entropy

VOCAB = 30528


class BertLayer(nn.Module):
    def __init__(self, hidden=768, heads=12, ffn=3072, dropout=0.1, index=0):
        super().__init__()
        self.heads = heads
        self.qkv = MfmaLinear(hidden, 3 * hidden)
        # packed QKV in, [B, S, hidden] out: one fused kernel per direction (ops/attention.py)
        self.attn = FusedSelfAttention(heads, p=dropout, seed=1000 + index)
        self.proj = MfmaLinear(hidden, hidden)
        # LayerNorm(x + dropout(branch)) as one fused kernel family (ops/layernorm.py)
        self.ln1 = FusedAddLayerNorm(hidden, eps=1e-12, p=dropout, seed=2 * index + 1)
        self.ffn1 = MfmaLinear(hidden, ffn, act="gelu")
        self.ffn2 = MfmaLinear(ffn, hidden)
        # ffn1's output feeds only ffn2: ffn2's bwd-data GEMM applies the GELU backward and sums
        # ffn1's bias gradient in its epilogue (ops/linear.py)
        self.ffn2.psd_gelu_input_from(self.ffn1)
        self.ln2 = FusedAddLayerNorm(hidden, eps=1e-12, p=dropout, seed=2 * index + 2)
        self.p = dropout

    def forward(self, x):
        # each residual LayerNorm hands the gradient of its x input to the Linear that also reads x
        # (folded into that Linear's bwd-data GEMM, ops/layernorm.py)
        x = self.ln1(x, self.proj(self.attn(self.qkv(x))), x_grad_to=self.qkv)
        return self.ln2(x, self.ffn2(self.ffn1(x)), x_grad_to=self.ffn1)


class BertForMLM(nn.Module):
    def __init__(self, layers=12, hidden=768, heads=12, vocab=VOCAB, max_pos=512, dropout=0.1):
        super().__init__()
        self.vocab = vocab
        # dropout(LayerNorm(word + position + token type)) on one fused kernel each way, with the
        # word table's deterministic sorted-scatter gradient (ops/embedding.py)
        self.emb = FusedBertEmbeddings(vocab, hidden, max_pos, 2, eps=1e-12, p=dropout, seed=4242)
        self.layers = nn.ModuleList([BertLayer(hidden, heads, 4 * hidden, dropout, i) for i in range(layers)])
        self.head = MfmaLinear(hidden, hidden, act="gelu")
        self.head_ln = nn.LayerNorm(hidden, eps=1e-12)
        self.decoder = MfmaLinear(hidden, vocab)
        self.p = dropout
        # device step counter for the fused LayerNorms' dropout masks (ops/layernorm.py)
        self.register_buffer("_psd_rng_step", torch.zeros(1, dtype=torch.int64), persistent=False)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, std=0.02)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Embedding):
                nn.init.normal_(m.weight, std=0.02)

    def forward(self, batch):
        ids, types, mlm_pos = batch
        bump_step(self)
        x = self.emb(ids, types)
        for layer in self.layers:
            x = layer(x)
        # MLM head only on the masked positions (max_predictions_per_seq per sequence, as in the
        # original BERT pre-training): 6-7x less head/decoder/softmax work than all tokens
        x = x.reshape(-1, x.shape[-1]).index_select(0, mlm_pos)
        return self.decoder(self.head_ln(self.head(x)))

    @staticmethod
    def loss(logits, labels):
        return cross_entropy(logits, labels)  # fused bf16 softmax-CE kernels (ops/loss.py)


def bert_batch(batch: int, seq: int, vocab: int, device, seed: int = 0, mask_prob: float = 0.15):
    """Synthetic pre-training batch: random ids, sentence-B types for the second half, and
    round(mask_prob * seq) masked positions per sequence (flat indices) with their labels."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    ids = torch.randint(0, vocab, (batch, seq), generator=g)
    types = (torch.arange(seq)[None, :] >= seq // 2).long().expand(batch, seq).contiguous()
    npred = max(1, round(mask_prob * seq))
    cols = torch.stack([torch.randperm(seq, generator=g)[:npred].sort().values for _ in range(batch)])
    flat = (cols + torch.arange(batch)[:, None] * seq).reshape(-1)
    labels = ids.reshape(-1)[flat]
    return (ids.to(device), types.to(device), flat.to(device)), labels.to(device)
