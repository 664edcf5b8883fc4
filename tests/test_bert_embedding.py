"""BERT's fused embedding block dropout(LayerNorm(word + position + type)) (ops/embedding.py
FusedBertEmbeddings, kernels/layernorm.hip emb_ln_*) against an fp32 composite with the kernel's own
dropout mask: the output, and the gradients of the three tables and of gamma / beta."""
import pytest
import torch
import torch.nn.functional as F


def _ref(emb, ids, types, mask, p):
    """fp32 composite of the same block (mask: the kernel's keep-mask, or ones)."""
    w = emb.word.weight.detach().float().requires_grad_(True)
    pt = emb.pos.weight.detach().float().requires_grad_(True)
    tt = emb.tok_type.weight.detach().float().requires_grad_(True)
    g = emb.ln.weight.detach().float().requires_grad_(True)
    b = emb.ln.bias.detach().float().requires_grad_(True)
    S = ids.shape[1]
    x = F.embedding(ids, w) + pt[:S][None] + F.embedding(types, tt)
    y = F.layer_norm(x, (w.shape[1],), g, b, emb.ln.eps) * mask / (1 - p)
    return y, (w, pt, tt, g, b)


def test_bert_embeddings_cpu_composite():
    from parameter_server_distributed_amd.ops.embedding import FusedBertEmbeddings

    torch.manual_seed(0)
    emb = FusedBertEmbeddings(100, 32, max_pos=16, p=0.0)
    ids = torch.randint(0, 100, (3, 9))
    types = torch.randint(0, 2, (3, 9))
    y = emb(ids, types)
    yr, _ = _ref(emb, ids, types, torch.ones(3, 9, 32), 0.0)
    torch.testing.assert_close(y, yr)
    y.sum().backward()
    assert emb.word.weight.grad is not None and emb.pos.weight.grad[9:].abs().sum() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("p,ntypes", [(0.0, 2), (0.1, 2), (0.1, 3)])
def test_bert_embeddings_match_fp32(gpu, p, ntypes):
    from parameter_server_distributed_amd import native
    from parameter_server_distributed_amd.ops.embedding import FusedBertEmbeddings

    from test_layernorm import _mask

    torch.manual_seed(1)
    V, H, B, S = 1000, 768, 4, 37
    emb = FusedBertEmbeddings(V, H, max_pos=64, type_vocab=ntypes, p=p, seed=11).to(gpu)
    with torch.no_grad():
        for t in (emb.word.weight, emb.pos.weight, emb.tok_type.weight):
            t.normal_(0, 0.5)
        emb.ln.weight.uniform_(0.5, 1.5)
        emb.ln.bias.uniform_(-0.5, 0.5)
    emb.to(torch.bfloat16)
    step = torch.tensor([5], device=gpu, dtype=torch.int64)
    emb.step = step
    ids = torch.randint(0, V, (B, S), device=gpu)
    ids[0, :10] = 3  # repeated ids: the word gradient's scatter sums runs
    types = torch.randint(0, ntypes, (B, S), device=gpu)
    y = emb(ids, types)
    g = torch.randn(B, S, H, device=gpu).to(torch.bfloat16)
    y.backward(g)

    mask = _mask(native(), (B, S, H), p, 11, step, gpu) if p > 0 else torch.ones(B, S, H, device=gpu)
    if p > 0:
        assert abs(mask.mean().item() - (1 - p)) < 0.03
    yr, leaves = _ref(emb, ids, types, mask, p)
    yr.backward(g.float())
    got = (y, emb.word.weight.grad, emb.pos.weight.grad, emb.tok_type.weight.grad, emb.ln.weight.grad,
           emb.ln.bias.grad)
    want = (yr,) + tuple(t.grad for t in leaves)
    for name, a, b in zip(("y", "word", "pos", "type", "gamma", "beta"), got, want):
        rel = ((a.float() - b).norm() / b.norm()).item()
        assert rel < 2e-2, (name, rel)
    assert emb.pos.weight.grad[S:].abs().sum().item() == 0

    first = [t.clone() for t in got[1:]]
    for t in (emb.word.weight, emb.pos.weight, emb.tok_type.weight, emb.ln.weight, emb.ln.bias):
        t.grad = None
    emb(ids, types).backward(g)
    again = (emb.word.weight.grad, emb.pos.weight.grad, emb.tok_type.weight.grad, emb.ln.weight.grad,
             emb.ln.bias.grad)
    assert all(torch.equal(a, b) for a, b in zip(first, again))  # deterministic


@pytest.mark.gpu
def test_bert_model_uses_fused_embedding_kernel(gpu):
    """The BERT model's embedding block runs the fused kernels (no PyTorch layer_norm / dropout)."""
    from parameter_server_distributed_amd import models
    from parameter_server_distributed_amd.ops import embedding

    spec = models.build("bert_base", gpu, torch.bfloat16, layers=1)
    for t in spec.model.parameters():  # bf16 working weights, as the PS data planes give them
        t.data = t.data.to(torch.bfloat16)
    calls = []
    orig = embedding._BertEmbLNFn.apply
    embedding._BertEmbLNFn.apply = lambda *a: calls.append(1) or orig(*a)
    try:
        x, y = spec.make_batch(2, gpu, seed=0)
        spec.loss(spec.model(x), y).backward()
    finally:
        embedding._BertEmbLNFn.apply = orig
    assert calls
    assert spec.model.emb.word.weight.grad is not None
