"""CPU check of the recomputing tail's backward algebra (ops/tail.py) in fp64 against autograd:
the BN-backward partials reduced with the BN input taken as 0 (sum g, -mean sum g) plus the rowdot
row (0, sum_i W[c][i] (g^T a2)[c][i]) give sum g (y - mean) for y = a2 W^T that was never formed,
and the finalize coefficients from them reproduce d(loss)/dy = A g + B y + C."""
import torch


def test_tail_partials_reproduce_bn_backward():
    torch.manual_seed(0)
    M, cin, cout, eps = 512, 16, 32, 1e-5
    a2 = torch.randn(M, cin, dtype=torch.float64).relu()
    W = torch.randn(cout, cin, dtype=torch.float64)
    gamma = torch.rand(cout, dtype=torch.float64) + 0.5
    beta = torch.randn(cout, dtype=torch.float64) * 0.1
    idt = torch.randn(M, cout, dtype=torch.float64)
    r = torch.randn(M, cout, dtype=torch.float64)

    y = (a2 @ W.t()).requires_grad_(True)
    mean = y.mean(0)
    var = y.var(0, unbiased=False)
    invstd = 1.0 / torch.sqrt(var + eps)
    out = torch.relu((y - mean) * invstd * gamma + beta + idt)
    (out * r).sum().backward()
    dy_ref = y.grad

    yd = y.detach()
    g = r * (out.detach() > 0)  # the masked upstream gradient the consumer epilogue writes
    s1 = g.sum(0)
    part_epi = torch.stack([s1, g.sum(0) * (0 - mean.detach())])  # bwd modes 2 / 5 with bx null
    P = g.t() @ a2  # the fold wgrad's g^T a2
    row = torch.stack([torch.zeros(cout, dtype=torch.float64), (W * P).sum(1)])
    s1_, s2_ = part_epi + row
    torch.testing.assert_close(s2_, (g * (yd - mean.detach())).sum(0))
    isd = invstd.detach()
    k1 = gamma * isd
    k3 = s2_ * isd * isd / M
    k2 = s1_ / M
    A, B, C = k1, -k1 * k3, -k1 * k2 + k1 * k3 * mean.detach()
    torch.testing.assert_close(A * g + B * yd + C, dy_ref)
