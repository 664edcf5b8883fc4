"""One identity bottleneck, bf16 kernel path vs fp32 composite reference: forward output and
gradient errors, and the same for each layer's pieces. Diagnostic; run on the GPU box."""
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from parameter_server_distributed_amd.models.resnet import Bottleneck  # noqa: E402
from parameter_server_distributed_amd.ops.bn import FusedBatchNorm2d  # noqa: E402

CL = torch.channels_last
dev = torch.device("cuda", 0)


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


def block(dt, bnrand):
    torch.manual_seed(2)
    blk = Bottleneck(256, 64)
    g = torch.Generator().manual_seed(4)
    for mod in blk.modules():
        if isinstance(mod, nn.Conv2d):
            nn.init.kaiming_normal_(mod.weight, mode="fan_out", nonlinearity="relu")
        if hasattr(mod, "running_mean") and mod.weight is not None and bnrand:
            mod.weight.data.copy_(0.5 + torch.rand(mod.weight.shape, generator=g))
            mod.bias.data.copy_(0.2 * torch.randn(mod.bias.shape, generator=g))
    blk = blk.to(dev)
    for p in blk.parameters():
        p.data = p.data.to(torch.bfloat16).to(dt)
        if p.dim() == 4:
            p.data = p.data.contiguous(memory_format=CL)
    x = torch.randn(8, 256, 28, 28, generator=torch.Generator().manual_seed(5)).to(torch.bfloat16).to(dev, dt)
    x = x.contiguous(memory_format=CL).requires_grad_(True)
    y = blk(x)
    gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(6)).to(torch.bfloat16).to(dev, dt)
    y.backward(gy.contiguous(memory_format=CL))
    grads = {n: p.grad.float() for n, p in blk.named_parameters()}
    grads["input"] = x.grad.float()
    return y.detach().float(), grads


for bnrand in (False, True):
    yb, gb = block(torch.bfloat16, bnrand)
    yf, gf = block(torch.float32, bnrand)
    print(f"bn random={bnrand}: output rel err {rel(yb, yf):.4f}")
    for n in gf:
        print(f"   {rel(gb[n], gf[n]):.4f} {n}")

# single BN(+relu) layer, bf16 kernels vs fp32 composite
for res in (False, True):
    torch.manual_seed(0)
    bn = FusedBatchNorm2d(64, relu=True).to(dev)
    bn.weight.data.uniform_(0.5, 1.5)
    bn.bias.data.normal_(0, 0.2)
    xb = (torch.randn(8, 64, 28, 28, device=dev) * 3 + 1).to(torch.bfloat16).contiguous(memory_format=CL)
    rb = torch.randn_like(xb) if res else None
    gy = torch.randn_like(xb)
    outs = []
    for dt in (torch.bfloat16, torch.float32):
        m = FusedBatchNorm2d(64, relu=True).to(dev)
        m.weight.data = bn.weight.data.to(torch.bfloat16).to(dt)
        m.bias.data = bn.bias.data.to(torch.bfloat16).to(dt)
        x = xb.to(dt).detach().requires_grad_(True)
        r = rb.to(dt).detach().requires_grad_(True) if res else None
        y = m(x, r)
        y.backward(gy.to(dt))
        outs.append((y.detach(), x.grad, m.weight.grad, m.bias.grad))
    print(f"single BN relu res={res}: y {rel(outs[0][0], outs[1][0]):.4f} dx {rel(outs[0][1], outs[1][1]):.4f} "
          f"dgamma {rel(outs[0][2], outs[1][2]):.4f} dbeta {rel(outs[0][3], outs[1][3]):.4f}")
