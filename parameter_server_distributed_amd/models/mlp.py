"""2-layer MLP on MNIST-shaped data (BASELINE.json config 1: the CPU/gloo plumbing config).

On a GPU its two Linear layers run on the hand-written MFMA bf16 GEMM (``ops.gemm.MfmaLinear``);
on the CPU they are plain ``nn.Linear`` (fp32).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class MLP(nn.Module):
    def __init__(self, in_features: int = 784, hidden: int = 512, num_classes: int = 10, linear_cls=None):
        super().__init__()
        if linear_cls is None:
            from ..ops.linear import MfmaLinear as linear_cls
        self.fc1 = linear_cls(in_features, hidden)
        self.fc2 = linear_cls(hidden, num_classes)

    def forward(self, x):
        return self.fc2(F.relu(self.fc1(x.flatten(1))))


def synthetic_mnist(batch: int, device, dtype=torch.float32, seed: int = 0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.rand(batch, 1, 28, 28, generator=g).to(device=device, dtype=dtype)
    y = torch.randint(0, 10, (batch,), generator=g).to(device)
    return x, y
