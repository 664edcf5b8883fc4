#!/usr/bin/env python3
"""How sensitive is the ResNet-50 tail-vs-fp32 loss comparison to bf16-sized perturbations?

For several (batch, image size, bn3 gain range) settings: the fp32 model's loss spread under
relative 2^-9 noise on the input (3 draws), and the bf16 unfused / recomputing-tail losses (tail
decisions timed once, the shared convolutions' decisions pinned from the unfused run) vs fp32. A
setting whose fp32 loss moves by percents under bf16-ulp noise cannot tell a tail bug from chaos
(tools/probes/tail_stats_probe.py: b8 64x64 gains 0.5-1.5 moves 2.49-2.60).
"""
import copy
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from parameter_server_distributed_amd import models  # noqa: E402
from parameter_server_distributed_amd.models.resnet import Bottleneck  # noqa: E402
from parameter_server_distributed_amd.ops import autotune  # noqa: E402


def one(batch, img, lo, hi):
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    spec = models.build("resnet50", dev, torch.bfloat16, image_size=img, num_classes=10)
    for mod in spec.model.modules():
        if isinstance(mod, Bottleneck):
            nn.init.uniform_(mod.bn3.weight, lo, hi)
    for p in spec.model.parameters():
        p.data = p.data.to(torch.bfloat16)
    init = copy.deepcopy(spec.model.state_dict())
    m32 = copy.deepcopy(spec.model).float()
    x, y = spec.make_batch(batch, dev, seed=3)

    def f32(xin):
        m32.load_state_dict(init)
        with torch.no_grad():
            return float(spec.loss(m32(xin), y))

    ref = f32(x.float())
    g = torch.Generator(device=dev).manual_seed(7)
    noisy = [f32(x.float() * (1 + 2 ** -9 * torch.randn(x.shape, device=dev, generator=g))) for _ in range(3)]
    spread = max(abs(v - ref) for v in noisy) / ref

    def run(tail_on):
        os.environ["PSD_FEATURES"] = f"tail_recompute={int(tail_on)}"
        m = spec.model
        m.load_state_dict(init)
        m.zero_grad(set_to_none=True)
        loss = spec.loss(m(x), y)
        loss.backward()
        return float(loss)

    autotune._DECISIONS.clear()
    off = [run(False) for _ in range(2)]
    on = [run(True) for _ in range(3)]
    autotune._DECISIONS.clear()
    print(f"b{batch} {img}px gain[{lo},{hi}]: fp32 {ref:.5f} noise-spread {spread:.3%} | "
          f"unfused {max(abs(v - ref) for v in off) / ref:.3%} | tail {max(abs(v - ref) for v in on) / ref:.3%}",
          flush=True)


if __name__ == "__main__":
    for cfg in ((8, 64, 0.5, 1.5), (32, 64, 0.5, 1.5), (8, 64, 0.1, 0.3), (32, 64, 0.1, 0.3), (16, 96, 0.5, 1.5),
                (32, 96, 0.2, 0.5)):
        one(*cfg)
