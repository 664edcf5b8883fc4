#!/usr/bin/env python3
"""Where does the fp8 path's gradient error come from? One forward/backward of a short Wide-ResNet
(width_per_group 128, one block per stage) in bf16 and in fp8 (forward only / forward + bwd-data),
same weights and batch; prints the overall relative gradient error and the worst parameters."""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parameter_server_distributed_amd.models import prepare  # noqa: E402
from parameter_server_distributed_amd.models.resnet import ResNet  # noqa: E402
from parameter_server_distributed_amd.ops.conv import Conv1x1, ConvNHWC  # noqa: E402


def grads(m, x, y):
    m.zero_grad(set_to_none=True)
    F.cross_entropy(m(x).float(), y).backward()
    return {n: p.grad.float().clone() for n, p in m.named_parameters()}


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    base = ResNet((1, 1, 1, 1), num_classes=100, width_per_group=128,
                  zero_init_residual=os.environ.get("ZIR", "0") == "1")
    models = {}
    for name, fp8 in (("bf16", False), ("fp8", True)):
        m = copy.deepcopy(base)
        for mod in m.modules():
            if isinstance(mod, (Conv1x1, ConvNHWC)):
                mod.fp8 = fp8
        m = prepare(m, dev, torch.bfloat16, channels_last=True)
        for p in m.parameters():
            p.data = p.data.to(torch.bfloat16)
        models[name] = m.train()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(int(os.environ.get("B", "16")), 3, 64, 64, generator=g).to(dev, torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 100, (x.shape[0],), generator=g).to(dev)
    ref = grads(models["bf16"], x, y)
    ref = grads(models["bf16"], x, y)  # after the first call: every route decided (autotune)
    grads(models["fp8"], x, y)
    ref2 = grads(models["bf16"], x, y)  # bf16 run-to-run (library nondeterminism)
    runs = {"bf16-again": ref2}
    os.environ["PSD_FEATURES"] = "fp8_dgrad=0"
    runs["fp8-fwd"] = grads(models["fp8"], x, y)
    os.environ["PSD_FEATURES"] = "fp8_dgrad=1"
    runs["fp8-fwd+dgrad"] = grads(models["fp8"], x, y)
    for name, gr in runs.items():
        num = sum(float((gr[n] - ref[n]).pow(2).sum()) for n in ref)
        den = sum(float(ref[n].pow(2).sum()) for n in ref)
        worst = sorted(((float((gr[n] - ref[n]).norm() / (ref[n].norm() + 1e-12)), n) for n in ref), reverse=True)[:6]
        big = sorted(((float(ref[n].pow(2).sum()) / den, n) for n in ref), reverse=True)[:4]
        print(f"{name}: overall rel err {(num / den) ** 0.5:.4f}; worst {[(round(e, 3), n) for e, n in worst]}")
        print(f"   largest-gradient params (share of |g|^2): {[(round(s_, 3), n) for s_, n in big]}")


if __name__ == "__main__":
    main()
