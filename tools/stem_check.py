#!/usr/bin/env python3
"""Stem conv kernel check: determinism (two runs bitwise) and error vs an fp32 conv."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from parameter_server_distributed_amd import native  # noqa: E402

dev = torch.device("cuda")
for shape in [(4, 3, 64, 64), (2, 3, 224, 224)]:
    torch.manual_seed(0)
    x = torch.randn(shape).to(torch.bfloat16).to(dev).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7) * 0.1).to(torch.bfloat16).to(dev).contiguous(memory_format=torch.channels_last)
    g, b = torch.ones(64, device=dev, dtype=torch.bfloat16), torch.zeros(64, device=dev, dtype=torch.bfloat16)
    outs = []
    for _ in range(3):
        rm, rv = torch.zeros(64, device=dev), torch.ones(64, device=dev)
        outs.append(native().stem_fwd(x, w, g, b, rm, rv, 0.1, 1e-5))
    ref = F.conv2d(x.float(), w.float(), stride=2, padding=3)
    c = outs[0][5].float()
    err = (c - ref).abs()
    print(shape, "max|conv-ref|", err.max().item(), "at", torch.nonzero(err == err.max())[0].tolist(),
          "ref max", ref.abs().max().item())
    for i in (1, 2):
        for j, name in enumerate(["y", "arg", "mean", "invstd", "ss", "conv"]):
            same = torch.equal(outs[0][j], outs[i][j])
            if not same:
                d = (outs[0][j].float() - outs[i][j].float()).abs()
                print(f"  run {i}: {name} differs: max {d.max().item()} count {(d > 0).sum().item()}")
    bad = err > 0.02 * ref.abs().max().item()
    print("  elements off by >2% of max:", bad.sum().item())
    if bad.any():
        idx = torch.nonzero(bad)[:8].tolist()
        print("  first:", idx)
