#!/usr/bin/env python3
"""Which zero-fills run in a ResNet-50 training step, and who asks for them?

The r5 bench profile shows ~16 `FillFunctor<BFloat16>` launches per step at ~66 us each. This
runs two untimed fwd+bwd steps (autotune settles), then records every aten fill / zero op of the
third under a TorchDispatchMode (the mode is propagated to the autograd device thread), with the
tensor's shape and the innermost frames of this package on the Python stack (an empty stack =
the autograd engine itself, e.g. materialized gradients of unused Function outputs).

    python tools/probes/fill_probe.py [batch] [image] [--all]   (--all: every kernel-launching aten op)
"""
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from parameter_server_distributed_amd import models  # noqa: E402

FILL_OPS = ("fill_", "zero_", "zeros", "zeros_like", "new_zeros", "full", "full_like", "fill")
# with --all: every aten op that may launch a kernel (views, allocations and metadata ops skipped)
NO_KERNEL = ("empty", "empty_like", "empty_strided", "new_empty", "new_empty_strided", "view", "_unsafe_view", "as_strided",
             "expand", "permute", "t", "transpose", "reshape", "alias", "detach", "slice", "select", "unsqueeze",
             "squeeze", "split", "split_with_sizes", "narrow", "_to_copy", "lift_fresh", "is_same_size", "size",
             "stride", "sym_size", "sym_stride", "numel", "dim", "_local_scalar_dense", "item", "unbind", "set_",
             "resize_", "contiguous", "clone_", "_reshape_alias", "view_as", "_has_compatible_shallow_copy_type")
ALL = "--all" in sys.argv


class FillLog(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rows = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.__name__.split(".")[0]
        if (name not in NO_KERNEL) if ALL else (name in FILL_OPS):
            t = out if isinstance(out, torch.Tensor) else next((x for x in args if isinstance(x, torch.Tensor)), None)
            if t is None or not t.is_cuda:
                return out
            frames = [f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in traceback.extract_stack()
                      if "parameter_server_distributed_amd" in f.filename][-3:]
            self.rows[(name, str(t.dtype).replace("torch.", ""), tuple(t.shape), " < ".join(reversed(frames)))] += 1
        return out


def main():
    pos = [a for a in sys.argv[1:] if not a.startswith("--")]
    batch = int(pos[0]) if pos else 64
    img = int(pos[1]) if len(pos) > 1 else 224
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    spec = models.build("resnet50", dev, torch.bfloat16, image_size=img)
    m = spec.model
    for p in m.parameters():
        p.data = p.data.to(torch.bfloat16)
    x, y = spec.make_batch(batch, dev, seed=3)
    for i in range(2):
        spec.loss(m(x), y).backward()
        torch.cuda.synchronize()
        print(f"warmup step {i} done", flush=True)
        for p in m.parameters():
            p.grad = None
    torch.cuda.synchronize()
    log = FillLog()
    with log:
        spec.loss(m(x), y).backward()
    torch.cuda.synchronize()
    tot = 0
    for (name, dt, shape, where), k in sorted(log.rows.items(), key=lambda kv: -kv[1] * (1 + sum(kv[0][2]))):
        n = 1
        for s in shape:
            n *= s
        tot += k * n
        print(f"{k:3d}x {name:10s} {dt:9s} {str(list(shape)):24s} {n / 1e6:8.2f} M  {where or '(autograd engine)'}")
    print(f"total filled elements: {tot / 1e6:.1f} M")


if __name__ == "__main__":
    main()
