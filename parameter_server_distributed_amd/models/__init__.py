"""Model zoo for the BASELINE.json configs (random init, synthetic data of the real shapes).

``build(name, ...)`` returns a ``ModelSpec`` with the module, a synthetic-batch factory, the loss and
the sample unit used for throughput (images or sequences).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

import torch
import torch.nn as nn
import torch.nn.functional as F

from .mlp import MLP, synthetic_mnist
from .resnet import ResNet, resnet50, resnet101, wide_resnet101_2

__all__ = ["MLP", "ResNet", "resnet50", "resnet101", "wide_resnet101_2", "build", "ModelSpec", "MODELS"]


@dataclass
class ModelSpec:
    name: str
    model: nn.Module
    make_batch: Callable[[int, torch.device], tuple]
    loss: Callable
    sample_desc: str
    channels_last: bool = False
    tied_weights: bool = False


def _ce(out, y):
    from ..ops.loss import cross_entropy  # fused bf16 kernels on the GPU, fp32 F.cross_entropy elsewhere

    return cross_entropy(out, y)


def _image_batch(size: int, classes: int, dtype, channels_last: bool):
    def make(batch: int, device, seed: int = 0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        x = torch.randn(batch, 3, size, size, generator=g).to(device=device, dtype=dtype)
        if channels_last:
            x = x.contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, classes, (batch,), generator=g).to(device)
        return x, y

    return make


def prepare(model: nn.Module, device, dtype=torch.bfloat16, channels_last: bool = False) -> nn.Module:
    """Move to device, cast *buffers* (BN running stats) to the compute dtype, NHWC weights.

    Parameters stay fp32 here: the PS data plane takes the fp32 values as the master copy and
    re-points ``.data`` at its flat bf16 working buffer.
    """
    model = model.to(device)
    if channels_last:
        model = model.to(memory_format=torch.channels_last)
    for m in model.modules():
        if getattr(m, "_psd_fp32_buffers", False):
            continue
        for k, b in list(m._buffers.items()):
            if b is not None and b.is_floating_point():
                m._buffers[k] = b.to(dtype)
    return model


def build(name: str, device, dtype=torch.bfloat16, num_classes: int | None = None, **kw) -> ModelSpec:
    name = name.lower().replace("-", "_")
    if name in ("resnet50", "resnet101", "wide_resnet101_2", "wrn101"):
        ctor = {"resnet50": resnet50, "resnet101": resnet101, "wide_resnet101_2": wide_resnet101_2,
                "wrn101": wide_resnet101_2}[name]
        cls = num_classes or 1000
        size = kw.get("image_size", 224)
        cl = device.type == "cuda" if isinstance(device, torch.device) else str(device).startswith("cuda")
        m = prepare(ctor(cls, fp8=bool(kw.get("fp8", False))), device, dtype, channels_last=cl)
        return ModelSpec(name, m, _image_batch(size, cls, dtype, cl), _ce, "images", channels_last=cl)
    if name == "mlp":
        m = prepare(MLP(hidden=kw.get("hidden", 512)), device, dtype)

        def make(batch, device, seed=0):
            return synthetic_mnist(batch, device, dtype, seed)

        return ModelSpec(name, m, make, _ce, "images")
    if name in ("bert_base", "bert"):
        from .bert import BertForMLM, bert_batch

        m = prepare(BertForMLM(**{k: v for k, v in kw.items() if k in ("layers", "hidden", "heads", "vocab")}),
                    device, dtype)
        seq = kw.get("seq_len", 128)

        def make(batch, device, seed=0):
            return bert_batch(batch, seq, m.vocab, device, seed)

        return ModelSpec(name, m, make, m.loss, "sequences")
    raise KeyError(f"unknown model {name!r}; available: {MODELS}")


MODELS = ["mlp", "resnet50", "resnet101", "wide_resnet101_2", "bert_base"]
