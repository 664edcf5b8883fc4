"""Python entry points for the hand-written gfx950 kernels.

Every function routes device tensors to the HIP kernels in ``csrc/kernels`` (on the caller's
current HIP stream) and host tensors to the bit-compatible C++ loops in ``csrc/ops.cpp``. There
is no silent eager-PyTorch fallback: if ``_C`` is missing these raise.
"""
from __future__ import annotations

import torch

from .. import native
from .optim import OptimConfig, OptimDyn, advance_, apply_no_advance_, fused_apply_  # noqa: F401

FP8_E4M3_MAX = 448.0
FP8_E5M2_MAX = 57344.0


def multi_reduce_(out: torch.Tensor, srcs, scale: float = 1.0) -> torch.Tensor:
    """``out = scale * sum(srcs)`` (fp32/bf16, up to 16 sources)."""
    native().multi_reduce_(out, list(srcs), float(scale))
    return out


def pack_cast_(srcs, dsts) -> None:
    """Copy+cast many tensors in one launch (fp32<->bf16)."""
    native().pack_cast_(list(srcs), list(dsts))


def quantize_fp8(x: torch.Tensor, amax: torch.Tensor | None = None, e5m2: bool = False):
    """Per-tensor OCP fp8 quantisation (e4m3fn, or e5m2 for gradients); returns ``(q, scale_inv)``
    with ``x ~= q * scale_inv``."""
    C = native()
    x = x.contiguous()
    q = torch.empty(x.shape, dtype=torch.float8_e5m2 if e5m2 else torch.float8_e4m3fn, device=x.device)
    sinv = torch.empty(1, dtype=torch.float32, device=x.device)
    if amax is None and x.is_cuda:  # amax + quantise in two launches, no atomics / zero-fill
        C.quant_fp8_jit_(x, q, sinv)
        return q, sinv
    if amax is None:
        amax = torch.zeros(1, dtype=torch.float32, device=x.device)
        C.amax_(x, amax)
    C.quant_fp8_(x, amax, FP8_E5M2_MAX if e5m2 else FP8_E4M3_MAX, q, sinv)
    return q, sinv


def dequantize_fp8(q: torch.Tensor, scale_inv: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    out = torch.empty(q.shape, dtype=dtype, device=q.device)
    native().dequant_fp8_(q.contiguous(), scale_inv, out)
    return out
