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


def quantize_mx(x: torch.Tensor, e5m2: bool = False):
    """MX (OCP microscaling) fp8: ``(q, scales)`` with one E8M0 byte per 32 consecutive elements of
    the contiguous ``x`` (numel % 32 == 0), ``x ~= q * 2^(scale - 127)`` blockwise -- the operand
    format of the block-scaled MFMA (``gemm_fp8_`` / ``conv_fwd_fp8_`` with uint8 scales). Device
    tensors run kernels/fp8.hip quant_mx_kernel; host tensors the reference below (same rounding)."""
    x = x.contiguous()
    if not x.is_cuda:
        return quantize_mx_ref(x, e5m2)
    q = torch.empty(x.shape, dtype=torch.float8_e5m2 if e5m2 else torch.float8_e4m3fn, device=x.device)
    s = torch.empty(x.numel() // 32, dtype=torch.uint8, device=x.device)
    native().quant_mx_(x, q, s)
    return q, s


def quantize_mx_ref(x: torch.Tensor, e5m2: bool = False):
    """PyTorch reference of quant_mx_kernel: per 32-block the smallest power of two 2^e with
    amax * 2^-e <= fp8 max (E8M0 byte e + 127; 127 for an all-zero block), round-to-nearest-even."""
    fmax = FP8_E5M2_MAX if e5m2 else FP8_E4M3_MAX
    xf = x.float().reshape(-1, 32)
    amax = xf.abs().amax(1)
    m, p = torch.frexp(amax / fmax)
    e = torch.where(m == 0.5, p - 1, p).clamp(-127, 127)
    e = torch.where((amax > 0) & torch.isfinite(amax), e, torch.zeros_like(e))
    q = (xf * torch.exp2(-e.float()).unsqueeze(1)).clamp(-fmax, fmax)
    q = q.to(torch.float8_e5m2 if e5m2 else torch.float8_e4m3fn).reshape(x.shape)
    return q, (e + 127).to(torch.uint8)


def dequantize_mx_ref(q: torch.Tensor, scales: torch.Tensor) -> torch.Tensor:
    """fp32 ``q * 2^(scale - 127)`` blockwise (reference / host path of dequant_mx_)."""
    v = q.float().reshape(-1, 32) * torch.exp2(scales.float() - 127.0).unsqueeze(1)
    return v.reshape(q.shape)
