"""Identity-bottleneck tail ``relu(bn3(conv3(a2)) + x)`` without storing the BN input.

The unfused tail writes y3 = conv3(a2) (the 4x-wide activation), reads it back for the BN statistics'
consumer pass (bn_apply: read y3 and the residual, write the output and its ReLU bit-mask), and
keeps y3 alive until backward, whose BN reduction reads it once more. Per identity block at ResNet-50
b1024 layer1 that is ~5 activation passes of 1.6 GB over a tensor that is a cheap 1x1 GEMM of a
4x-narrower input (K = 64..512).

Here y3 is recomputed instead of stored (kernels/convn.hip):
  forward   1. conv3 statistics pass: the narrow GEMM with the BN statistics epilogue and no store
            2. BN finalize from those partials (mean, invstd, scale/shift, running statistics)
            3. conv3 apply pass: the same GEMM whose epilogue writes relu(bf16(y3) * scale + shift + x)
               and the ReLU bit-mask (bwd mode 8) -- y3 never reaches HBM
  backward  the consumer convolution's bwd-data epilogue (the next block's conv1, modes 2 / 5) reduces
            g = mask (dX + dr) with the BN input taken as 0: sum g and -mean sum g. The missing
            sum g y3 is sum_i W[c][i] (g^T a2)[c][i] -- the fold wgrad's g^T a2, which conv3's
            BN-backward fold computes anyway (kernels/bnfold.hip rowdot) -- so the finalize runs
            after that wgrad, then the folded dgrad / wgrad combination (ops/conv.py _fold_backward).
  Without that fused consumer (e.g. the network's last block, whose output feeds the pooling), the
  backward recomputes y3 once and runs the ordinary BN backward + fold.

Numerics: the statistics (Gram moments or the statistics-only pass) and the apply pass all use the
fp32 product y3 -- the apply normalises it before its one rounding to bf16 -- so the moments are
exactly those of the normalised tensor (within 1e-5 of fp64 per layer,
tests/test_tail.py::test_tail_statistics_match_fp64). The unfused tail normalises the bf16-rounded
stored y3 instead: a rounding-level difference (normalising bf16(y3) with the Gram moments of the
fp32 y3 moved the b8 ResNet-50 test loss by 0.55 %, tools/probes/tail_stats_probe.py). The
backward's sum g y3 also uses the fp32 product.

Reference: the reference's worker has no model at all (its "gradient" is a constant,
/root/reference/src/worker.cpp:316-329); this is the MI355X data-movement design of the
bottleneck tail ResNet-50 training needs.
"""
from __future__ import annotations

import torch

from ..utils.config import feature as _feat
from . import autotune as _at
from .conv import (Conv1x1, _fold_backward, _from_2d, _fwd_records, _native, _part_rows, _sink_view, fold_ok)
from .bn import FusedBatchNorm2d, take_dr

__all__ = ["tail_ok", "conv_bn_tail", "TAIL_CALLS"]

TAIL_CALLS = {"fwd": 0, "bwd_fused": 0, "bwd_recompute": 0}


def tail_ok(conv, bn, a2: torch.Tensor, idt: torch.Tensor) -> bool:
    """The recomputing tail applies: a bf16 Conv1x1 (no fp8) into a training ReLU FusedBatchNorm2d
    with an identity residual, channels_last operands, a shape the narrow kernel and the fold take."""
    if not (_feat("tail_recompute") and _feat("convn")) or not isinstance(conv, Conv1x1) \
            or conv.fp8:
        return False
    if not isinstance(bn, FusedBatchNorm2d) or not bn.relu or not bn.training or bn.weight is None:
        return False
    if not (a2.is_cuda and a2.dtype == torch.bfloat16 and idt.dtype == torch.bfloat16 and torch.is_grad_enabled()):
        return False
    if conv.weight.dtype != torch.bfloat16 or getattr(bn, "_psd_q8_consumer", None) is not None:
        return False
    cin, cout = conv.in_channels, conv.out_channels
    if idt.shape != (a2.shape[0], cout, a2.shape[2], a2.shape[3]):
        return False
    if not (a2.is_contiguous(memory_format=torch.channels_last) and idt.is_contiguous(memory_format=torch.channels_last)):
        return False
    C = _native()
    return fold_ok(cin, cout) and C.convn_variants(cout) > 0 and (a2.shape[0] * a2.shape[2] * a2.shape[3]) % 8 == 0


def _variant(a2, w2, M: int, cin: int, cout: int, h: int, w: int, shift) -> int:
    """Narrow-kernel tile variant of the two tail passes (timed together on scratch buffers: the
    statistics pass, then the apply pass with placeholder coefficients)."""
    C = _native()
    dev = a2.device

    def make(v):
        def fn():
            part = torch.empty(_part_rows(M, cout, v, h, w, 1), 2, cout, device=dev, dtype=torch.float32)
            if C.convn_(a2, w2, part, 1, 1, 1, 0, part=part, shift=shift, variant=v, no_store=True) == 0:
                raise _at.Declined("convn statistics-only pass")
            out = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
            ss = torch.zeros(2 * cout, device=dev, dtype=torch.float32)
            mb = torch.empty(M * cout // 8, device=dev, dtype=torch.uint8)
            if C.convn_(a2, w2, out, 1, 1, 1, 0, variant=v, apply_ss=ss, apply_res=out, apply_mask=mb) == 0:
                raise _at.Declined("convn apply pass")
            return out
        return fn

    cands = {f"psdn{v}": make(v) for v in range(C.convn_variants(cout))
             if C.convn_variant_kind(cout, v) in (0, 3) and C.convn_variant_ok(cout, v, 1, 1, 1, 0, w)}
    how = _at.choose(("tail", "conv1x1_bn_res_relu", M, cin, cout), cands, next(iter(cands)))
    return int(how[4:])


def _stats_route(a2, w2, M: int, cin: int, cout: int, v: int, h: int, w: int, shift) -> str:
    """The tail's statistics: "gram" (one pass over a2 for its Gram matrix and column sums, then
    W^T G W per channel: kernels/bnfold.hip gram stats) or "pass" (the narrow kernel's
    statistics-only pass recomputing the GEMM), timed per shape. The Gram statistics are those of the
    fp32 product, the pass's those of the bf16-rounded one (what the apply pass normalises)."""
    C = _native()
    if not _feat("tail_gram") or C.convw_gram_rows(cin) <= 0 or cout % 4:
        return "pass"
    dev = a2.device

    def gram():
        P = torch.empty(C.convw_gram_rows(cin), cin, device=dev, dtype=torch.float32)
        if not C.convw_gram_(a2, P):
            raise _at.Declined("convw Gram launch")
        row = torch.empty(2, cout, device=dev, dtype=torch.float32)
        C.bnfold_gram_stats(P, w2, shift, M, row)
        return row

    def pas():
        part = torch.empty(_part_rows(M, cout, v, h, w, 1), 2, cout, device=dev, dtype=torch.float32)
        rows = C.convn_(a2, w2, part, 1, 1, 1, 0, part=part, shift=shift, variant=v, no_store=True)
        if rows == 0:
            raise _at.Declined("convn statistics-only pass")
        return part[:rows].sum(0)  # comparable with the Gram row (same shifted sums)

    return _at.choose(("tail", "stats", M, cin, cout), {"gram": gram, "pass": pas}, "pass")


class _TailFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a2, weight, gamma, beta, idt, conv, bn, resid_to):
        C = _native()
        n, cin, h, w = a2.shape
        cout = weight.shape[0]
        M = n * h * w
        w2 = weight.reshape(cout, cin)
        if not w2.is_contiguous():
            w2 = w2.contiguous()
        v = _variant(a2, w2, M, cin, cout, h, w, bn.running_mean)
        if _stats_route(a2, w2, M, cin, cout, v, h, w, bn.running_mean) == "gram":
            # sum y = W s, sum y^2 = W^T G W from one read of a2 (G = a2^T a2, s = 1^T a2: the Gram
            # launch of the weight-gradient kernel) -- the GEMM is not recomputed for the statistics
            P = torch.empty(C.convw_gram_rows(cin), cin, device=a2.device, dtype=torch.float32)
            if not C.convw_gram_(a2, P):
                raise RuntimeError("psd tail: convw declined the Gram launch")
            part = torch.empty(1, 2, cout, device=a2.device, dtype=torch.float32)
            C.bnfold_gram_stats(P, w2, bn.running_mean, M, part[0])
            rows = 1
        else:
            part = torch.empty(_part_rows(M, cout, v, h, w, 1), 2, cout, device=a2.device, dtype=torch.float32)
            rows = C.convn_(a2, w2, part, 1, 1, 1, 0, part=part, shift=bn.running_mean, variant=v, no_store=True)
            if rows == 0:
                raise RuntimeError("psd tail: convn declined the statistics-only pass")
        mean, invstd, ss = C.bn_finalize(part, rows, M, gamma, beta, bn.running_mean, bn.running_var,
                                         bn.momentum if bn.momentum is not None else 0.1, bn.eps,
                                         bn.num_batches_tracked)
        out = torch.empty(M, cout, device=a2.device, dtype=torch.bfloat16)
        mbits = torch.empty(M * cout // 8, device=a2.device, dtype=torch.uint8)
        if C.convn_(a2, w2, out, 1, 1, 1, 0, variant=v, apply_ss=ss, apply_res=idt, apply_mask=mbits) == 0:
            raise RuntimeError("psd tail: convn declined the apply pass")
        y = _from_2d(out, n, h, w)
        # the consumer convolution's bwd-data epilogue runs this BN's backward reduction without its
        # input (bx None: ops/conv.py _bn_bwd_fusion / _dgrad_route)
        bn._psd_fwd = (y, None, mean, ss, mbits, None, None)
        ctx.mod = conv
        _fwd_records(ctx, conv)
        ctx.bn, ctx.resid_to, ctx.v = bn, resid_to, v
        ctx.save_for_backward(a2, weight, gamma, mean, invstd, mbits)
        TAIL_CALLS["fwd"] += 1
        return y

    @staticmethod
    def backward(ctx, dy):
        a2, weight, gamma, mean, invstd, mbits = ctx.saved_tensors
        C = _native()
        bn = ctx.bn
        bn._psd_fwd = None
        n, cin, h, w = a2.shape
        cout = weight.shape[0]
        M = n * h * w
        sink = getattr(bn, "_psd_grad_sink", None)
        dgo = dbo = None
        if sink is not None:
            dgo, dbo = sink(bn.weight), sink(bn.bias)
        pre = getattr(bn, "_psd_bwd_pre", None)
        bn._psd_bwd_pre = None
        if pre is not None and not (len(pre) == 3 and pre[0].data_ptr() == dy.data_ptr() and pre[0].shape == dy.shape):
            pre = None
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if pre is not None:
            # g = mask (dX + dr) and its partials (sum g, -mean sum g) from the consumer's epilogue
            g, part, rows = pre
            if part.shape[0] <= rows:
                raise RuntimeError("psd tail: the partials buffer has no row for sum g y")
            P = torch.empty(C.convw_fold_rows(cout, cin), cin, device=dy.device, dtype=torch.float32)
            if not C.convw_(g, a2, P, 1, 1, 1, 0, fold=True):
                raise RuntimeError("psd tail: convw_ declined the fold wgrad")
            C.bnfold_rowdot(P, weight, part[rows])
            g, coef, dg, db = C.bn_bwd_coef(g, g, gamma, mean, invstd, part=part, rows=rows + 1, dgamma_out=dgo,
                                            dbeta_out=dbo)
            y = None
            TAIL_CALLS["bwd_fused"] += 1
        else:
            # no fused consumer: recompute y3 once and run the ordinary BN backward (+ fold)
            P = None
            w2 = weight.reshape(cout, cin).contiguous()
            out = torch.empty(M, cout, device=dy.device, dtype=torch.bfloat16)
            if C.convn_(a2, w2, out, 1, 1, 1, 0, variant=ctx.v) == 0:
                raise RuntimeError("psd tail: convn declined the recompute")
            y = _from_2d(out, n, h, w)
            dy2 = take_dr(bn._psd_pending_dr.pop()) if getattr(bn, "_psd_pending_dr", None) else None
            g, coef, dg, db = C.bn_bwd_coef(dy, y, gamma, mean, invstd, mbits=mbits, dy2=dy2, dgamma_out=dgo,
                                            dbeta_out=dbo)
            TAIL_CALLS["bwd_recompute"] += 1
        res_grad = None
        if ctx.resid_to is not None:
            ctx.resid_to._psd_pending_dr.append(g)
        else:
            res_grad = g
        dx, dw, dyu = _fold_backward(ctx, (g, coef, y), a2, weight, need_x, need_w, P=P)
        if dyu is not None:  # (y present and the unfolded path won): the ordinary conv backward on dy
            conv_bwd = torch.ops.aten.convolution_backward
            args = (None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1)
            dx, dw, _ = conv_bwd(dyu, a2, weight, *args, [need_x, need_w, False])
            sv = _sink_view(ctx.mod, weight)
            if dw is not None and sv is not None:
                dw = sv.copy_(dw)
        return dx, dw, dg, db, res_grad, None, None, None


def conv_bn_tail(conv, bn, a2: torch.Tensor, idt: torch.Tensor, resid_to=None) -> torch.Tensor:
    """``relu(bn(conv(a2)) + idt)`` with conv's output never stored (see module docstring).
    ``resid_to``: the fused BN that produced ``idt`` (the residual gradient is handed to it)."""
    return _TailFn.apply(a2, conv.weight, bn.weight, bn.bias, idt, conv, bn, resid_to)
