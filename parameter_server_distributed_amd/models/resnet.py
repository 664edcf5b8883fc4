"""ResNet-50 / ResNet-101 / Wide-ResNet-101-2 (v1.5 bottleneck: stride on the 3x3 conv).

The worker model for the BASELINE.json ResNet configs (the reference itself has no model: its
"gradient" is the constant 0.01 on a dummy [10,10] tensor, src/worker.cpp:316-329,346-353).

MI355X layout choices: NHWC (``channels_last``) activations and weights, bf16 compute, the stem
on our own gfx950 kernels (ops/conv.py), every BatchNorm (+ residual + ReLU) on the fused NHWC
kernels (ops/bn.py), 1x1 convolutions routed per shape between MIOpen and hipBLASLt, the 3x3 and
strided convolutions between MIOpen and our implicit-GEMM MFMA kernel (ops/conv.py); with
``fp8=True`` (the Wide-ResNet-101-2 config, "CDNA4 fp8 MFMA") the bottleneck convolutions' forward
runs on e4m3 operands through the fp8 GEMM / implicit-GEMM kernels. The 1000-way
classifier is a plain ``nn.Linear`` (hipBLASLt; 0.02 ms of an 89 ms step). Random init, synthetic
data.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops.bn import FusedBatchNorm2d, bn_add_bn_relu
from ..ops.conv import Conv1x1, ConvNHWC, stem_forward
from ..ops.pool import MaxPool3x3s2, global_avg_pool
from ..ops.tail import conv_bn_dual_tail, conv_bn_tail, dual_tail_ok, tail_ok
from ..utils.config import feature as _feat


class _Fork(torch.autograd.Function):
    """Two aliases of a block input for its two consumers (conv1 and the downsample conv). Autograd
    hands their gradients to backward separately; the downsample-branch one is passed to the fused
    BN (or the stem max-pool) that produced the input and added inside its backward kernels,
    instead of by an autograd add kernel over the whole activation. Ordering is by construction:
    this node's backward runs before the producer's, which consumes the gradient it returns."""

    @staticmethod
    def forward(ctx, x, bn):
        ctx.bn = bn
        return x.view_as(x), x.view_as(x)

    @staticmethod
    def backward(ctx, g_main, g_ds):
        if g_ds is not None and g_ds.dim() > 0 and all(st == 0 for st in g_ds.stride()):
            g_ds = None  # the downsample conv queued its quarter-grid gradient itself (ops/conv.py)
        if g_main is None or g_ds is None:
            if g_main is None and g_ds is None:
                return None, None
            return (g_ds if g_main is None else g_main), None
        ctx.bn._psd_pending_dr.append(g_ds)
        return g_main, None


def _conv(cin, cout, k, stride=1, groups=1, fp8=False):
    if k == 1 and stride == 1 and groups == 1:
        return Conv1x1(cin, cout, fp8=fp8)  # per-shape MIOpen / hipBLASLt / MFMA GEMM (ops/conv.py)
    if groups == 1:
        return ConvNHWC(cin, cout, k, stride, fp8=fp8)  # per-shape MIOpen / implicit-GEMM MFMA kernel (ops/conv.py)
    return nn.Conv2d(cin, cout, k, stride=stride, padding=k // 2, groups=groups, bias=False)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride=1, width_per_group=64, downsample=None, fp8=False):
        super().__init__()
        width = int(planes * (width_per_group / 64.0))
        # BN + ReLU (+ residual) run as one fused NHWC kernel family (ops/bn.py)
        self.conv1 = _conv(cin, width, 1, fp8=fp8)
        self.bn1 = FusedBatchNorm2d(width, relu=True)
        self.conv2 = _conv(width, width, 3, stride, fp8=fp8)
        self.bn2 = FusedBatchNorm2d(width, relu=True)
        self.conv3 = _conv(width, planes * self.expansion, 1, fp8=fp8)
        self.bn3 = FusedBatchNorm2d(planes * self.expansion, relu=True)  # relu(bn3(conv3) + identity)
        self.downsample = downsample
        self.fuse_residual_grad = True
        # each convolution's consumer BN: the conv epilogue can reduce its batch statistics
        # (ops/conv.py, kernels/convn.hip); plain attributes, not submodules
        for conv, bn in ((self.conv1, self.bn1), (self.conv2, self.bn2), (self.conv3, self.bn3)):
            object.__setattr__(conv, "_psd_bn", bn)
        if downsample is not None and len(downsample) == 2:
            object.__setattr__(downsample[0], "_psd_bn", downsample[1])
        # the BN whose output each convolution consumes (its backward reduction can run in the
        # convolution's bwd-data epilogue); conv1's is set per forward (identity blocks only)
        object.__setattr__(self.conv2, "_psd_bn_in", self.bn1)
        object.__setattr__(self.conv3, "_psd_bn_in", self.bn2)
        object.__setattr__(self.conv1, "_psd_bn_in", None)
        # bn3's input gradient can be folded into conv3's backward GEMMs (ops/conv.py _fold_backward)
        if isinstance(self.conv1, Conv1x1) and not fp8:
            # bn1's into conv1 (when conv2's bwd-data epilogue pre-reduced it: ops/bn.py)
            object.__setattr__(self.bn1, "_psd_fold_conv", self.conv1)
        # fp8 identity blocks (feature tail_fp8): conv3 + bn3 run as the bf16 recomputing tail
        # (ops/tail.py) -- bn3's input gradient folded into conv3's bf16 backward, conv3's output never
        # stored -- so bn2 writes no e4m3 copy for conv3 and bn3 none of its input gradient
        self._tail8 = bool(fp8 and downsample is None and isinstance(self.conv3, Conv1x1) and _feat("tail_fp8"))
        if isinstance(self.conv3, Conv1x1) and (not fp8 or self._tail8):
            object.__setattr__(self.bn3, "_psd_fold_conv", self.conv3)
            # and a stride-1 downsample BN's into the downsample conv (layer 1's first block)
            if downsample is not None and len(downsample) == 2 and isinstance(downsample[0], Conv1x1):
                object.__setattr__(downsample[1], "_psd_fold_conv", downsample[0])
        if fp8:  # bn1 / bn2 quantise their outputs for the fp8 conv2 / conv3 in their apply pass
            # (plain attributes: object.__setattr__ keeps the consumer from becoming a submodule)
            object.__setattr__(self.bn1, "_psd_q8_consumer", self.conv2)
            if not self._tail8:
                object.__setattr__(self.bn2, "_psd_q8_consumer", self.conv3)
            # and each BN's backward quantises its input gradient for the producing conv's fp8 bwd-data
            for conv, bn in ((self.conv1, self.bn1), (self.conv2, self.bn2), (self.conv3, self.bn3)):
                if conv is self.conv3 and self._tail8:
                    continue
                if hasattr(conv, "psd_fp8_dgrad"):
                    object.__setattr__(bn, "_psd_dq8_producer", conv)

    def forward(self, x, prev_bn=None):
        """``prev_bn``: the fused BN that produced ``x`` (the previous block's bn3). The second
        gradient of ``x`` -- the identity residual's, or the downsample conv's -- is then handed to
        it inside the BN kernels (no autograd add over the activation)."""
        xm = xd = x
        forked = False
        if (self.downsample is not None and prev_bn is not None and self.fuse_residual_grad
                and torch.is_grad_enabled() and x.requires_grad and prev_bn.training and x.is_cuda
                and x.dtype == torch.bfloat16):  # (the fused BN kernels that consume the hand-over)
            xm, xd = _Fork.apply(x, prev_bn)  # downsample-branch gradient -> prev_bn's kernels
            forked = True
        if self.downsample is not None and self.fuse_residual_grad and len(self.downsample) == 2:
            # relu(bn3(conv3) + bn_ds(conv_ds)): the downsample BN is applied inside bn3's apply pass.
            # The downsample conv runs last: autograd then runs its backward before conv1's, so a
            # stride-2 one can queue its quarter-grid input gradient for conv1's bwd-data epilogue
            # (ops/conv.py _strided_dgrad, kernels/convn.hip mode 5)
            to = prev_bn if forked and isinstance(prev_bn, FusedBatchNorm2d) else None
            # conv1's bwd-data may then run prev_bn's backward reduction with that gradient added
            object.__setattr__(self.conv1, "_psd_bn_in", to if self.fuse_residual_grad else None)
            a2 = self.bn2(self.conv2(self.bn1(self.conv1(xm))))
            object.__setattr__(self.downsample[0], "_psd_strided_to", to)
            if dual_tail_ok(self.conv3, self.bn3, a2, self.downsample[0], self.downsample[1], xd):
                # 1x1 downsample of stride 1 or 2 (layers 1-2): neither conv3's nor the downsample
                # conv's output is stored -- Gram statistics, one K-concatenated apply GEMM (ops/tail.py)
                return conv_bn_dual_tail(self.conv3, self.bn3, a2, self.downsample[0], self.downsample[1], xd)
            y3 = self.conv3(a2)
            r = self.downsample[0](xd)
            return bn_add_bn_relu(self.bn3, y3, self.downsample[1], r)
        idt = x if self.downsample is None else self.downsample(xd)
        # identity block: x (prev_bn's output) feeds conv1 and the residual, whose gradient is handed
        # to prev_bn -- conv1's bwd-data can run prev_bn's backward reduction
        object.__setattr__(self.conv1, "_psd_bn_in",
                           prev_bn if (self.fuse_residual_grad and isinstance(prev_bn, FusedBatchNorm2d)) else None)
        out = self.bn1(self.conv1(xm))
        out = self.bn2(self.conv2(out))
        fuse = prev_bn if (self.downsample is None and self.fuse_residual_grad) else None
        if self.downsample is None and tail_ok(self.conv3, self.bn3, out, idt):
            # conv3's output is never stored: statistics pass + apply pass, recomputed (ops/tail.py)
            return conv_bn_tail(self.conv3, self.bn3, out, idt, fuse)
        return self.bn3(self.conv3(out), idt, resid_grad_to=fuse)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, width_per_group=64, zero_init_residual=True,
                 fp8=False):
        """``fp8``: bottleneck convolutions run their forward on e4m3 operands (fp8 MFMA GEMM /
        implicit GEMM, per-tensor scales) and their backward in bf16, where the shape allows
        (ops/conv.py); the stem and the classifier stay bf16."""
        super().__init__()
        self.fp8 = fp8
        self.width_per_group = width_per_group
        self.cin = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = FusedBatchNorm2d(64, relu=True)
        self.maxpool = MaxPool3x3s2()
        self.layer1 = self._make(64, layers[0])
        self.layer2 = self._make(128, layers[1], stride=2)
        self.layer3 = self._make(256, layers[2], stride=2)
        self.layer4 = self._make(512, layers[3], stride=2)
        self.fc = nn.Linear(512 * Bottleneck.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):  # includes FusedBatchNorm2d
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
        if fp8:  # each block's bn3 quantises the block output for the next block's fp8 conv1
            blocks = [b for layer in (self.layer1, self.layer2, self.layer3, self.layer4) for b in layer]
            for prev, nxt in zip(blocks, blocks[1:]):
                object.__setattr__(prev.bn3, "_psd_q8_consumer", nxt.conv1)

    def _make(self, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.cin != planes * Bottleneck.expansion:
            down = nn.Sequential(_conv(self.cin, planes * Bottleneck.expansion, 1, stride, fp8=self.fp8),
                                 FusedBatchNorm2d(planes * Bottleneck.expansion))
        mods = [Bottleneck(self.cin, planes, stride, self.width_per_group, down, fp8=self.fp8)]
        self.cin = planes * Bottleneck.expansion
        for _ in range(1, blocks):
            mods.append(Bottleneck(self.cin, planes, 1, self.width_per_group, fp8=self.fp8))
        return nn.Sequential(*mods)

    def forward(self, x):
        x = stem_forward(self.conv1, self.bn1, self.maxpool, x)  # conv + BN + ReLU + pool, fused on gfx950
        # the first bottleneck's downsample-branch gradient goes to the max-pool's backward kernel
        prev = self.maxpool if self.maxpool.native_last else None
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in layer:
                x = blk(x, prev)
                prev = blk.bn3
        return self.fc(global_avg_pool(x))


def resnet50(num_classes=1000, fp8=False):
    return ResNet((3, 4, 6, 3), num_classes, fp8=fp8)


def resnet101(num_classes=1000, fp8=False):
    return ResNet((3, 4, 23, 3), num_classes, fp8=fp8)


def wide_resnet101_2(num_classes=1000, fp8=False):
    return ResNet((3, 4, 23, 3), num_classes, width_per_group=128, fp8=fp8)
