"""Fused NHWC BatchNorm2d (+ residual add) (+ ReLU) on the gfx950 kernels of ``csrc/kernels/bn.hip``.

``FusedBatchNorm2d`` is a drop-in ``nn.BatchNorm2d`` whose forward also takes an optional residual
and applies ReLU in the same pass; backward fuses the ReLU mask, the residual-branch gradient and
the BN input gradient. Running statistics are fp32 (the kernels also use them as the variance
shift), parameters are whatever dtype the PS data plane gives them (bf16 views).

Grad sink: when the PS data plane owns the parameters it installs ``_psd_grad_sink`` on the
module; backward then writes dgamma/dbeta straight into the flat gradient buffer (no separate
accumulate kernel) and returns those views, which autograd's AccumulateGrad adopts.

Device tensors that are not bf16 or whose channel count is not a multiple of 8 -- and every CPU
tensor -- take the reference composite path (fp32 ``F.batch_norm``), which is also what the tests
compare the kernels against.
"""
from __future__ import annotations


import torch
import torch.nn as nn
import torch.nn.functional as F

from ..utils.config import feature as _feat
from .. import native


def _kernel_ok(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype == torch.bfloat16 and x.dim() in (2, 4) and x.shape[1] % 8 == 0


def _q8_args(mod, x: torch.Tensor) -> dict:
    """If ``mod``'s output feeds an MX fp8 convolution (``_psd_q8_consumer``, wired by the model), the
    apply pass also writes the e4m3 copy + one E8M0 scale per 32 channels (a lane quad's block
    maximum, kernels/bn.hip Q8 == 2) -- the consumer's own quantise pass (a full read of y) never
    runs. Per-tensor operands (feature fp8_mx off) are quantised by the consumer with its delayed
    scale: a per-tensor hand-over from this pass measured no faster (WRN-101-2 b512 3,589 vs 3,606
    img/s) and was removed in round 6. feature fp8_mx_handover off: the consumer quantises."""
    cons = getattr(mod, "_psd_q8_consumer", None)
    if cons is None or not mod.relu or x.dim() != 4 or not cons.psd_fp8_consumes(x.shape[1]):
        return {}
    if not _feat("fp8_mx") or x.shape[1] % 32 or not _feat("fp8_mx_handover"):
        return {}
    q = torch.empty_like(x, dtype=torch.float8_e4m3fn, memory_format=torch.channels_last)
    return {"q8_out": q, "q8_mx": torch.empty(x.numel() // 32, dtype=torch.uint8, device=x.device)}


def _stats_args(mod, x: torch.Tensor) -> dict:
    """The batch-statistics partials the producing convolution reduced in its epilogue for exactly
    this tensor (ops/conv.py, kernels/convn.hip), as bn_fwd arguments; consumed once."""
    pend = getattr(mod, "_psd_stats_pending", None)
    if pend is None:
        return {}
    mod._psd_stats_pending = None
    y, part, rows = pend
    if y.data_ptr() != x.data_ptr() or y.shape != x.shape or y.stride() != x.stride():
        return {}
    return {"part_in": part, "part_rows": rows}


def _dq8_args(mod, x: torch.Tensor) -> dict:
    """If ``mod``'s input gradient is the output gradient of an fp8 convolution that runs its
    bwd-data in fp8 (``_psd_dq8_producer``, wired by the model), the BN's elementwise backward pass
    also writes the MX e5m2 copy of it (kernels/bn.hip bn_bwd_elemt_kernel DQ): the convolution's own
    quantise pass (a full read of dY) never runs."""
    prod = getattr(mod, "_psd_dq8_producer", None)
    if (prod is None or x.dim() != 4 or x.shape[1] % 32 or not _feat("fp8_mx")
            or not _feat("fp8_mx_handover") or not prod.psd_fp8_dgrad()):
        return {}
    q = torch.empty_like(x, dtype=torch.float8_e5m2, memory_format=torch.channels_last)
    return {"dq": q, "dqmx": torch.empty(x.numel() // 32, dtype=torch.uint8, device=x.device)}


def _dq8_hand_over(mod, dx: torch.Tensor, kw: dict) -> None:
    if kw:
        mod._psd_dq8_producer._psd_dq8_pending = (dx, kw["dq"], kw["dqmx"])


def _q8_hand_over(mod, y: torch.Tensor, kw: dict) -> None:
    if kw:  # (y, e4m3 copy, its MX scales uint8 [numel / 32])
        mod._psd_q8_consumer._psd_q8_pending = (y, kw["q8_out"], kw["q8_mx"])


class StridedDr:
    """A residual-branch gradient handed to a BN (``_psd_pending_dr``) by a stride-2 1x1 (downsample)
    convolution, kept on its quarter grid: ``t4`` = dY . W of the strided positions, [N, C, H/2, W/2]
    channels_last. The full-size gradient is zero except at even (h, w); the consumer convolution's
    bwd-data epilogue adds it there (kernels/convn.hip bwd mode 5) and only other consumers build the
    full tensor (``full``)."""

    def __init__(self, t4: torch.Tensor, H: int, W: int):
        self.t4, self.H, self.W = t4, H, W

    def full(self) -> torch.Tensor:
        n, c = self.t4.shape[:2]
        out = torch.zeros(n, self.H, self.W, c, device=self.t4.device, dtype=self.t4.dtype).permute(0, 3, 1, 2)
        out[:, :, ::2, ::2] = self.t4
        return out


def take_dr(t):
    """A pending residual gradient as a full-size tensor (StridedDr materialised)."""
    return t.full() if isinstance(t, StridedDr) else t


def _fold_target(mod, x: torch.Tensor):
    """The 1x1 convolution whose output ``x`` this BN consumed and whose backward can take the BN's
    input gradient folded (ops/conv.py _fold_backward, kernels/bnfold.hip), or None. The convolution
    records the output it produced through its fold-aware Function; a mismatch (another producer, a
    stale record) means no fold."""
    conv = getattr(mod, "_psd_fold_conv", None)
    if conv is None or not _feat("bn_fold"):
        return None
    rec = getattr(conv, "_psd_fold_out", None)
    if rec is None or rec[0] != x.data_ptr() or rec[1] != tuple(x.shape):
        return None
    return conv


def _hand_fold(conv, g, coef, x, P=None):
    """Give ``conv``'s backward what replaces the BN input gradient: (g, coef, the BN input[, the
    fold wgrad products [g | x | 1]^T x_in already taken])."""
    conv._psd_fold_out = None
    conv._psd_fold_x = None
    conv._psd_fold_pending = (g, coef, x) if P is None else (g, coef, x, P)


def _fold_pair_ok(bn3, x, bnd, r):
    """Both tail BNs fold into stride-1 1x1 convolutions whose fold wgrad takes their whole input:
    the dual tail can then take sum g y3 / sum g yd from g^T a2 / g^T x_in (rowdot) instead of
    reading y3 / yd in the consumer's epilogue. Returns (conv3, convd) or None."""
    if not (_feat("bn_fold_ds") and _feat("dual_nobx")):
        return None
    c3, cd = _fold_target(bn3, x), _fold_target(bnd, r)
    if c3 is None or cd is None:
        return None
    C = native()
    for conv in (c3, cd):
        xin = getattr(conv, "_psd_fold_x", None)
        if xin is None or not xin.is_contiguous(memory_format=torch.channels_last) \
                or C.convw_fold_rows(conv.weight.shape[0], conv.weight.shape[1]) <= 0:
            return None
    return c3, cd


class _FusedBNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, mod, resid_to=None):
        C = native()
        has_res = residual is not None
        q8 = _q8_args(mod, x)
        y, mean, invstd, ss, mbits = C.bn_fwd(x, weight, bias, mod.running_mean, mod.running_var, residual, mod.relu,
                                              True, mod.momentum if mod.momentum is not None else 0.1, mod.eps,
                                              mod.num_batches_tracked, None, mask_out=mod.relu and has_res, **q8,
                                              **_stats_args(mod, x))
        _q8_hand_over(mod, y, q8)
        # for the consumer convolution's bwd-data epilogue (ops/conv.py _bn_bwd_fusion): ReLU BNs
        mod._psd_fwd = (y, x, mean, ss, mbits if has_res else None, None, None) if mod.relu else None
        ctx.relu = mod.relu
        ctx.has_res = residual is not None
        ctx.mod = mod
        ctx.resid_to = resid_to
        # ReLU mask for backward: without a residual it is recomputed from x and the fp32
        # scale/shift (one [M, C] read less per backward pass); with one, the forward kernel wrote
        # it as a bit-mask (1/16 of y's bytes)
        ctx.save_for_backward(x, mbits if mod.relu and has_res else None, weight, mean, invstd,
                              ss if (mod.relu and not has_res) else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mbits, w, mean, invstd, ss = ctx.saved_tensors
        mod = ctx.mod
        mod._psd_fwd = None
        sink = getattr(mod, "_psd_grad_sink", None)
        dgo = dbo = None
        if sink is not None and w is not None:
            dgo, dbo = sink(mod.weight), sink(mod.bias)
        pre = getattr(mod, "_psd_bwd_pre", None)
        mod._psd_bwd_pre = None
        if pre is not None and not (pre[0].data_ptr() == dy.data_ptr() and pre[0].shape == dy.shape):
            pre = None
        # a residual BN (bn3) folds into its producing 1x1 convolution (its stored mask or the partials
        # the consumer's bwd-data epilogue pre-reduced). (bn1 folded into conv1 measured slower -- 70.9
        # vs 68.0 ms/step, profiles/r5/ab_bn1_fold.md -- and was removed in round 6.)
        foldable = ctx.relu and w is not None and ctx.has_res and mbits is not None
        conv = _fold_target(mod, x) if foldable else None
        if conv is not None:
            # BN-backward fold: reduction + finalize only; the producing 1x1 convolution's dgrad / wgrad
            # take g and the coefficients (no elementwise pass, no input-gradient tensor)
            if pre is not None:
                g, coef, dg, db = native().bn_bwd_coef(pre[0], x, w, mean, invstd, part=pre[1], rows=pre[2],
                                                       dgamma_out=dgo, dbeta_out=dbo)
            else:
                dy2 = take_dr(mod._psd_pending_dr.pop()) if getattr(mod, "_psd_pending_dr", None) else None
                g, coef, dg, db = native().bn_bwd_coef(dy, x, w, mean, invstd, mbits=mbits, dy2=dy2, dgamma_out=dgo,
                                                       dbeta_out=dbo)
            _hand_fold(conv, g, coef, x)
            res_grad = None
            if ctx.has_res:
                if ctx.resid_to is not None:
                    ctx.resid_to._psd_pending_dr.append(g)
                else:
                    res_grad = g
            return g, dg, db, res_grad, None, None
        if pre is not None:
            # the consumer convolution's bwd-data epilogue reduced this BN's backward and wrote the
            # masked gradient g (= the residual-branch gradient for a residual BN): finalize + one
            # elementwise pass here
            g, part, rows = pre
            dq8 = _dq8_args(mod, x)
            dx, dg, db = native().bn_bwd_pre(g, x, w, mean, invstd, part, rows, dgo, dbo, **dq8)
            _dq8_hand_over(mod, dx, dq8)
            res_grad = None
            if ctx.has_res:
                if ctx.resid_to is not None:
                    ctx.resid_to._psd_pending_dr.append(g)
                else:
                    res_grad = g
            return dx, (dg if w is not None else None), (db if w is not None else None), res_grad, None, None
        # residual-branch fusion: the identity-path gradient of this BN's output was stashed by the
        # next block's bn3 backward; fold it in here instead of an autograd add kernel
        dy2 = take_dr(mod._psd_pending_dr.pop()) if getattr(mod, "_psd_pending_dr", None) else None
        dq8 = _dq8_args(mod, x)
        dx, dr, dg, db = native().bn_bwd(dy, x, None, w, mean, invstd, ctx.relu, ctx.has_res, dgo, dbo, dy2, ss,
                                         mbits, **dq8)
        _dq8_hand_over(mod, dx, dq8)
        res_grad = None
        if ctx.has_res:
            if ctx.resid_to is not None:
                ctx.resid_to._psd_pending_dr.append(dr)
            else:
                res_grad = dr
        return dx, (dg if w is not None else None), (db if w is not None else None), res_grad, None, None


class _BNAddBNReluFn(torch.autograd.Function):
    """``relu(bn3(x) + bnd(r))`` -- a bottleneck's tail when the residual is the downsample branch
    (conv -> BN). The downsample BN only reduces its statistics; its scale/shift is applied to r
    inside bn3's apply kernel, so the downsample BN output (a full [M, C] write and read) never
    exists. Backward: both BNs in one reduce pass and one elementwise pass (the downsample BN's
    upstream gradient is bn3's residual gradient dr)."""

    @staticmethod
    def forward(ctx, x, w3, b3, r, wd, bd, bn3, bnd):
        C = native()
        mom = lambda m: m.momentum if m.momentum is not None else 0.1  # noqa: E731
        _, mean_d, invstd_d, ss_d, _ = C.bn_fwd(r, wd, bd, bnd.running_mean, bnd.running_var, None, False, True,
                                                mom(bnd), bnd.eps, bnd.num_batches_tracked, None, stats_only=True,
                                                **_stats_args(bnd, r))
        q8 = _q8_args(bn3, x)
        y, mean, invstd, _, mbits = C.bn_fwd(x, w3, b3, bn3.running_mean, bn3.running_var, r, True, True, mom(bn3),
                                             bn3.eps, bn3.num_batches_tracked, None, mask_out=True, residual_ss=ss_d,
                                             **q8, **_stats_args(bn3, x))
        _q8_hand_over(bn3, y, q8)
        # for the consumer convolution's bwd-data epilogue (ops/conv.py _bn_bwd_fusion, mode 3): both
        # BNs' backward reductions ride on it. With both BNs folded (layer 1) the epilogue reduces
        # only sum g (mode 2 without the BN input) and backward completes sum g y3 / sum g yd from
        # the fold products: y3 and yd are not read there
        pair = _fold_pair_ok(bn3, x, bnd, r)
        ctx.pair = None if pair is None else (pair[0], pair[1], pair[0]._psd_fold_x, pair[1]._psd_fold_x)
        bn3._psd_fwd = (y, x, mean, None, mbits, r, mean_d) if pair is None else (y, None, mean, None, mbits, None, None)
        ctx.bn3, ctx.bnd = bn3, bnd
        ctx.save_for_backward(x, mbits, w3, mean, invstd, r, wd, mean_d, invstd_d)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mbits, w3, mean, invstd, r, wd, mean_d, invstd_d = ctx.saved_tensors
        bn3, bnd = ctx.bn3, ctx.bnd
        C = native()

        def sinks(m):
            sink = getattr(m, "_psd_grad_sink", None)
            return (sink(m.weight), sink(m.bias)) if sink is not None else (None, None)

        dg3o, db3o = sinks(bn3)
        dgdo, dbdo = sinks(bnd)
        bn3._psd_fwd = None
        conv = _fold_target(bn3, x)
        pre = getattr(bn3, "_psd_bwd_pre", None)
        bn3._psd_bwd_pre = None
        pair = ctx.pair
        ctx.pair = None
        if pair is not None and pre is not None and len(pre) == 3 and pre[0].data_ptr() == dy.data_ptr() \
                and pre[0].shape == dy.shape and conv is pair[0] and _fold_target(bnd, r) is pair[1]:
            # the consumer reduced (sum g, -mean3 sum g); sum g y3 = sum_i W3 (g^T a2), sum g yd =
            # sum_i Wd (g^T x_in) from the fold wgrads taken now (and handed on, not retaken)
            g, part, rows = pre
            if part.shape[0] <= rows:
                raise RuntimeError("psd dual tail: the partials buffer has no row for sum g y")
            (c3, cd, a2, xin) = pair
            Ps = []
            for conv_, xin_ in ((c3, a2), (cd, xin)):
                P = torch.empty(C.convw_fold_rows(conv_.weight.shape[0], conv_.weight.shape[1]), xin_.shape[1],
                                device=g.device, dtype=torch.float32)
                if not C.convw_(g, xin_, P, 1, 1, 1, 0, variant=int(_feat("convw_fold2")), fold=True):
                    raise RuntimeError("psd dual tail: convw_ declined the fold wgrad")
                Ps.append(P)
            # the downsample BN's sums derive from bn3's sum g (same masked g) and its own sum g yd
            part_d = torch.empty(2, part.shape[-1], device=part.device, dtype=torch.float32)
            C.bnfold_rowdot(Ps[0], c3.weight, part[rows])
            C.bnfold_rowdot(Ps[1], cd.weight, part_d)
            _, _, dg3, db3, dgd, dbd, coef, coef_d = C.bn_bwd_dual_pre(
                g, x, w3, mean, invstd, part, part_d, rows + 1, r, wd, mean_d, invstd_d, dg3o, db3o, dgdo, dbdo,
                fold=True, fold_d=True, derive_d=True)
            _hand_fold(c3, g, coef, x, Ps[0])
            _hand_fold(cd, g, coef_d, r, Ps[1])
            return g, dg3, db3, g, dgd, dbd, None, None
        if pre is not None and len(pre) == 4 and pre[0].data_ptr() == dy.data_ptr() and pre[0].shape == dy.shape:
            # both reductions ran in the consumer convolution's bwd-data epilogue (convn mode 3): g is
            # the masked gradient incl. the residual branch; finalize both + one elementwise pass
            g, part, rows, part_d = pre
            # the downsample BN folded into its (stride-1 1x1) convolution too: no elementwise pass
            # at all -- both convolutions take g and their BN's coefficients (ops/conv.py _fold_backward)
            convd = _fold_target(bnd, r) if conv is not None and _feat("bn_fold_ds") else None
            dx, drr, dg3, db3, dgd, dbd, coef, coef_d = C.bn_bwd_dual_pre(
                g, x, w3, mean, invstd, part, part_d, rows, r, wd, mean_d, invstd_d, dg3o, db3o, dgdo, dbdo,
                fold=conv is not None, fold_d=convd is not None)
            if conv is not None:
                _hand_fold(conv, g, coef, x)
                if convd is not None:
                    _hand_fold(convd, g, coef_d, r)
                    return g, dg3, db3, g, dgd, dbd, None, None
                return g, dg3, db3, drr, dgd, dbd, None, None
            return dx, dg3, db3, drr, dgd, dbd, None, None
        dy2 = take_dr(bn3._psd_pending_dr.pop()) if getattr(bn3, "_psd_pending_dr", None) else None
        if conv is not None:  # bn3's input gradient folded into conv3's backward (see _FusedBNFn)
            _, drr, dg3, db3, dgd, dbd, coef, g = C.bn_bwd_dual(dy, x, w3, mean, invstd, mbits, dy2, r, wd, mean_d,
                                                                invstd_d, dg3o, db3o, dgdo, dbdo, fold=True)
            _hand_fold(conv, g, coef, x)
            return g, dg3, db3, drr, dgd, dbd, None, None
        # one reduce pass for both BNs (the downsample BN's upstream gradient is bn3's dr) and one
        # elementwise pass writing both input gradients (kernels/bn.hip, dual mode)
        dx, drr, dg3, db3, dgd, dbd = C.bn_bwd_dual(dy, x, w3, mean, invstd, mbits, dy2, r, wd, mean_d, invstd_d,
                                                    dg3o, db3o, dgdo, dbdo)
        return dx, dg3, db3, drr, dgd, dbd, None, None


def bn_add_bn_relu(bn3: "FusedBatchNorm2d", x: torch.Tensor, bnd: "FusedBatchNorm2d", r: torch.Tensor):
    """``relu(bn3(x) + bnd(r))`` with the downsample BN applied inside bn3's apply pass (training,
    bf16 NHWC on gfx950); anything else composes the two modules."""
    if (bn3.training and bnd.training and bn3.relu and not bnd.relu and _kernel_ok(x) and _kernel_ok(r)
            and x.shape == r.shape and x.dim() == 4 and bn3.running_mean is not None and bnd.running_mean is not None
            and bn3.weight is not None and bnd.weight is not None and bn3.weight.dtype == torch.bfloat16
            and bnd.weight.dtype == torch.bfloat16 and torch.is_grad_enabled()):
        return _BNAddBNReluFn.apply(x, bn3.weight, bn3.bias, r, bnd.weight, bnd.bias, bn3, bnd)
    return bn3(x, bnd(r))


class _BNReluPoolFn(torch.autograd.Function):
    """Stem: maxpool3x3s2(relu(bn(x))) without materialising the BN output (kernels/bn.hip)."""

    @staticmethod
    def forward(ctx, x, weight, bias, mod, pool):
        y, arg, mean, invstd, ss = native().bn_pool_fwd(x, weight, bias, mod.running_mean, mod.running_var,
                                                        mod.momentum if mod.momentum is not None else 0.1, mod.eps,
                                                        mod.num_batches_tracked)
        ctx.mod, ctx.pool = mod, pool
        ctx.save_for_backward(x, arg, weight, mean, invstd, ss)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, arg, w, mean, invstd, ss = ctx.saved_tensors
        sink = getattr(ctx.mod, "_psd_grad_sink", None)
        dgo = dbo = None
        if sink is not None:
            dgo, dbo = sink(ctx.mod.weight), sink(ctx.mod.bias)
        pend = getattr(ctx.pool, "_psd_pending_dr", None)
        gy2 = pend.pop() if pend else None  # the first bottleneck's downsample-branch gradient
        dx, dg, db = native().bn_pool_bwd(gy, gy2, arg, x, w, mean, invstd, ss, dgo, dbo)
        return dx, dg, db, None, None


def bn_relu_maxpool(bn: "FusedBatchNorm2d", pool, x: torch.Tensor) -> torch.Tensor:
    """``pool(bn(x))`` for the ResNet stem (``bn`` with ReLU, ``pool`` a 3x3/s2/p1 max-pool module
    that can take a second output gradient through ``_psd_pending_dr``). Training on gfx950 runs
    the fused kernels; everything else composes the two modules."""
    if (bn.training and bn.relu and _kernel_ok(x) and x.dim() == 4 and bn.running_mean is not None
            and bn.weight is not None and bn.weight.dtype == torch.bfloat16
            and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0 and 256 % (x.shape[1] // 8) == 0):
        pool.native_last = True
        return _BNReluPoolFn.apply(x, bn.weight, bn.bias, bn, pool)
    return pool(bn(x))


class FusedBatchNorm2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` + optional residual + optional ReLU, one fused kernel family on MI355X."""

    _psd_fp32_buffers = True  # models.prepare() keeps our running stats fp32

    def __init__(self, num_features: int, eps: float = 1e-5, momentum: float = 0.1, relu: bool = False):
        super().__init__(num_features, eps=eps, momentum=momentum)
        self.relu = relu
        self._psd_pending_dr: list = []
        self._psd_stats_pending = None  # (conv output, statistics partials, rows) from the producing conv
        self._psd_fwd = None  # (output, input, mean, scale/shift, ReLU bits) for the consumer conv's bwd fusion
        self._psd_bwd_pre = None  # (masked gradient, partials, rows) from the consumer conv's bwd-data

    def psd_direct_grad_params(self):
        return [self.weight, self.bias]

    def forward(self, x, residual=None, resid_grad_to: "FusedBatchNorm2d | None" = None):
        """``resid_grad_to``: the FusedBatchNorm2d that produced ``residual``. Its gradient is then
        handed to that module's backward directly (fused into its kernels) and ``residual`` is used
        detached -- the caller guarantees the residual has no other consumer needing autograd."""
        if self.training and _kernel_ok(x) and self.running_mean is not None:
            if resid_grad_to is not None and residual is not None and torch.is_grad_enabled() \
                    and isinstance(resid_grad_to, FusedBatchNorm2d) and resid_grad_to.training \
                    and _kernel_ok(residual) and residual.requires_grad:
                return _FusedBNFn.apply(x, self.weight, self.bias, residual.detach(), self, resid_grad_to)
            return _FusedBNFn.apply(x, self.weight, self.bias, residual, self)
        if not self.training and _kernel_ok(x) and self.running_mean is not None:
            scale = self.weight.float() * torch.rsqrt(self.running_var + self.eps)
            shift = self.bias.float() - self.running_mean * scale
            ss = torch.cat([scale, shift]).contiguous()
            if torch.is_grad_enabled() and (x.requires_grad or self.weight.requires_grad):
                return self._reference(x, residual)
            return native().bn_fwd(x, None, None, None, None, residual, self.relu, False, 0.0, self.eps, None, ss)[0]
        return self._reference(x, residual)

    def _reference(self, x, residual=None):
        """fp32 composite (CPU / odd shapes / eval-with-grad): numerics reference for the kernels."""
        y = F.batch_norm(x.float(), self.running_mean, self.running_var,
                         None if self.weight is None else self.weight.float(),
                         None if self.bias is None else self.bias.float(),
                         self.training, self.momentum if self.momentum is not None else 0.1, self.eps)
        if residual is not None:
            y = y + residual.float()
        if self.relu:
            y = F.relu(y)
        return y.to(x.dtype)
