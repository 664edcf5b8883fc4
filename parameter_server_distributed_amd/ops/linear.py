"""Linear layer on the hand-written MFMA GEMM (csrc/kernels/gemm.hip).

forward   y  = act(x W^T + b)     NT GEMM, bias + ReLU/GELU fused in the epilogue (GELU keeps the
                                  pre-activation for backward)
backward  dx = dy' W              NN GEMM (W read N-major through ds_read_b64_tr_b16: no transpose)
          dW = dy'^T x            TN split-K GEMM, reduced straight into the PS flat-gradient
                                  buffer when the data plane installed a grad sink
          db = colsum(dy')        column-sum kernel (also into the sink); for GELU the activation
                                  backward and this column sum are one pass (gelu_bwd_colsum_)

fp8 (``MfmaLinear(..., fp8=True)``): the forward GEMM runs on OCP e4m3 operands with per-tensor
amax scaling (x and W quantised each step by the amax/quant kernels) on the MX-scaled
v_mfma_scale_f32_16x16x128_f8f6f4 (2x the bf16 MFMA rate); the backward GEMMs stay bf16 on the
saved bf16 x and W (fp8 forward / bf16 backward recipe). Needs in_features % 128 == 0.

Per-shape routing (ops/autotune.py): for bf16 the forward, dgrad and wgrad GEMMs are each timed
once against hipBLASLt (torch.addmm / mm; bias + activation then run as separate passes) and the
faster path is kept. Measured on BERT-base (M = 8192 tokens) hipBLASLt wins most forward / dgrad
shapes, the split-K MFMA wgrad writing straight into the PS gradient buffer stays competitive.
Feature ``linear_tune`` off pins everything to the MFMA kernels.

CPU tensors (and non-bf16 / unaligned shapes) use ``F.linear`` -- the reference the tests compare
against.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..utils.config import feature as _feat
from .. import native
from . import autotune as _at

ACTS = {None: 0, "none": 0, "relu": 1, "gelu": 2}


def _ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.shape[0] % 8 == 0
            and w.shape[1] % 8 == 0)


def _route(key: tuple, mfma, blas, out: torch.Tensor | None = None, extra: dict | None = None):
    """The fastest of the MFMA kernel(s) and hipBLASLt for this GEMM shape (ops/autotune.py); ``out``
    is the buffer every candidate writes (validated against each other on the first call);
    ``extra``: more MFMA candidates by name (e.g. "mfma_ct", the 192 x 256 transposed-store tile)."""
    if not _feat("linear_tune"):
        return mfma
    probe = (lambda: out) if out is not None else None
    cands = {"mfma": mfma, **(extra or {}), "blas": blas}
    return cands[_at.choose(("linear",) + key, cands, "mfma", probe)]


def _ct(A, B, out, bias=None, act=0, aux=None):
    """Y = B A^T (+bias)(act) on the 192 x 256 transposed-store tile (kernels/gemm.hip CT): for 768-wide
    outputs 512 tiles = 2.0 rounds on 256 CUs where the 256 x 256 tile makes 384 = 1.5 rounds."""
    if not native().gemm_ct_(A, B, out, bias, act, aux):
        raise _at.Declined("192x256 transposed-store GEMM: shape outside the kernel's contract")


def _dgrad_route(key: tuple, dy2: torch.Tensor, w: torch.Tensor, dx: torch.Tensor):
    """dX = dY . W on the fastest of: the MFMA GEMM with W read N-major (NN), the MFMA GEMM on a
    transposed copy of W (NT: both operands K-major, the kernel's fastest layout; the copy is
    |W| bytes), or hipBLASLt -- timed and validated once per shape (ops/autotune.py)."""
    C = native()

    def nn_():
        C.gemm_(dy2, w, True, False, dx)

    def nt_():
        C.gemm_(dy2, w.t().contiguous(), True, True, dx)

    def blas():
        torch.mm(dy2, w, out=dx)

    def sk():  # split-K (fp32 slabs + reduce): a long K over few output tiles (the MLM head's dgrad,
        # K = 30,528 against 19 x 3 256-tiles, ran one K-loop per tile on 57 of 256 CUs)
        C.gemm_splitk_(dy2, w, True, False, dx)

    def ct():  # dX = dY W on the 192 x 256 transposed-store tile: A = W^T [in, out], B = dY [tokens, out]
        _ct(w.t().contiguous(), dy2, dx)

    if not _feat("linear_tune"):
        return nn_
    cands = {"mfma": nn_, "mfma_t": nt_, "mfma_ct": ct, "blas": blas}
    if dy2.shape[1] >= 4096 and dy2.shape[1] % 64 == 0:
        cands["mfma_sk"] = sk
    return cands[_at.choose(("linear",) + key, cands, "mfma", lambda: dx)]


def _gelu_dgrad(ctx, dy2, w, pre, M: int, K: int, N: int) -> bool:
    """Bwd-data GEMM with the producing GELU Linear's backward in its epilogue: g = dY W * gelu'(pre)
    and that Linear's bias gradient (into its grad sink when the data plane installed one), handed
    over with the producer's forward token; False when the kernel declines the shape (nothing ran)."""
    C = native()
    src = ctx.gelu_src
    g = torch.empty(M, K, dtype=dy2.dtype, device=dy2.device)
    sink = getattr(src, "_psd_grad_sink", None)
    db = sink(src.bias) if (sink is not None and src.bias is not None) else None
    if db is None:
        db = torch.empty(K, dtype=w.dtype, device=w.device)

    def nn_():
        if not C.gemm_gelu_bwd_(dy2, w, True, False, pre, g, db):
            raise _at.Declined("gelu-bwd GEMM (NN)")

    def nt_():
        if not C.gemm_gelu_bwd_(dy2, w.t().contiguous(), True, True, pre, g, db):
            raise _at.Declined("gelu-bwd GEMM (NT)")

    try:
        fn = {"nn": nn_, "nt": nt_}[_at.choose(("linear", "dgrad_gelu", M, K, N), {"nn": nn_, "nt": nt_}, "nn",
                                              lambda: g)]
        fn()
    except _at.Declined:
        return False
    # keyed by the producer's forward token: its backward must find exactly this hand-over (a
    # fused gradient consumed as an ordinary one would apply GELU' twice)
    src._psd_gelu_hands[ctx.gelu_tok] = (g, db if src.bias is not None else None)
    return True


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, mod):
        C = native()
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).contiguous()
        M, N = x2.shape[0], weight.shape[0]
        y = torch.empty(M, N, dtype=x.dtype, device=x.device)
        act = ACTS[mod.act]
        aux = torch.empty_like(y) if act == 2 else None
        if mod.fp8 and x2.shape[1] % 128 == 0:
            from . import quantize_fp8

            xq, sx = quantize_fp8(x2)
            wq, sw = quantize_fp8(weight)
            C.gemm_fp8_(xq, wq, sx, sw, y, bias, act, aux)
        else:
            def mfma():
                C.gemm_(x2, weight, True, True, y, bias, act, aux)

            def blas():
                pre = aux if act == 2 else y
                if bias is not None:
                    torch.addmm(bias, x2, weight.t(), out=pre)
                else:
                    torch.mm(x2, weight.t(), out=pre)
                if act == 1:
                    torch.relu_(y)
                elif act == 2:
                    torch.ops.aten.gelu.out(aux, approximate="tanh", out=y)

            _route(("fwd", M, x2.shape[1], N, act, bias is not None), mfma, blas, y,
                   {"mfma_ct": lambda: _ct(weight, x2, y, bias, act, aux)})()
        ctx.act = act
        ctx.mod = mod
        # per-forward token: a residual LayerNorm that hands this forward's input gradient over
        # records it, and backward only takes a hand-over carrying its own token (a backward that
        # stopped between the two -- an exception, autograd.grad on a partial graph -- can never
        # leave a stale gradient for the next step)
        ctx.tok = mod._psd_tok = getattr(mod, "_psd_tok", 0) + 1
        ctx.has_bias = bias is not None
        ctx.in_shape = shp
        # GELU hand-over (MfmaLinear.psd_gelu_input_from): this Linear's bwd-data GEMM applies the
        # producing GELU Linear's activation backward in its epilogue when x is that Linear's output
        # of the current forward
        src = getattr(mod, "_psd_gelu_from", None)
        fuse = (src is not None and _feat("gelu_fuse") and getattr(x, "_psd_gelu_tok", None) is not None
                and x._psd_gelu_tok == (id(src), src._psd_tok) and getattr(src, "_psd_gelu_pre", None) is not None)
        ctx.gelu_src = src if fuse else None
        ctx.gelu_tok = src._psd_tok if fuse else None
        pre_src = src._psd_gelu_pre if fuse else None
        ctx.save_for_backward(x2, weight, y if act == 1 else aux, pre_src)
        out = y.view(*shp[:-1], N)
        out._psd_src = (mod, ctx.tok)  # a consumer that can hand this Linear its bias gradient
        if act == 2:
            mod._psd_gelu_pre = aux  # what a fused consumer's backward reads (also saved in this ctx)
            out._psd_gelu_tok = (id(mod), ctx.tok)
        return out

    @staticmethod
    def backward(ctx, dy):
        C = native()
        x2, w, keep, pre_src = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0]).contiguous()
        sink = getattr(ctx.mod, "_psd_grad_sink", None)
        db = None
        hands = ctx.mod._psd_gelu_hands
        hand = hands.pop(ctx.tok, None)
        for t in [t for t in hands if t < ctx.tok]:  # left by an aborted backward
            del hands[t]
        if hand is not None:
            if ctx.act != 2 or hand[0].data_ptr() != dy2.data_ptr():
                raise RuntimeError(
                    "psd MfmaLinear: the consumer fused this GELU's backward (psd_gelu_input_from) but the "
                    "gradient reaching it is not the handed-over one -- the GELU output has another consumer")
            # the consumer's bwd-data GEMM already applied this GELU's backward and summed the bias
            # gradient (gemm_gelu_bwd_): dy IS the pre-activation gradient
            db = hand[1]
        elif ctx.act == 1:
            dy2 = dy2 * (keep > 0)
        elif ctx.act == 2 and ctx.has_bias and ctx.needs_input_grad[2] and dy2.shape[1] % 8 == 0:
            # GELU backward and the bias gradient in one pass over dy / pre (kernels/gemm.hip)
            db = sink(ctx.mod.bias) if sink is not None else None
            if db is None:
                db = torch.empty(w.shape[0], dtype=w.dtype, device=w.device)
            g = torch.empty_like(dy2)
            C.gelu_bwd_colsum_(dy2, keep, g, db, False)
            dy2 = g
        elif ctx.act == 2:
            dy2 = torch.ops.aten.gelu_backward(dy2, keep, approximate="tanh")
        M, K, N = x2.shape[0], x2.shape[1], w.shape[0]
        dx = None
        pend = ctx.mod._psd_pending_dx
        got = None
        while pend:  # older hand-overs (of an aborted backward) are dropped
            tok, g = pend.pop()
            if tok == ctx.tok:
                got = g
                break
        pend.clear()
        if ctx.needs_input_grad[0] and got is not None:
            # x's other gradient (a residual LayerNorm's, ops/layernorm.py): accumulated by the GEMM
            dx = got.view(M, K)
            dx.addmm_(dy2, w)
            dx = dx.view(ctx.in_shape)
        elif ctx.needs_input_grad[0] and ctx.gelu_src is not None and _gelu_dgrad(ctx, dy2, w, pre_src, M, K, N):
            dx = ctx.gelu_src._psd_gelu_hands[ctx.gelu_tok][0].view(ctx.in_shape)
        elif ctx.needs_input_grad[0]:
            dx = torch.empty(x2.shape, dtype=dy2.dtype, device=dy2.device)
            _dgrad_route(("dgrad", M, K, N), dy2, w, dx)()
            dx = dx.view(ctx.in_shape)
        if ctx.gelu_src is not None and ctx.gelu_src._psd_gelu_pre is pre_src:
            ctx.gelu_src._psd_gelu_pre = None  # not kept alive between steps
        dw = None
        if ctx.needs_input_grad[1]:
            dw = sink(ctx.mod.weight) if sink is not None else None
            if dw is None:
                dw = torch.empty(w.shape, dtype=w.dtype, device=w.device)
            _route(("wgrad", M, K, N), lambda: C.gemm_splitk_(dy2, x2, False, False, dw, False, 1.0, 0),
                   lambda: torch.mm(dy2.t(), x2, out=dw), dw)()
        bh = getattr(ctx.mod, "_psd_bias_hand", None)
        ctx.mod._psd_bias_hand = None
        if db is None and bh is not None and bh[0] == ctx.tok and bh[1] == dy2.data_ptr():
            db = bh[2]  # summed by the consumer LayerNorm's backward (ops/layernorm.py)
        if ctx.has_bias and ctx.needs_input_grad[2] and db is None:
            db = sink(ctx.mod.bias) if sink is not None else None
            if db is None:
                db = torch.empty(w.shape[0], dtype=w.dtype, device=w.device)
            C.colsum_(dy2, db, False)
        return dx, dw, db, None


class MfmaLinear(nn.Linear):
    """``nn.Linear`` (+ fused activation) running on the gfx950 MFMA GEMM for bf16 device tensors."""

    def __init__(self, in_features, out_features, bias=True, act=None, device=None, dtype=None, fp8=False):
        super().__init__(in_features, out_features, bias=bias, device=device, dtype=dtype)
        self.act = act
        self.fp8 = fp8
        self._psd_pending_dx: list = []  # gradients of the input handed over by a residual LayerNorm
        self._psd_gelu_from = None  # psd_gelu_input_from: the GELU Linear whose output is this one's input
        self._psd_gelu_hands: dict = {}  # forward token -> (pre-activation gradient, bias gradient) from the consumer
        self._psd_gelu_pre = None
        self._psd_bias_hand = None  # (forward token, dy data pointer, bias gradient) from a consumer LayerNorm

    def psd_gelu_input_from(self, src: "MfmaLinear") -> None:
        """Declare that this Linear's input is ``src``'s GELU output and nothing else reads it: the
        bwd-data GEMM here then returns d(pre-activation) with the GELU backward and src's bias
        gradient fused in its epilogue (src's backward skips both). Only valid when src's output
        has no other consumer (e.g. BERT's FFN: ffn2(ffn1(x)))."""
        assert src.act == "gelu"
        self._psd_gelu_from = src

    def psd_takes_pending_dx(self, x) -> bool:
        """True when this module's forward on ``x`` ran the autograd Function whose backward folds a
        handed-over input gradient into its bwd-data GEMM."""
        return _ok(x, self.weight) and x.shape[-1] == self.in_features

    def psd_direct_grad_params(self):
        return [p for p in (self.weight, self.bias) if p is not None]

    def forward(self, x):
        if _ok(x, self.weight):
            return _LinearFn.apply(x, self.weight, self.bias, self)
        y = F.linear(x, self.weight.to(x.dtype), None if self.bias is None else self.bias.to(x.dtype))
        if self.act == "relu":
            y = F.relu(y)
        elif self.act == "gelu":
            y = F.gelu(y, approximate="tanh")
        return y
