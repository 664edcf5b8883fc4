"""Convolution routing for the NHWC ResNets: 1x1 / stride-1 convolutions as GEMMs where that is
faster than MIOpen, and the stem convolution on its own gfx950 kernel (bottom of this file).

On NHWC bf16 a 1x1 stride-1 convolution *is* a GEMM over the [N*H*W, C] view of the activation:

  forward  Y[M, cout] = X[M, cin] . W[cout, cin]^T
  dgrad    dX[M, cin] = dY[M, cout] . W[cout, cin]
  wgrad    dW[cout, cin] = dY^T . X            (a K = N*H*W reduction)

rocprofv3 of the b1024 ResNet-50 step (profiles/resnet50_b1024_r1_kernels.md) showed MIOpen
running every 1x1 bwd-data as a CK kernel that needs its output zero-filled first (a 50-240 us
``fillBufferAligned`` per layer) and, including that fill, 1.2-1.9x slower than hipBLASLt on the
same GEMM (tools/gemm_bench.py, profiles/gemm_vs_hipblaslt_miopen_r1.md). Forward is a toss-up per
shape, wgrad is MIOpen's (hipBLASLt is 4-9x slower on the K = N*H*W reduction).

So each shape is autotuned once, in the first eager step (the same role as MIOpen's own Find):
forward and bwd-data pick MIOpen, hipBLASLt or our MFMA GEMM (kernels/gemm.hip), bwd-weight MIOpen
or our split-K MFMA GEMM, by timing the candidates with HIP events (and validating their outputs). Decisions are cached per (M, cin, cout); inside a
hipGraph capture no timing happens (an undecided shape takes MIOpen). feature ``conv1x1`` off (utils/config.py FEATURES) turns the
GEMM routes off (A/B switch).

Every other convolution (3x3 at any stride, strided 1x1 downsample) is a ``ConvNHWC``: forward
picks MIOpen or the implicit-GEMM kernel (the persistent 8-phase MFMA GEMM of kernels/gemm.hip
with its A operand gathered from the NHWC input, ``conv_fwd_``; 1.2-1.6x MIOpen on the ResNet-50 /
WRN-101-2 b1024 shapes, profiles/conv_igemm_vs_miopen_r2.md), and a stride-1 bwd-data is the same
kernel run on dY with the flipped, transposed weights. The weight gradient picks MIOpen or the
implicit-GEMM weight-gradient mode of the same kernel (dY^T . im2col(x), the im2col image gathered
per K-tile; split-K over the output pixels).

Reference parity: none -- the reference has no model (its gradient is the constant 0.01,
src/worker.cpp:316-329). This is worker-side compute for the BASELINE.json ResNet configs.
"""
from __future__ import annotations


import torch
import torch.nn as nn
import torch.nn.functional as F

from ..utils.config import feature as _feat
from . import wprep as _wprep
from . import autotune as _at
from .bn import StridedDr, take_dr


def _enabled() -> bool:
    return _feat("conv1x1")


def _choose(key: tuple, candidates: dict) -> str:
    """Fastest candidate for ``key`` (ops/autotune.py); MIOpen while a graph is being captured."""
    return _at.choose(("conv1x1",) + key, candidates, "miopen")


def decisions() -> dict:
    """The cached per-shape 1x1-conv choices, keyed (kind, M, cin, cout) (for logs / tests)."""
    return {k[1:]: v for k, v in _at.decisions().items() if k[0] == "conv1x1"}


def set_decision(key: tuple, name: str | None) -> None:
    _at.set_decision(("conv1x1",) + key, name)


def _native():
    from .. import native

    return native()


def _psd_ok(k: int, n: int) -> bool:
    """Shapes the MFMA GEMM takes as a 1x1 convolution (bf16 rows of 16-B multiples)."""
    return k % 8 == 0 and n % 8 == 0 and _feat("conv1x1_mfma")


def _as_2d(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels_last -> the [N*H*W, C] row-major view."""
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _from_2d(t2: torch.Tensor, n: int, h: int, w: int) -> torch.Tensor:
    return t2.view(n, h, w, t2.shape[1]).permute(0, 3, 1, 2)


def _fp8_ok(k: int, n: int) -> bool:
    """Shapes the fp8 MFMA GEMM / implicit-GEMM kernel takes (K a multiple of 128, >= 256 columns)."""
    return k % 128 == 0 and k >= 256 and n >= 256 and n % 8 == 0 and _feat("fp8_compute")


def _q8(t2: torch.Tensor, e5m2: bool = False, scaler: "DelayedScale | None" = None):
    """Per-tensor OCP fp8 quantisation of a contiguous tensor: (q, scale_inv). e4m3 for activations
    and weights, e5m2 (wider range) for output gradients. Weights: just-in-time amax (two launches);
    activations / gradients with a ``scaler``: delayed scaling (one pass, see DelayedScale)."""
    from . import quantize_fp8

    if scaler is not None:
        return scaler.quantize(t2, e5m2)
    return quantize_fp8(t2, e5m2=e5m2)


FP8_CALLS = {"fwd": 0, "dgrad": 0, "ps_weights": 0}  # fp8 kernel launches by role (tests / logs)


def _mx_on() -> bool:
    """MX block scaling for every fp8 operand (feature ``fp8_mx``, default on): one E8M0 scale per 32
    contiguous K-elements (kernels/fp8.hip quant_mx_kernel; the block-scaled MFMA consumes the
    scales), no amax pass and no scale history; 0: per-tensor scales (delayed for activations and
    gradients, just-in-time for weights)."""
    return _feat("fp8_mx")


def _q_act(t: torch.Tensor, e5m2: bool = False, scaler: "DelayedScale | None" = None):
    """fp8 activation / output-gradient operand: MX (q, uint8 scales) or per-tensor (q, fp32 scale)."""
    if _mx_on():
        from . import quantize_mx

        return quantize_mx(t, e5m2=e5m2)
    return _q8(t, e5m2=e5m2, scaler=scaler)


def _q_weight(mod, w2: torch.Tensor):
    """fp8 forward weight operand [Cout, K]: the MX copy the PS data plane published with the
    weights this step's forward uses (``_psd_w8``, parallel/collective_ps.py / async_ps.py: no
    per-step weight quantisation), else quantised here."""
    if _mx_on():
        pub = getattr(mod, "_psd_w8", None) if mod is not None else None
        got = pub(w2) if pub is not None else None
        if got is not None:
            FP8_CALLS["ps_weights"] += 1
            return got
        from . import quantize_mx

        return quantize_mx(w2)
    return _q8(w2)


def _take_dq8(mod, dy: torch.Tensor):
    """The MX e5m2 copy of ``dy`` the consumer BN's backward pass wrote for this module (ops/bn.py
    _dq8_args): (q [N, C, H, W] channels_last, uint8 scales), or None. Consumed once."""
    pend = getattr(mod, "_psd_dq8_pending", None) if mod is not None else None
    if pend is None:
        return None
    mod._psd_dq8_pending = None
    d, q, sc = pend
    if d.data_ptr() != dy.data_ptr() or d.shape != dy.shape or d.stride() != dy.stride():
        return None
    return q, sc


def _take_q8(mod, x: torch.Tensor):
    """The MX e4m3 copy of ``x`` that the producing BN's apply pass wrote for this module (ops/bn.py),
    as (q [N, C, H, W] channels_last, E8M0 scales uint8 [numel / 32]), or None. Consumed once."""
    pend = getattr(mod, "_psd_q8_pending", None) if mod is not None else None
    if pend is None:
        return None
    mod._psd_q8_pending = None
    y, q, sinv = pend
    if y.data_ptr() != x.data_ptr() or y.shape != x.shape or y.stride() != x.stride():
        return None
    return q, sinv


# ---------------------------------------------------------------------------------------------
# narrow-output implicit-GEMM kernel (kernels/convn.hip) + the consumer BN's statistics


def _psdn_ok(cin: int, cout: int) -> bool:
    """convn_'s contract: C a power of two >= 64, Cout 64 / 128 / a multiple of 256."""
    return cin >= 64 and (cin & (cin - 1)) == 0 and (cout in (64, 128) or cout % 256 == 0) and \
        _feat("convn")


def _bn_consumer(mod):
    """The training-mode FusedBatchNorm2d that consumes ``mod``'s output (wired by the model as
    ``_psd_bn``), whose batch statistics the convolution epilogue can reduce, or None."""
    bn = getattr(mod, "_psd_bn", None) if mod is not None else None
    # (no grad-mode test: this runs inside the autograd Function's forward, where grad mode is off;
    # the module's forward only takes the Function path with grad enabled)
    if bn is None or not bn.training or bn.running_mean is None or not _feat("convn_stats"):
        return None
    return bn


class _Lazy:
    """A weight operand made on first use (``w.t().contiguous()`` for candidates the autotuner may
    never pick: building it eagerly cost a copy launch per convolution per step). ``shape`` is known
    up front; ``()`` returns the tensor."""
    __slots__ = ("fn", "t", "shape")

    def __init__(self, fn, shape):
        self.fn, self.t, self.shape = fn, None, tuple(shape)

    def __call__(self) -> torch.Tensor:
        if self.t is None:
            self.t = self.fn()
        return self.t


def _wt(w2: torch.Tensor, mod=None, weight=None) -> _Lazy:
    """w2^T (contiguous), made on first use: the step's batched operand (ops/wprep.py) when ``mod``'s
    forward registered ``weight``, else a transpose copy."""
    def make():
        t = _wprep.get(mod, weight, "t") if weight is not None else None
        return t if t is not None else w2.t().contiguous()
    return _Lazy(make, (w2.shape[1], w2.shape[0]))


def _wflip(mod, weight: torch.Tensor) -> torch.Tensor:
    """The stride-1 bwd-data weight W'[ci][r][s][co] = W[co][ci][k-1-r][k-1-s] as [Ci, k k Co]."""
    t = _wprep.get(mod, weight, "f")
    if t is not None:
        return t
    cout, cin, k, _ = weight.shape
    return weight.flip(2, 3).permute(1, 2, 3, 0).reshape(cin, k * k * cout).contiguous()


def _get(w):
    return w() if isinstance(w, _Lazy) else w


def _convn_variants(x, w2, k: int, stride: int, pad: int, bn=None) -> dict:
    """{"psdn<v>": fn} over the kernel's tile variants; fn() -> the channels_last conv output. With a
    consumer ``bn`` every "psdn" call also reduces the BN's statistics partials in its epilogue and
    hands them to the BN (``_psd_stats_pending``: its forward then skips the statistics pass), and
    "psdu<v>" candidates run the same variants without that epilogue."""
    C = _native()
    n, _, h, w = x.shape
    cout = w2.shape[0]
    ho, wo = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
    M = n * ho * wo

    def make(v, stats):
        def fn():
            out = torch.empty(M, cout, device=x.device, dtype=x.dtype)
            part = None
            if stats:
                part = torch.empty(_part_rows(M, cout, v, ho, wo, k), 2, cout, device=x.device, dtype=torch.float32)
            rows = C.convn_(x, _get(w2), out, k, k, stride, pad, part=part,
                            shift=bn.running_mean if stats else None, variant=v)
            if rows == 0:
                raise RuntimeError("convn_ declined a shape _psdn_ok accepted")
            y = _from_2d(out, n, ho, wo)
            if stats:
                bn._psd_stats_pending = (y, part, rows)
            return y
        return fn

    ok = [v for v in range(C.convn_variants(cout)) if _variant_ok(cout, v, k, stride, pad, wo, x.shape[1], h)]
    cands = {f"psdn{v}": make(v, bn is not None) for v in ok}
    if bn is not None:
        # the same kernels without the statistics epilogue ("psdu": the BN then runs its own reduce
        # pass, and _route times them with it)
        cands.update({f"psdu{v}": make(v, False) for v in ok})
    return cands


def _variant_ok(cout: int, v: int, k: int, stride: int, pad: int, wo: int, cin: int | None = None,
                h: int | None = None) -> bool:
    """Variant v of the narrow kernel takes this shape: the gathered variants (kind 0), the
    persistent HALO variant (kind 2, C = N = 64 3x3 stride 1, H = Ho) and the persistent 1x1 variant
    (kind 3; kind 4 at two workgroups per CU) whenever their contract holds (features convn_persist /
    convn_p1 / convn_p2)."""
    C = _native()
    if not C.convn_variant_ok(cout, v, k, k, stride, pad, wo):
        return False
    kind = C.convn_variant_kind(cout, v)
    if kind == 2:
        return _feat("convn_persist") and cin == 64 and (h is None or h == wo)
    if kind == 3:  # persistent 1x1 (convp_kernel)
        return _feat("convn_p1")
    if kind == 4:  # the same at two workgroups per CU
        return _feat("convn_p1") and _feat("convn_p2")
    return kind == 0


def _part_rows(M: int, N: int, v: int, ho: int, wo: int, k: int) -> int:
    """Statistics partial rows to allocate for a convn launch of variant v (HALO variants tile by
    output rows, kernels/convn.hip)."""
    C = _native()
    return max(C.convn_stats_rows(M), C.convn_part_rows(M, N, v, ho, wo, k))


def _fwd_records(ctx, mod) -> None:
    """Capture at forward the model wiring the backward consults (``_psd_bn_in``: the BN whose
    output this convolution consumes; ``_psd_strided_to``: where a downsample convolution hands its
    quarter-grid input gradient). The model rewrites these attributes on every forward, so reading
    them from the module at backward time could pick up a later forward's wiring."""
    ctx.bn_in = getattr(mod, "_psd_bn_in", None) if mod is not None else None
    ctx.strided_to = getattr(mod, "_psd_strided_to", None) if mod is not None else None


def _bn_bwd_fusion(bn, x: torch.Tensor):
    """When the convolution's input ``x`` is exactly the output of a FusedBatchNorm2d + ReLU ``bn``
    (wired by the model as ``_psd_bn_in``, recorded at forward) whose only autograd consumer is the
    convolution, the bwd-data epilogue can run
    that BN's backward reduction (kernels/convn.hip bwd modes): mode 1 (no residual: ReLU mask from
    its x and scale/shift) or mode 2 (a residual BN: bit-mask, plus the residual-branch gradient
    handed over by the next block). Returns the arguments, or None."""
    st = getattr(bn, "_psd_fwd", None) if bn is not None else None
    if st is None or not _feat("convn_bwd"):
        return None
    y, bx, mean, ss, mbits, xd, mean_d = st
    if y.data_ptr() != x.data_ptr() or y.shape != x.shape or y.stride() != x.stride():
        return None
    if mbits is not None:
        if not bn._psd_pending_dr:
            return None
        if isinstance(bn._psd_pending_dr[-1], StridedDr):  # a downsample conv's quarter-grid gradient
            if xd is not None or x.shape[2] % 2 or x.shape[3] % 2 or not _feat("convn_bwd5"):
                return None
            return dict(mode=5, bn=bn, bx=bx, mean=mean, mbits=mbits)
        if xd is not None:  # a downsample block's dual tail: both BNs' reductions (mode 3)
            if not _feat("convn_bwd3"):
                return None
            return dict(mode=3, bn=bn, bx=bx, mean=mean, mbits=mbits, bxd=xd, mean_d=mean_d)
        return dict(mode=2, bn=bn, bx=bx, mean=mean, mbits=mbits)
    return dict(mode=1, bn=bn, bx=bx, mean=mean, ss=ss)


def _convn_bwd_variants(dy, w2, k: int, pad: int, fu: dict, dr) -> dict:
    """{"psdnb<v>": fn}: stride-1 bwd-data on the narrow kernel whose epilogue runs the producing
    BN's backward reduction; fn() -> g (the masked gradient the BN's elementwise pass takes), with
    the partials handed to the BN (``_psd_bwd_pre``)."""
    C = _native()
    n, _, h, w = dy.shape
    cout = w2.shape[0]
    M = n * h * w

    def make(v):
        def fn():
            out = torch.empty(M, cout, device=dy.device, dtype=dy.dtype)
            # (+ 1 row: a BN whose input was never stored completes its partials there, ops/tail.py)
            part = torch.empty(_part_rows(M, cout, v, h, w, k) + 1, 2, cout, device=dy.device, dtype=torch.float32)
            part_d = torch.empty_like(part) if fu["mode"] == 3 else None
            rows = C.convn_bwd_(dy, _get(w2), out, k, k, 1, pad, part, v, fu["mode"], fu["bx"], fu["mean"],
                                bss=fu.get("ss"), bdr=_dr_arg(dr), bmbits=fu.get("mbits"), bxd=fu.get("bxd"),
                                bmean_d=fu.get("mean_d"), part_d=part_d)
            if rows == 0:
                raise RuntimeError("convn_bwd_ declined a shape _psdn_ok accepted")
            g = _from_2d(out, n, h, w)
            fu["bn"]._psd_bwd_pre = (g, part, rows) if part_d is None else (g, part, rows, part_d)
            return g
        return fn

    return {f"psdnb{v}": make(v) for v in range(C.convn_variants(cout))
            if _variant_ok(cout, v, k, 1, pad, w, dy.shape[1], h)}


def _s2_phase_weights(weight: torch.Tensor) -> list:
    """The four output-parity phase weights of a stride-2 / pad-1 3x3 bwd-data (kernels/convn.hip
    ophase): dX[2i + ph][2j + pw] = sum over dY rows i (+ i + 1 when ph = 1) and columns likewise, so
    phase k = ph << 1 | pw takes taps r in (1,) / (2, 0) and s alike -- bf16 [Ci, R' S' Co] in
    (dr, ds, co) order: W'[ci][dr][ds][co] = W[co][ci][r(dr)][s(ds)]."""
    cin = weight.shape[1]
    # tap subsets by slicing only: r in (1,) = [1:2], r in (2, 0) = [0::2] reversed. (Indexing with a
    # Python list uploads the index tensor host -> device on every call: 24 blocking copies per
    # ResNet-50 step, each leaving the GPU idle ~25 us, profiles/r5/resnet50_b1024_r5g_kernels.md.)
    sel = (lambda t, d: t.narrow(d, 1, 1), lambda t, d: t[(slice(None),) * d + (slice(None, None, 2),)].flip(d))
    out = []
    for ph in (0, 1):
        for pw in (0, 1):
            wsel = sel[pw](sel[ph](weight, 2), 3)
            out.append(wsel.permute(1, 2, 3, 0).reshape(cin, -1).contiguous())
    return out


def _dgrad_s2_phases(dy, weight, x, fu, mod=None) -> dict:
    """{"psdns<v>" / "psdnbs<v>": fn}: a stride-2 3x3 bwd-data on the narrow kernel as four phase
    launches (no zero-insertion, no zero-filled dX; MIOpen's kernel runs a fill pass over dX first)
    -- with ``fu`` (mode 1: the producing BN + ReLU) the fused candidates also reduce that BN's
    backward in their epilogues and hand the partials over, as _convn_bwd_variants does."""
    C = _native()
    n, cin, h, w = x.shape
    ho, wo = dy.shape[2], dy.shape[3]
    def phases():
        got = _wprep.get(mod, weight, "p")
        return got if got is not None else _s2_phase_weights(weight)

    wph = _Lazy(phases, (4,))

    def make(v, fused):
        def fn():
            out = torch.empty(n * h * w, cin, device=dy.device, dtype=dy.dtype)
            if fused:
                part = torch.empty(C.convn_dgrad_s2_rows(n, ho, wo, cin, v) + 1, 2, cin, device=dy.device,
                                   dtype=torch.float32)
                rows = C.convn_dgrad_s2_(dy, wph(), out, v, part=part, bx=fu["bx"], bmean=fu["mean"], bss=fu["ss"])
            else:
                rows = C.convn_dgrad_s2_(dy, wph(), out, v)
            if rows == 0:
                raise RuntimeError("convn_dgrad_s2_ declined a shape it was offered for")
            g = _from_2d(out, n, h, w)
            if fused:
                fu["bn"]._psd_bwd_pre = (g, part, rows)
            return g
        return fn

    cands = {}
    for v in range(C.convn_variants(cin)):
        if C.convn_variant_kind(cin, v) != 0 or not C.convn_variant_ok(cin, v, 2, 2, 1, 0, wo, False):
            continue
        cands[f"psdns{v}"] = make(v, False)
        if fu is not None:
            cands[f"psdnbs{v}"] = make(v, True)
    return cands


def _dgrad_route(key: tuple, cands: dict, default: str, fu, dy_like) -> torch.Tensor:
    """bwd-data: the fastest candidate; with a BN backward fusion available the library and
    unfused candidates are timed with the reduction pass they leave to the BN. A non-fused choice
    returns the handed-over residual gradient to the BN's queue."""
    if fu is None:
        return cands[_at.choose(key, cands, default)]()
    if fu.get("bx") is None:
        # the BN's input was never stored (ops/tail.py): only the fused epilogue can reduce its backward
        cands = {name: fn for name, fn in cands.items() if name.startswith("psdnb")}
        if not cands:
            raise RuntimeError("psd: a BN without its stored input needs the fused bwd-data epilogue")
        key, default = key + ("nobx",), next(iter(cands))
    timed = {name: (fn if name.startswith("psdnb") else _with_bn_bwd_reduce(fn, fu)) for name, fn in cands.items()}
    # (the fused candidates return the BN-masked gradient g, the others dX: validated per family)
    how = _at.choose(key + ("bnbwd",), timed, default, group=lambda n: n.startswith("psdnb"))
    out = cands[how]()
    if not how.startswith("psdnb"):
        fu["bn"]._psd_bwd_pre = None
        if fu.get("dr") is not None:
            fu["bn"]._psd_pending_dr.append(fu["dr"])
    return out


def _with_bn_reduce(fn, bn):
    """Timing twin of a library candidate: its output plus the BN statistics pass it leaves to the
    BN (so the autotuner compares the fused kernel against library conv + reduce)."""
    def g():
        y = fn()
        _native().bn_reduce_(y, bn.running_mean)
        return y
    return g


def _with_bn_bwd_reduce(fn, fu):
    """Timing twin of an unfused bwd-data candidate: its output plus the BN backward reduction it
    leaves to the BN -- the same pass the BN then runs (mask from x and scale/shift, or the residual
    BN's bit-mask with the handed-over residual gradient folded in and dr written; a quarter-grid
    downsample gradient is materialised first, as the BN then does)."""
    def g():
        dx = fn()
        _native().bn_bwd_reduce_(dx, fu["bx"], fu["mean"], ss=fu.get("ss"), dy2=take_dr(fu.get("dr")),
                                 mbits=fu.get("mbits"))
        return dx
    return g


def _stats_part(bn, M: int, cout: int, device):
    """Statistics-partials buffer for an 8-phase GEMM / implicit-GEMM launch whose epilogue reduces
    the consumer BN's batch statistics (kernels/gemm.hip ST), or None without a consumer BN."""
    if bn is None or not _feat("gemm_stats"):
        return None
    return torch.empty(_native().gemm_stats_rows(M), 2, cout, device=device, dtype=torch.float32)


def _hand_stats(bn, y, part, rows: int):
    """Queue the partials a GEMM epilogue reduced for ``y`` on its consumer BN (skips its reduce)."""
    if part is not None and rows > 0:
        bn._psd_stats_pending = (y, part, rows)


def _dr_arg(dr):
    """The convn_bwd_ dr operand: a quarter-grid StridedDr's tensor (mode 5) or the full gradient."""
    return dr.t4 if isinstance(dr, StridedDr) else dr


def _route(key: tuple, cands: dict, default: str, bn=None) -> str:
    """Autotuned choice among ``cands``; with a consumer BN the library candidates are timed with
    the statistics pass they leave behind (the psdn ones reduce it in their epilogue)."""
    if bn is None:
        return _at.choose(key, cands, default)
    timed = {name: (fn if name.startswith(("psdn", "psds")) else _with_bn_reduce(fn, bn))
             for name, fn in cands.items()}
    how = _at.choose(key + ("bnstats",), timed, default)
    bn._psd_stats_pending = None  # (a timed candidate's hand-over; the chosen one, run next, sets its own)
    return how


def _convw_cands(dy, x, k: int, stride: int, pad: int) -> dict:
    """{"psdw<v>": fn(into=None)} over the narrow weight-gradient kernel's tile variants
    (kernels/convw.hip); fn writes dW in OHWI order into ``into`` (a contiguous [Cout, k*k*Cin] view,
    e.g. the PS gradient sink) or a fresh tensor and returns the [Cout, Cin, k, k] channels_last view;
    raises autotune.Declined when the kernel does not take the shape."""
    if not _feat("convw"):
        return {}
    C = _native()
    cout, cin = dy.shape[1], x.shape[1]
    kk = k * k * cin
    if cin < 64 or (cin & (cin - 1)) or not (cout in (64, 128) or cout % 256 == 0):
        return {}

    def make(v):
        def fn(into=None):
            o = into if into is not None else torch.empty(cout, kk, device=dy.device, dtype=dy.dtype)
            if not C.convw_(dy, x, o, k, k, stride, pad, variant=v):
                raise _at.Declined(f"convw_ variant {v}")
            return o.view(cout, k, k, cin).permute(0, 3, 1, 2)
        return fn

    nv = C.convw_variants(cout, kk)
    persist = 1 if (cout == 64 and kk == 576) else 0  # the persistent HALO wgrad: the last variant
    shapes = (nv - persist) // 2  # tile shapes, then their two-stage-ring twins (kernels/convw.hip)
    vs = [v for v in range(nv) if (v < shapes or _feat("convw_twostage")) and (v < 2 * shapes or _feat("convw_persist"))]
    return {f"psdw{v}": make(v) for v in vs}


class DelayedScale:
    """Delayed fp8 scaling for one tensor role of one layer (its input activations, or its output
    gradient): each call quantises with the amax the previous call recorded (times ``margin``) and
    records its own in the same pass (kernels/fp8.hip quant_delayed_kernel), so the tensor is read
    once instead of twice (amax pass + quantise pass). The first call scales just-in-time and seeds
    the history. Values above the previous step's amax saturate at the fp8 maximum. The history is a
    device tensor, so a captured hipGraph keeps updating it. feature ``fp8_delayed`` off: always
    just-in-time."""

    def __init__(self, margin: float = 1.0):
        self.margin = float(margin)
        self.hist = None

    def quantize(self, x: torch.Tensor, e5m2: bool):
        from . import FP8_E4M3_MAX, FP8_E5M2_MAX, quantize_fp8

        x = x.contiguous()
        if self.hist is None or self.hist.device != x.device or not _feat("fp8_delayed"):
            q, sinv = quantize_fp8(x, e5m2=e5m2)
            if _feat("fp8_delayed"):
                self.hist = torch.zeros(2, dtype=torch.float32, device=x.device)
                self.hist[:1].copy_(sinv * (FP8_E5M2_MAX if e5m2 else FP8_E4M3_MAX) / self.margin)
            return q, sinv
        q = torch.empty(x.shape, dtype=torch.float8_e5m2 if e5m2 else torch.float8_e4m3fn, device=x.device)
        sinv = torch.empty(1, dtype=torch.float32, device=x.device)
        _native().quant_fp8_delayed_(x, q, sinv, self.hist, self.margin)
        return q, sinv


def _sink_view(mod, weight):
    """The PS data plane's gradient view for ``weight`` (written instead of returning a fresh dW that
    autograd would then add into the flat gradient buffer), or None."""
    sink = getattr(mod, "_psd_grad_sink", None) if mod is not None else None
    return sink(weight) if sink is not None else None


def _fold_v() -> int:
    """convw variant of the fold / Gram launches: 1 = the two-stage ring at two workgroups per CU."""
    return 1 if _feat("convw_fold2") else 0


def fold_ok(cin: int, cout: int) -> bool:
    """The BN-backward fold of a 1x1 convolution (cin -> cout) runs on our kernels for this shape:
    the K-concatenated dgrad on the narrow kernel and the fold wgrad (kernels/convw.hip)."""
    C = _native()
    return (_psdn_ok(cout, cin) and cin >= 64 and (cin & (cin - 1)) == 0 and cout % 64 == 0
            and C.convw_fold_rows(cout, cin) > 0)


def _fold_backward(ctx, fold, x, weight, need_x: bool, need_w: bool, P=None):
    """conv3's backward with its consumer BN's input gradient folded in (kernels/bnfold.hip): the BN
    handed over g (the masked upstream gradient) and the coefficients of dy = A g + B y + C, where
    y = conv(x) is the BN input. dgrad runs on the narrow kernel with the K-concatenated operand
    [g | x] (and the producing BN's backward reduction in its epilogue where that wins); wgrad on
    the narrow wgrad kernel's fold mode (g^T x, x^T x, 1^T x in one pass) + the combination. The
    unfolded path -- the BN elementwise pass, then the ordinary dgrad -- is one of the timed
    candidates (and the correctness reference); when it wins, (None, None, dy) is returned and the
    caller runs the ordinary backward on dy. Returns (dx, dw, None) when folded.

    y None (ops/tail.py: the BN input was never stored): only the folded candidates; ``P`` the fold
    wgrad products the caller already ran (its BN statistics needed g^T x), combined here."""
    g, coef, y = fold
    C = _native()
    n, cin, h, w = x.shape
    cout = weight.shape[0]
    M = n * h * w
    keep = {}

    def unfolded_dy():
        if "dy" not in keep:
            keep["dy"] = C.bn_elemt_coef(g, y, coef)
        return keep["dy"]

    dx = dw = None
    how = "unfold"
    frows = C.convw_fold_rows(cout, cin)
    foldable = fold_ok(cin, cout) and x.is_contiguous(memory_format=torch.channels_last)
    if y is None and not foldable:
        raise RuntimeError("psd BN-backward fold without the BN input needs a foldable shape")
    conv_bwd = torch.ops.aten.convolution_backward
    wargs = (None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1)

    def fold_wgrad(into):
        Pw = P
        if Pw is None:
            Pw = torch.empty(frows, cin, device=g.device, dtype=torch.float32)
            if not C.convw_(g, x, Pw, 1, 1, 1, 0, variant=_fold_v(), fold=True):
                raise RuntimeError("convw_ declined a fold shape convw_fold_rows accepted")
        C.bnfold_combine(Pw, weight, coef, into)

    if need_x and foldable:
        w2, bvec = C.bnfold_dgrad_weights(weight, coef)
        wt = _wt(weight.reshape(cout, cin), ctx.mod, weight)
        fu = _bn_bwd_fusion(ctx.bn_in, x)
        if fu is not None:
            fu["dr"] = fu["bn"]._psd_pending_dr.pop() if fu["mode"] >= 2 else None

        # timed as dgrad + wgrad pairs: the unfolded path pays the BN elementwise pass and the plain
        # wgrad on it, the folded one the K-concatenated dgrad and the fold wgrad + combination
        timing = {"on": True}

        def unfold():
            out = torch.empty(M, cin, device=g.device, dtype=g.dtype)
            keep.pop("dy", None)
            if not C.convn_(unfolded_dy(), wt(), out, 1, 1, 1, 0, variant=0):
                raise RuntimeError("convn_ declined the unfolded dgrad")
            if timing["on"] and need_w:
                conv_bwd(keep["dy"], x, weight, *wargs, [False, True, False])
            return _from_2d(out, n, h, w)

        def make(v, fused):
            def fn():
                o = dgrad(v, fused)
                if timing["on"] and need_w:
                    fold_wgrad(torch.empty(cout, cin, device=g.device, dtype=g.dtype))
                return o
            return fn

        def dgrad(v, fused):
            out = torch.empty(M, cin, device=g.device, dtype=g.dtype)
            part_d = None
            if fused:
                part = torch.empty(C.convn_stats_rows(M), 2, cin, device=g.device, dtype=torch.float32)
                part_d = torch.empty_like(part) if fu["mode"] == 3 else None
                rows = C.convn_bwd_(g, w2, out, 1, 1, 1, 0, part, v, fu["mode"], fu["bx"], fu["mean"],
                                    bss=fu.get("ss"), bdr=_dr_arg(fu.get("dr")), bmbits=fu.get("mbits"), x2=x, bias=bvec,
                                    bxd=fu.get("bxd"), bmean_d=fu.get("mean_d"), part_d=part_d)
            else:
                rows = C.convn_(g, w2, out, 1, 1, 1, 0, variant=v, x2=x, bias=bvec)
            if rows == 0:
                raise RuntimeError("convn_ declined the folded dgrad")
            o = _from_2d(out, n, h, w)
            if fused:
                fu["bn"]._psd_bwd_pre = (o, part, rows) if part_d is None else (o, part, rows, part_d)
            return o

        cands = {"unfold": unfold} if y is not None else {}
        for v in range(C.convn_variants(cin)):
            if not C.convn_variant_ok(cin, v, 1, 1, 1, 0, w, True):
                continue
            cands[f"psdnf{v}"] = make(v, False)
            if fu is not None:
                cands[f"psdnb{v}"] = make(v, True)
        key = ("conv1x1", "dgrad_fold", M, cin, cout) + (() if y is not None else ("noy",))
        if fu is not None and fu.get("bx") is None:
            # the producing BN's input was never stored (a recomputing tail, ops/tail.py): only the
            # fused epilogue can reduce its backward (as in _dgrad_route)
            cands = {nm: fn for nm, fn in cands.items() if nm.startswith("psdnb")}
            if not cands:
                raise RuntimeError("psd: a BN without its stored input needs the fused folded bwd-data epilogue")
            key = key + ("nobx",)
        default = "unfold" if "unfold" in cands else next(iter(cands))
        if fu is None:
            how = _at.choose(key, cands, default)
        else:
            timed = {nm: (fn if nm.startswith("psdnb") else _with_bn_bwd_reduce(fn, fu)) for nm, fn in cands.items()}
            # (fused epilogues return the BN-masked gradient, the others dX: validated per family)
            how = _at.choose(key + ("bnbwd",), timed, default, group=lambda nm: nm.startswith("psdnb"))
        timing["on"] = False
        if how != "unfold":
            dx = cands[how]()
            if not how.startswith("psdnb") and fu is not None:
                fu["bn"]._psd_bwd_pre = None
                if fu.get("dr") is not None:
                    fu["bn"]._psd_pending_dr.append(fu["dr"])
        elif fu is not None:
            fu["bn"]._psd_bwd_pre = None  # (a timed fused candidate's hand-over)
            if fu.get("dr") is not None:
                fu["bn"]._psd_pending_dr.append(fu["dr"])  # the ordinary path pops it again
    elif not need_x:
        how = "fold" if foldable else "unfold"
    if how == "unfold":
        return None, None, unfolded_dy()
    if need_w:
        sv = _sink_view(ctx.mod, weight)
        if sv is not None and sv.is_contiguous():
            fold_wgrad(sv.view(cout, cin))
            dw = sv
        else:
            o = torch.empty(cout, cin, device=g.device, dtype=g.dtype)
            fold_wgrad(o)
            dw = o.view(cout, cin, 1, 1)
            if sv is not None:
                dw = sv.copy_(dw)
    return dx, dw, None


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, f8=None, mod=None):
        """``f8``: (activation scaler, gradient scaler) of an fp8 module, else None. ``mod``: the
        module, whose ``_psd_grad_sink`` (installed by the PS data plane) receives dW directly."""
        fp8 = f8 is not None
        ctx.mod = mod
        _fwd_records(ctx, mod)
        if ctx.needs_input_grad[0]:
            _wprep.note(mod, weight, "t")
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        w2 = weight.reshape(cout, cin)
        x2 = _as_2d(x)
        ctx.save_for_backward(x, weight)
        ctx.fp8, ctx.f8 = fp8, f8
        if fp8 and _fp8_ok(cin, cout):
            # fp8 forward: e4m3 operands on the MX-scaled MFMA (2x the bf16 rate), dequantised in the
            # epilogue; the weight gradient runs on the saved bf16 x and W
            got = _take_q8(mod, x)
            if got is not None:  # quantised by the producing BN's apply pass
                xq, sx = got[0].permute(0, 2, 3, 1).reshape(n * h * w, cin), got[1]
            else:
                xq, sx = _q_act(x2, scaler=f8[0])
            wq, sw = _q_weight(mod, w2)
            out = torch.empty(n * h * w, cout, device=x.device, dtype=x.dtype)
            bn = _bn_consumer(mod)
            part = _stats_part(bn, n * h * w, cout, x.device)
            rows = _native().gemm_fp8_(xq, wq, sx, sw, out, part=part,
                                       shift=bn.running_mean if part is not None else None)
            if rows == 0:  # the statistics epilogue declined the shape: plain launch, the BN reduces
                part = None
                _native().gemm_fp8_(xq, wq, sx, sw, out)
            FP8_CALLS["fwd"] += 1
            y = _from_2d(out, n, h, w)
            _hand_stats(bn, y, part, rows)
            return y
        key = ("fwd", n * h * w, cin, cout)

        def gemm():
            return _from_2d(torch.mm(x2, w2.t()), n, h, w)

        def miopen():
            return F.conv2d(x, weight)

        def psd():  # the persistent 8-phase MFMA GEMM (kernels/gemm.hip)
            out = torch.empty(n * h * w, cout, device=x.device, dtype=x.dtype)
            _native().gemm_(x2, w2, True, True, out)
            return _from_2d(out, n, h, w)

        def psds():  # the same with the consumer BN's statistics in its epilogue
            out = torch.empty(n * h * w, cout, device=x.device, dtype=x.dtype)
            part = _stats_part(bn, n * h * w, cout, x.device)
            rows = _native().gemm_(x2, w2, True, True, out, part=part, shift=bn.running_mean)
            if rows == 0:  # too few tiles for the statistics epilogue: not a candidate for this shape
                raise _at.Declined("gemm_ statistics epilogue")
            y = _from_2d(out, n, h, w)
            _hand_stats(bn, y, part, rows)
            return y

        cands = {"gemm": gemm, "miopen": miopen}
        bn = _bn_consumer(mod)
        if _psd_ok(cin, cout):
            cands["psd"] = psd
            if bn is not None and _feat("gemm_stats") and n * h * w >= 128 and cout >= 256 and cin >= 256 \
                    and cin % 64 == 0:
                cands["psds"] = psds
        if _psdn_ok(cin, cout):
            cands.update(_convn_variants(x, w2 if w2.is_contiguous() else w2.contiguous(), 1, 1, 0, bn))
        y = cands[_route(("conv1x1",) + key, cands, "miopen", bn if len(cands) > 2 else None)]()
        if mod is not None:  # this output may have its consumer BN's backward folded (_fold_backward)
            mod._psd_fold_out = (y.data_ptr(), tuple(y.shape))
            mod._psd_fold_x = x  # (a dual tail takes g^T x before the BN finalize: ops/bn.py)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dx = dw = None
        fold = getattr(ctx.mod, "_psd_fold_pending", None) if ctx.mod is not None else None
        if fold is not None:
            ctx.mod._psd_fold_pending = None
            if fold[0].data_ptr() != dy.data_ptr() or fold[0].shape != dy.shape:
                raise RuntimeError("psd BN-backward fold: the gradient reaching the convolution is not the one its BN "
                                   "handed over (its input gradient was never formed)")
            dx, dw, dy = _fold_backward(ctx, fold[:3], x, weight, need_x, need_w, P=fold[3] if len(fold) > 3 else None)
            if dy is None:
                return dx, dw, None, None
            need_x = need_x and dx is None  # unfolded: dy now holds the BN input gradient
            need_w = need_w and dw is None
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        conv_bwd = torch.ops.aten.convolution_backward
        args = (None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1)
        if need_x and ctx.fp8 and _fp8_ok(cout, cin) and _feat("fp8_dgrad"):
            # fp8 bwd-data: e5m2 dY (K-major [M, cout]) x e4m3 W^T ([cin, cout], K-major)
            got = _take_dq8(ctx.mod, dy) if _mx_on() else None
            if got is not None:  # written by the consumer BN's backward pass
                dyq, sdy = got[0].permute(0, 2, 3, 1).reshape(n * h * w, cout), got[1]
            else:
                dyq, sdy = _q_act(_as_2d(dy), e5m2=True, scaler=ctx.f8[1])
            wtq, swt = _q_act(_wt(weight.reshape(cout, cin), ctx.mod, weight)())
            out = torch.empty(n * h * w, cin, device=dy.device, dtype=dy.dtype)
            _native().gemm_fp8_(dyq, wtq, sdy, swt, out)
            FP8_CALLS["dgrad"] += 1
            dx = _from_2d(out, n, h, w)
            need_x = False
        if need_x:
            w2 = weight.reshape(cout, cin)
            dy2 = _as_2d(dy)
            key = ("dgrad", n * h * w, cin, cout)

            def gemm():
                return _from_2d(torch.mm(dy2, w2), n, h, w)

            def miopen():
                return conv_bwd(dy, x, weight, *args, [True, False, False])[0]

            def psd():
                out = torch.empty(n * h * w, cin, device=dy.device, dtype=dy.dtype)
                _native().gemm_(dy2, w2, True, False, out)
                return _from_2d(out, n, h, w)

            cands = {"gemm": gemm, "miopen": miopen}
            if _psd_ok(cout, cin):
                cands["psd"] = psd
            fu = None
            if _psdn_ok(cout, cin):  # dX = dY . W as a 1x1 convolution of dY with W^T [cin, cout]
                wt = _wt(w2, ctx.mod, weight)
                cands.update(_convn_variants(dy, wt, 1, 1, 0))
                fu = _bn_bwd_fusion(ctx.bn_in, x)
                if fu is not None:
                    fu["dr"] = fu["bn"]._psd_pending_dr.pop() if fu["mode"] >= 2 else None
                    cands.update(_convn_bwd_variants(dy, wt, 1, 0, fu, fu["dr"]))
            dx = _dgrad_route(("conv1x1",) + key, cands, "miopen", fu, x)
        if need_w:
            def miopen_w():
                return conv_bwd(dy, x, weight, *args, [False, True, False])[1]

            def psd_w():  # dW = dY^T X: split-K MFMA GEMM over the N*H*W reduction
                out = torch.empty(cout, cin, device=dy.device, dtype=dy.dtype)
                _native().gemm_splitk_(_as_2d(dy), _as_2d(x), False, False, out)
                return out.view(cout, cin, 1, 1)

            cands = {"miopen": miopen_w}
            if _psd_ok(cout, cin) and cout % 8 == 0:
                cands["psd"] = psd_w
            wcands = _convw_cands(dy, x, 1, 1, 0)
            cands.update(wcands)
            how = _choose(("wgrad", n * h * w, cin, cout), cands)
            sv = _sink_view(ctx.mod, weight)
            dw = None
            if sv is not None and how == "psd":  # split-K result reduced straight into the PS buffer
                _native().gemm_splitk_(_as_2d(dy), _as_2d(x), False, False, sv.view(cout, cin))
                dw = sv
            elif how in wcands:  # narrow wgrad kernel: its slab reduce writes the PS buffer / dW directly
                if sv is not None and sv.is_contiguous():
                    dw = wcands[how](sv.view(cout, cin))
                    if dw is not None:
                        dw = sv
                else:
                    dw = wcands[how]()
                    if dw is not None and sv is not None:
                        dw = sv.copy_(dw)
            if dw is None:
                dw = cands[how]() if how not in wcands else miopen_w()
                if sv is not None:
                    dw = sv.copy_(dw)
                elif how == "psd" and weight.is_contiguous(memory_format=torch.channels_last):
                    dw = dw.contiguous(memory_format=torch.channels_last)
        return dx, dw, None, None


class Conv1x1(nn.Conv2d):
    """``nn.Conv2d(cin, cout, 1, bias=False)`` whose NHWC bf16 training path runs the per-shape
    fastest of MIOpen / hipBLASLt for forward and bwd-data (see module docstring)."""

    def __init__(self, cin: int, cout: int, fp8: bool = False):
        super().__init__(cin, cout, 1, stride=1, padding=0, bias=False)
        self.fp8 = fp8  # fp8 forward (e4m3) and bwd-data (e5m2 dY) where the shape allows
        self._f8 = (DelayedScale(1.0), DelayedScale(2.0))  # input activations, output gradient

    def psd_direct_grad_params(self):
        return [self.weight]

    def psd_fp8_consumes(self, cin: int) -> bool:
        """True when this module's forward quantises its input (so a producer may do it instead)."""
        return self.fp8 and _fp8_ok(cin, self.out_channels) and _enabled()

    def psd_fp8_dgrad(self) -> bool:
        """True when this module's bwd-data runs in fp8 (quantising its output gradient)."""
        return (self.fp8 and _fp8_ok(self.out_channels, self.in_channels) and _enabled()
                and _feat("fp8_dgrad"))

    def forward(self, x):
        if (_enabled() and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
                and self.weight.dtype == torch.bfloat16 and torch.is_grad_enabled()
                and x.is_contiguous(memory_format=torch.channels_last)):
            return _Conv1x1Fn.apply(x, self.weight, self._f8 if self.fp8 else None, self)
        return F.conv2d(x, self.weight)


# ---------------------------------------------------------------------------------------------
# general NHWC convolution: implicit-GEMM forward / stride-1 bwd-data, MIOpen otherwise


def _pow2_ge64(c: int) -> bool:
    return c >= 64 and (c & (c - 1)) == 0


def _igemm_ok(cin: int, cout: int) -> bool:
    """conv_fwd_'s contract (kernels/gemm.hip launch_conv_fwd): C a power of two >= 64 (one (r, s)
    per 64-wide K-tile), Cout >= 256 (one 256-wide N tile) and a multiple of 8."""
    return _pow2_ge64(cin) and cout >= 256 and cout % 8 == 0


def _wgrad_ok(cin: int, cout: int, k: int, dy: torch.Tensor) -> bool:
    """conv_wgrad_'s contract (kernels/gemm.hip launch_conv_wgrad): C a power of two >= 8, Cout >= 256
    (one 256-row tile) and a multiple of 8, R*S*C >= 256, >= 128 output pixels."""
    n, _, ho, wo = dy.shape
    return (cin >= 8 and (cin & (cin - 1)) == 0 and cout >= 256 and cout % 8 == 0 and k * k * cin >= 256
            and n * ho * wo >= 128)


def _igemm(x: torch.Tensor, w2: torch.Tensor, k: int, stride: int, pad: int, bn=None):
    """conv(x, w) on the implicit-GEMM kernel, as a channels_last [N, Cout, Ho, Wo] tensor, or None
    when the kernel declines the shape. With a consumer ``bn`` the epilogue also reduces its batch
    statistics (handed over as for the narrow kernel)."""
    from .. import native

    n, _, h, w = x.shape
    ho, wo = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
    out = torch.empty(n * ho * wo, w2.shape[0], device=x.device, dtype=x.dtype)
    part = _stats_part(bn, n * ho * wo, w2.shape[0], x.device)
    rows = native().conv_fwd_(x, w2, out, k, k, stride, pad, part=part,
                              shift=bn.running_mean if part is not None else None)
    if not rows:
        return None
    y = _from_2d(out, n, ho, wo)
    _hand_stats(bn, y, part, rows)
    return y


def _igemm_fp8(x: torch.Tensor, w2: torch.Tensor, k: int, stride: int, pad: int, e5m2: bool = False,
               scaler: "DelayedScale | None" = None, pre=None, mod=None, bn=None):
    """conv(x, w) with fp8 operands on the implicit-GEMM kernel (per-tensor just-in-time scales; x
    e4m3, or e5m2 when it is an output gradient), bf16 channels_last out, or None when the kernel
    declines the shape."""
    from .. import native

    n, c, h, w = x.shape
    ho, wo = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
    if pre is not None:  # (q channels_last [N, C, H, W], scale_inv) from the producing BN
        xq, sx = pre[0].permute(0, 2, 3, 1), pre[1]
    else:
        xq, sx = _q_act(x.permute(0, 2, 3, 1), e5m2=e5m2, scaler=scaler)  # the NHWC storage, in place order
    wq, sw = _q_weight(mod, w2) if mod is not None else _q_act(w2)
    out = torch.empty(n * ho * wo, w2.shape[0], device=x.device, dtype=x.dtype)
    part = _stats_part(bn, n * ho * wo, w2.shape[0], x.device)
    rows = native().conv_fwd_fp8_(xq.permute(0, 3, 1, 2), wq, sx, sw, out, k, k, stride, pad, part=part,
                                  shift=bn.running_mean if part is not None else None)
    if not rows:
        return None
    FP8_CALLS["dgrad" if e5m2 else "fwd"] += 1
    y = _from_2d(out, n, ho, wo)
    _hand_stats(bn, y, part, rows)
    return y


def _strided_dgrad(mod, dy, weight, to, H: int, W: int):
    """bwd-data of a stride-2 1x1 convolution kept on the quarter grid: t4 = dY . W ([N, Cin, H/2,
    W/2]), queued on ``to`` (the BN that produced the input) as a StridedDr; returns the zero-stride
    marker autograd passes to the block's _Fork (which then queues nothing itself)."""
    n, cout, ho, wo = dy.shape
    cin = weight.shape[1]
    M4 = n * ho * wo
    w2 = weight.reshape(cout, cin)
    dy2 = _as_2d(dy)

    def gemm():
        return _from_2d(torch.mm(dy2, w2), n, ho, wo)

    def psd():  # the persistent 8-phase MFMA GEMM (kernels/gemm.hip)
        out = torch.empty(M4, cin, device=dy.device, dtype=dy.dtype)
        _native().gemm_(dy2, w2, True, False, out)
        return _from_2d(out, n, ho, wo)

    cands = {"gemm": gemm}
    if _psd_ok(cout, cin):
        cands["psd"] = psd
    if _psdn_ok(cout, cin):
        cands.update(_convn_variants(dy, _wt(w2, mod, weight), 1, 1, 0))
    t4 = cands[_choose(("dgrad_s2", M4, cin, cout), cands)]()
    if not t4.is_contiguous(memory_format=torch.channels_last):
        t4 = t4.contiguous(memory_format=torch.channels_last)
    to._psd_pending_dr.append(StridedDr(t4, H, W))
    marker = torch.zeros((), device=dy.device, dtype=dy.dtype).expand(n, cin, H, W)
    mod._psd_strided_marker = marker
    return marker


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride, pad, f8=None, mod=None):
        """``f8``: (activation scaler, gradient scaler) of an fp8 module, else None; ``mod`` as for
        _Conv1x1Fn (dW straight into the PS gradient buffer)."""
        fp8 = f8 is not None
        ctx.mod = mod
        _fwd_records(ctx, mod)
        cout, cin, k, _ = weight.shape
        n, _, h, w = x.shape
        ctx.stride, ctx.pad, ctx.fp8, ctx.f8 = stride, pad, fp8, f8
        ctx.save_for_backward(x, weight)
        if ctx.needs_input_grad[0]:
            if k == 1:
                _wprep.note(mod, weight, "t")
            elif stride == 1 and 2 * pad == k - 1:
                _wprep.note(mod, weight, "f")
            elif stride == 2 and k == 3 and pad == 1:
                _wprep.note(mod, weight, "p")

        def miopen():
            return F.conv2d(x, weight, stride=stride, padding=pad)

        ho_, wo_ = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
        if fp8 and cin % 128 == 0 and _fp8_ok(k * k * cin, cout) and n * ho_ * wo_ >= 128:  # (kernel contract)
            w2 = weight.permute(0, 2, 3, 1).reshape(cout, k * k * cin)
            y = _igemm_fp8(x, w2 if w2.is_contiguous() else w2.contiguous(), k, stride, pad, scaler=f8[0],
                           pre=_take_q8(mod, x), mod=mod, bn=_bn_consumer(mod))
            if y is None:  # the guard above is the kernel's contract: a decline is a bug, not a bf16 run
                raise RuntimeError(f"conv_fwd_fp8_ declined {tuple(x.shape)} x {tuple(weight.shape)}")
            return y

        if not _igemm_ok(cin, cout) and not _psdn_ok(cin, cout):
            return miopen()
        w2 = weight.permute(0, 2, 3, 1).reshape(cout, k * k * cin)
        if not w2.is_contiguous():
            w2 = w2.contiguous()

        def igemm():
            y = _igemm(x, w2, k, stride, pad)
            if y is None:
                raise _at.Declined("conv_fwd_")
            return y

        bn = _bn_consumer(mod)

        def igemm_stats():  # the implicit GEMM with the consumer BN's statistics in its epilogue
            y = _igemm(x, w2, k, stride, pad, bn)
            if y is None:
                raise _at.Declined("conv_fwd_ statistics epilogue")
            return y

        cands = {"miopen": miopen}
        if _igemm_ok(cin, cout):
            cands["igemm"] = igemm
            if bn is not None and _feat("gemm_stats"):
                cands["psds_igemm"] = igemm_stats
        if _psdn_ok(cin, cout):
            cands.update(_convn_variants(x, w2, k, stride, pad, bn))
        key = ("fwd", n, cin, h, w, cout, k, stride)
        return cands[_route(("conv",) + key, cands, "miopen", bn if len(cands) > 1 else None)]()

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        stride, pad = ctx.stride, ctx.pad
        cout, cin, k, _ = weight.shape
        n, _, h, w = x.shape
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        conv_bwd = torch.ops.aten.convolution_backward
        args = (None, [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1)
        dx = dw = None
        to = ctx.strided_to
        if (ctx.needs_input_grad[0] and to is not None and k == 1 and stride == 2 and pad == 0 and h % 2 == 0
                and w % 2 == 0 and _feat("convn_bwd5")):
            # downsample conv whose input gradient goes to the producing BN (the block's _Fork): dY . W
            # on the quarter grid only, handed over as a StridedDr (the consumer convolution's bwd-data
            # adds it at even pixels, kernels/convn.hip mode 5, or the BN's own backward materialises
            # it -- ops/bn.py take_dr -- where the consumer is an fp8 convolution); autograd gets a
            # zero-stride marker. (fp8 downsample convolutions too: their bf16 bwd-data went to MIOpen's
            # zero-fill + implicit GEMM, 3 launches / 0.6 ms per Wide-ResNet-101-2 step)
            dx = _strided_dgrad(ctx.mod, dy, weight, to, h, w)
        if ctx.needs_input_grad[0] and dx is None:
            def miopen():
                return conv_bwd(dy, x, weight, *args, [True, False, False])[0]

            if stride == 1 and _igemm_ok(cout, cin) and 2 * pad == k - 1 and ctx.fp8 and cout % 128 == 0 \
                    and _fp8_ok(k * k * cout, cin) and n * h * w >= 128 and _feat("fp8_dgrad"):
                # fp8 bwd-data: e5m2 dY gathered by the implicit GEMM, e4m3 flipped weights
                wf = _wflip(ctx.mod, weight)
                got = _take_dq8(ctx.mod, dy) if _mx_on() else None
                dx = _igemm_fp8(dy, wf, k, 1, pad, e5m2=True, scaler=ctx.f8[1], pre=got)
                if dx is None:
                    raise RuntimeError(f"conv_fwd_fp8_ (bwd-data) declined {tuple(dy.shape)} x {tuple(weight.shape)}")
            elif stride == 1 and (_igemm_ok(cout, cin) or _psdn_ok(cout, cin)) and 2 * pad == k - 1:
                # dX = conv(dY, W'), W'[ci, r, s, co] = W[co, ci, k-1-r, k-1-s]: same kernel, same padding
                wf = _wflip(ctx.mod, weight)

                def igemm():
                    y = _igemm(dy, wf, k, 1, pad)
                    if y is None:
                        raise _at.Declined("conv_fwd_ (bwd-data)")
                    return y

                cands = {"miopen": miopen}
                if _igemm_ok(cout, cin):
                    cands["igemm"] = igemm
                fu = None
                if _psdn_ok(cout, cin):
                    cands.update(_convn_variants(dy, wf, k, 1, pad))
                    fu = _bn_bwd_fusion(ctx.bn_in, x)
                    if fu is not None:
                        fu["dr"] = fu["bn"]._psd_pending_dr.pop() if fu["mode"] >= 2 else None
                        cands.update(_convn_bwd_variants(dy, wf, k, pad, fu, fu["dr"]))
                key = ("dgrad", n, cin, h, w, cout, k, stride)
                dx = _dgrad_route(("conv",) + key, cands, "miopen", fu, x)
            elif stride == 2 and k == 3 and pad == 1 and h == 2 * dy.shape[2] and w == 2 * dy.shape[3] \
                    and _psdn_ok(cout, cin) and _feat("dgrad_s2_phase") \
                    and x.is_contiguous(memory_format=torch.channels_last) \
                    and dy.is_contiguous(memory_format=torch.channels_last):
                # four output-parity phases of the narrow kernel vs MIOpen (its bwd-data zero-fills dX
                # first), with bn1's backward reduction in the epilogue where that wins (bf16, as the
                # fp8 convolutions' strided bwd-data was: Wide-ResNet-101-2's layer 2-4 conv2)
                fu = _bn_bwd_fusion(ctx.bn_in, x)
                if fu is not None and fu["mode"] != 1:
                    fu = None
                if fu is not None:
                    fu["dr"] = None
                cands = {"miopen": miopen}
                cands.update(_dgrad_s2_phases(dy, weight, x, fu, ctx.mod))
                key = ("dgrad", n, cin, h, w, cout, k, stride)
                dx = _dgrad_route(("conv",) + key, cands, "miopen", fu, x)
            else:
                dx = miopen()
        if ctx.needs_input_grad[1]:
            sv = _sink_view(ctx.mod, weight)

            def miopen_w():
                return conv_bwd(dy, x, weight, *args, [False, True, False])[1]

            def igemm_w(into=None):  # dW = dY^T . im2col(x): split-K implicit GEMM (kernels/gemm.hip)
                o = into if into is not None else torch.empty(cout, k, k, cin, device=dy.device, dtype=dy.dtype)
                if not _native().conv_wgrad_(dy, x, o.view(cout, k * k * cin), k, k, stride, pad):
                    return None
                return o.permute(0, 3, 1, 2)  # OHWI storage = the channels_last [Cout, Cin, k, k] weight

            def igemm_c():
                y = igemm_w()
                if y is None:
                    raise _at.Declined("conv_wgrad_")
                return y

            cands = {"miopen": miopen_w}
            if (_feat("conv_wgrad") and _wgrad_ok(cin, cout, k, dy)
                    and weight.is_contiguous(memory_format=torch.channels_last)):
                cands["igemm"] = igemm_c
            wcands = _convw_cands(dy, x, k, stride, pad) if weight.is_contiguous(
                memory_format=torch.channels_last) else {}
            cands.update(wcands)
            key = ("wgrad", n, cin, h, w, cout, k, stride)
            how = _at.choose(("conv",) + key, cands, "miopen") if len(cands) > 1 else "miopen"
            if how == "igemm":
                dw = igemm_w(sv.permute(0, 2, 3, 1) if sv is not None else None)
                if dw is None:
                    raise RuntimeError(f"conv_wgrad_ declined {key} after it was chosen")
            elif how in wcands:
                ohwi = sv.permute(0, 2, 3, 1) if sv is not None else None
                if ohwi is not None and ohwi.is_contiguous():  # the sink itself, in the kernel's layout
                    dw = wcands[how](ohwi.view(cout, -1))
                    if dw is not None:
                        dw = sv
                else:
                    dw = wcands[how]()
                    if dw is not None and sv is not None:
                        dw = sv.copy_(dw)
                if dw is None:
                    raise RuntimeError(f"convw_ {how} declined {key} after it was chosen")
            else:
                dw = miopen_w()
                if sv is not None:
                    dw = sv.copy_(dw)
        return dx, dw, None, None, None, None


class ConvNHWC(nn.Conv2d):
    """``nn.Conv2d(cin, cout, k, stride, padding=k//2, bias=False)`` whose NHWC bf16 training path
    runs forward (and a stride-1 bwd-data) on the implicit-GEMM kernel where that is faster than
    MIOpen (per shape, validated; see module docstring)."""

    def __init__(self, cin: int, cout: int, k: int, stride: int = 1, fp8: bool = False):
        super().__init__(cin, cout, k, stride=stride, padding=k // 2, bias=False)
        self.fp8 = fp8  # fp8 forward (e4m3 implicit GEMM) and stride-1 bwd-data (e5m2 dY) where allowed
        self._f8 = (DelayedScale(1.0), DelayedScale(2.0))  # input activations, output gradient

    def psd_direct_grad_params(self):
        return [self.weight]

    def psd_fp8_dgrad(self) -> bool:
        """True when this module's stride-1 bwd-data runs in fp8 (implicit GEMM on e5m2 dY)."""
        k, cin, cout = self.kernel_size[0], self.in_channels, self.out_channels
        return (self.fp8 and self.stride[0] == 1 and 2 * self.padding[0] == k - 1 and _igemm_ok(cout, cin)
                and cout % 128 == 0 and _fp8_ok(k * k * cout, cin) and _enabled() and _feat("fp8_dgrad")
                and _feat("conv_igemm"))

    def psd_fp8_consumes(self, cin: int) -> bool:
        k = self.kernel_size[0]
        return (self.fp8 and cin % 128 == 0 and _fp8_ok(k * k * cin, self.out_channels) and _enabled()
                and _feat("conv_igemm"))

    def forward(self, x):
        if (_enabled() and _feat("conv_igemm") and x.is_cuda and x.dtype == torch.bfloat16
                and x.dim() == 4 and self.weight.dtype == torch.bfloat16 and self.groups == 1
                and self.dilation == (1, 1) and x.is_contiguous(memory_format=torch.channels_last)
                and self.weight.is_contiguous(memory_format=torch.channels_last)):
            return _ConvFn.apply(x, self.weight, self.stride[0], self.padding[0], self._f8 if self.fp8 else None,
                                 self)
        return F.conv2d(x, self.weight, stride=self.stride, padding=self.padding)


# ---------------------------------------------------------------------------------------------
# ResNet stem: conv 7x7/s2/p3 (3 -> 64) + BN + ReLU + 3x3/s2 max-pool


class _StemFn(torch.autograd.Function):
    """Forward: the gfx950 stem convolution (kernels/stem.hip, BN statistics in its epilogue) and
    the fused BN + ReLU + max-pool; nothing between the image and the pooled map is written except
    the conv output the BN backward needs. Backward: the pool-fused BN backward, then the weight
    gradient on the gfx950 stem wgrad kernel (the image needs no gradient)."""

    @staticmethod
    def forward(ctx, x, w, bn_w, bn_b, bn, pool):
        from .. import native

        y, arg, mean, invstd, ss, conv_out = native().stem_fwd(
            x, w, bn_w, bn_b, bn.running_mean, bn.running_var, bn.momentum if bn.momentum is not None else 0.1, bn.eps,
            bn.num_batches_tracked)
        ctx.bn, ctx.pool = bn, pool
        ctx.save_for_backward(x, w, conv_out, arg, bn_w, mean, invstd, ss)
        return y

    @staticmethod
    def backward(ctx, gy):
        from .. import native

        x, w, conv_out, arg, bn_w, mean, invstd, ss = ctx.saved_tensors
        sink = getattr(ctx.bn, "_psd_grad_sink", None)
        dgo = dbo = None
        if sink is not None:
            dgo, dbo = sink(ctx.bn.weight), sink(ctx.bn.bias)
        pend = getattr(ctx.pool, "_psd_pending_dr", None)
        gy2 = pend.pop() if pend else None
        dconv, dg, db = native().bn_pool_bwd(gy, gy2, arg, conv_out, bn_w, mean, invstd, ss, dgo, dbo)
        dw = native().stem_wgrad(x, dconv) if ctx.needs_input_grad[1] else None
        return None, dw, dg, db, None, None


def stem_forward(conv: nn.Conv2d, bn, pool, x: torch.Tensor) -> torch.Tensor:
    """``pool(relu(bn(conv(x))))`` for the ResNet stem: the fused gfx950 path when training on a
    supported shape, else the composition (``ops.bn.bn_relu_maxpool`` after ``conv``)."""
    from .bn import bn_relu_maxpool

    w = conv.weight
    if (_enabled() and bn.training and bn.relu and torch.is_grad_enabled() and x.is_cuda and x.dim() == 4
            and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and tuple(w.shape) == (64, 3, 7, 7)
            and conv.stride == (2, 2) and conv.padding == (3, 3) and conv.bias is None and not x.requires_grad
            and bn.weight is not None and bn.weight.dtype == torch.bfloat16 and bn.running_mean is not None
            and x.shape[2] % 8 == 0 and x.shape[3] % 32 == 0 and x.shape[3] <= 352):
        pool.native_last = True
        return _StemFn.apply(x, w, bn.weight, bn.bias, bn, pool)
    return bn_relu_maxpool(bn, pool, conv(x))
