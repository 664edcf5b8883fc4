"""Sharded parameter server over RCCL collectives, colocated with the workers (one rank per GPU).

Every rank is a worker; P of the ranks also hold PS shards (P = world by default: every GPU is a
PS shard). The model's parameters live in ONE flat bf16 working buffer (the model's ``.data`` are
views into it) and their gradients in one flat bf16 buffer (``.grad`` views), both laid out in
gradient-ready (reverse registration) order and cut into buckets of ``bucket_mb``. Each bucket is
split into P equal slices; slice k is owned by PS shard k, which keeps the fp32 master copy and the
optimizer state for it in HBM.

Per bucket, as soon as backward has accumulated all of its gradients (post-accumulate-grad hook,
on a dedicated comm stream, overlapped with the rest of backward):

  push   RS(grad bucket) -> owner slices      (reduce per slice when P < world)
  apply  fused gfx950 kernel: grad/W -> SGD|momentum|Adam(W) on the fp32 master slice -> bf16
         slice written straight into the working buffer
  pull   AG(working bucket) in place          (broadcast per slice when P < world)

Staleness: with ``staleness=S`` the apply at step t uses the gradient pushed at step t-S (kept in
S+1 rotating slots), i.e. every update is applied exactly S versions after the weights it was
computed on (bounded-staleness / SSP semantics; S=0 is the reference's synchronous barrier,
src/parameter_server.cpp:37). Versions and the staleness histogram are kept by the native
``StalenessTracker``.

A bucket's weights are never read again in the same backward once all of its gradients have been
accumulated (each weight's dgrad and wgrad come from the same autograd node), so updating and
re-gathering it during backward is race-free. Tied weights (a parameter used by two nodes) would
break that invariant; such models must pass ``overlap=False``.
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass, field

import torch
import torch.nn as nn

from .. import native
from ..ops import multi_reduce_
from ..ops.optim import OptimConfig, OptimDyn, advance_, apply_no_advance_
from ..utils.config import feature
from .transport import LocalTransport, Transport

ALIGN = 64  # elements: every tensor starts 128-B aligned in the bf16 buffers


def _round(x: int, a: int) -> int:
    return (x + a - 1) // a * a


@dataclass
class Bucket:
    index: int
    params: list = field(default_factory=list)  # (name, param, offset_in_flat, numel)
    offset: int = 0  # element offset in the flat buffers
    numel: int = 0  # padded: multiple of P * ALIGN
    slice_numel: int = 0
    local_offset: int = 0  # offset of this rank's owned slice inside the local shard buffers
    pending: int = 0
    launched: bool = False


def zero_plan(spans, total: int, max_ranges: int = 8):
    """Ranges of a flat gradient buffer to zero before a step: the merged ``(offset, numel)`` spans of
    the parameters whose gradients are *accumulated* into their views (everything but the grad-sink
    params, whose kernels overwrite their views). ``None`` (zero the whole buffer in one launch)
    when that is most of the buffer or would take more than ``max_ranges`` launches. BERT-base:
    the embeddings only, 24M of 110M elements."""
    merged = []
    for off, n in sorted(spans):
        if merged and off <= merged[-1][0] + merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], off + n - merged[-1][0])
        else:
            merged.append([off, n])
    if len(merged) > max_ranges or sum(n for _, n in merged) > total // 2:
        return None
    return [tuple(r) for r in merged]


def zero_grads_(flat: torch.Tensor, plan) -> None:
    if plan is None:
        flat.zero_()
        return
    for off, n in plan:
        flat.narrow(0, off, n).zero_()


def install_fp8_weights(model: nn.Module, resolve) -> None:
    """Give every fp8 module (``fp8 = True``) a ``_psd_w8(w2)`` hook that returns the MX e4m3 copy
    of its weight the data plane pulled with the bf16 working copy -- views (q [Cout, K], E8M0
    scales [Cout*K/32]) into the flat fp8 buffers -- or None when the weight is not in them.
    ``resolve()`` -> (q_flat, scale_flat, params_flat) of the current working buffers (AsyncPS
    alternates two)."""
    for m in model.modules():
        w = getattr(m, "weight", None)
        if not getattr(m, "fp8", False) or not isinstance(w, nn.Parameter):
            continue

        def pub(w2, m=m):
            bufs = resolve()
            if bufs is None:
                return None
            qf, sf, pf = bufs
            wt = m.weight
            off = (wt.data_ptr() - pf.data_ptr()) // wt.element_size()
            n = wt.numel()
            if off < 0 or off + n > pf.numel() or off % 32 or n % 32 or w2.numel() != n:
                return None
            return qf.narrow(0, off, n).view(w2.shape), sf.narrow(0, off // 32, n // 32)

        m._psd_w8 = pub


def _flat_view(flat: torch.Tensor, off: int, p: torch.Tensor) -> torch.Tensor:
    """View of ``flat[off:off+numel]`` with the same shape *and strides* as ``p`` (channels_last
    conv weights stay channels_last)."""
    n = p.numel()
    seg = flat.narrow(0, off, n)
    if p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last) and not p.is_contiguous():
        o, i, kh, kw = p.shape
        return seg.view(o, kh, kw, i).permute(0, 3, 1, 2)
    return seg.view(p.shape)


class CollectivePS:
    def __init__(self, model: nn.Module, optim: OptimConfig, transport: Transport | None = None,
                 num_shards: int | None = None, staleness: int = 0, bucket_mb: float = 16.0,
                 overlap: bool = True, grad_dtype: torch.dtype = torch.bfloat16,
                 param_dtype: torch.dtype = torch.bfloat16, device: torch.device | None = None,
                 ps_ranks: list[int] | None = None, worker_ranks: list[int] | None = None,
                 pull_dtype: str = "bf16", push_mode: str = "auto"):
        self.model = model
        self.cfg = optim
        self.t = transport or LocalTransport()
        self.world, self.rank = self.t.world, self.t.rank
        # world 1 with the local transport: push / pull are identities and are skipped; any other
        # transport (RCCL at world 1 in tests) runs the real collectives
        self._trivial = self.world == 1 and isinstance(self.t, LocalTransport)
        # placement: by default every rank is a worker and the P shards are spread evenly over the
        # node (2 of 8 -> ranks 0 and 4); ps_ranks / worker_ranks give disjoint placements
        # (e.g. 4 PS GPUs + 4 worker GPUs). Non-worker ranks run idle_step(): they take part in the
        # collectives with zero gradients and apply/publish their shards.
        self.worker_ranks = list(worker_ranks) if worker_ranks is not None else list(range(self.world))
        self.is_worker = self.rank in self.worker_ranks
        if ps_ranks is not None:
            self.owners = list(ps_ranks)
            self.P = len(self.owners)
        else:
            self.P = num_shards or self.world
            if not 1 <= self.P <= self.world:
                raise ValueError(f"num_shards must be in [1, world={self.world}], got {self.P}")
            self.owners = [k * self.world // self.P for k in range(self.P)]
        if not self.owners or any(not 0 <= r < self.world for r in self.owners) or len(set(self.owners)) != self.P:
            raise ValueError(f"invalid PS ranks {self.owners} for world {self.world}")
        self.my_shards = [k for k, r in enumerate(self.owners) if r == self.rank]
        self.collective_rs = self.owners == list(range(self.world))  # every rank owns its slice
        # push when not every rank owns a slice: "reduce" = one RCCL reduce per slice onto its owner
        # (a ring through every rank); "p2p" = grouped send of slice k from each worker straight to
        # owner k into a per-worker inbox, summed by the fused apply's multi-source reduce (the
        # SURVEY 5.8 plan for PS shards that are fewer than / disjoint from the workers).
        if push_mode not in ("auto", "reduce", "p2p"):
            raise ValueError(f"push_mode must be auto|reduce|p2p, got {push_mode}")
        self.push_p2p = (not self.collective_rs) and self.world > 1 and push_mode == "p2p"
        self.remote_workers = [w for w in self.worker_ranks if w != self.rank]
        if self.push_p2p and len(self.worker_ranks) > 16:
            raise ValueError("p2p push sums at most 16 worker sources per shard")
        self.S = int(staleness)
        self.overlap = overlap
        self.device = device or next(model.parameters()).device
        self.is_cuda = self.device.type == "cuda"
        if grad_dtype != param_dtype:
            raise ValueError("grad_dtype must equal param_dtype (.grad views must match the parameter dtype)")
        self.grad_dtype, self.param_dtype = grad_dtype, param_dtype
        C = native()
        self.tracker = C.StalenessTracker(self.P, 64)
        self.step_idx = 0

        params = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        params.reverse()  # gradient-ready order ~ reverse of registration
        elem = torch.finfo(param_dtype).bits // 8
        cap = max(ALIGN, int(bucket_mb * (1 << 20)) // elem)
        gran = self.P * ALIGN
        buckets: list[Bucket] = []
        cur = Bucket(0)
        off = 0
        for name, p in params:
            n = p.numel()
            cur.params.append((name, p, off, n))
            off += _round(n, ALIGN)
            if off - cur.offset >= cap:
                cur.numel = _round(off - cur.offset, gran)
                off = cur.offset + cur.numel
                buckets.append(cur)
                cur = Bucket(len(buckets), offset=off)
        if cur.params:
            cur.numel = _round(off - cur.offset, gran)
            off = cur.offset + cur.numel
            buckets.append(cur)
        self.buckets = buckets
        self.total = off
        lo = 0
        for b in buckets:
            b.slice_numel = b.numel // self.P
            b.local_offset = lo
            lo += b.slice_numel * len(self.my_shards)
        self.local_total = lo

        dev = self.device
        # fp32 staging of the initial values (rank-consistent init is the caller's job: same seed)
        init = torch.zeros(self.total, dtype=torch.float32, device=dev)
        for b in buckets:
            for _, p, o, _n in b.params:
                _flat_view(init, o, p).copy_(p.detach().float())
        self.params_flat = init.to(param_dtype)
        self.grads_flat = torch.zeros(self.total, dtype=grad_dtype, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        self.master = torch.zeros(max(self.local_total, ALIGN), **f32)
        self.state1 = torch.zeros_like(self.master) if optim.num_states >= 1 else None
        self.state2 = torch.zeros_like(self.master) if optim.num_states >= 2 else None
        for b in buckets:
            for j, k in enumerate(self.my_shards):
                src = init.narrow(0, b.offset + k * b.slice_numel, b.slice_numel)
                self.master.narrow(0, b.local_offset + j * b.slice_numel, b.slice_numel).copy_(src)
        del init
        # gradient slots for bounded staleness (slot s holds the reduced owned slices of one step)
        # (S = 0 reduces in place inside the gradient buffer and needs none)
        self.slots = [torch.zeros(max(self.local_total, ALIGN), dtype=grad_dtype, device=dev)
                      for _ in range(self.S + 1)] if self.S > 0 else []
        self.dyn = OptimDyn(dev, lr=optim.lr, grad_scale=1.0 / len(self.worker_ranks))
        # p2p inbox: one slice per (owned shard, remote worker)
        self.inbox = torch.zeros(max(self.local_total * len(self.remote_workers), ALIGN), dtype=grad_dtype,
                                 device=dev) if self.push_p2p and self.my_shards else None
        # fp8 pull (Wide-ResNet fp8-weights config): owners quantise their fp32 master slices to OCP
        # e4m3fn with a per-(bucket, shard) amax scale; the all-gather moves 1 byte/param (half of
        # bf16) and every rank dequantises into its bf16 working buffer.
        if pull_dtype not in ("bf16", "fp8"):
            raise ValueError(f"pull_dtype must be bf16 or fp8, got {pull_dtype}")
        self.pull_fp8 = pull_dtype == "fp8" and param_dtype == torch.bfloat16
        # MX (default): one E8M0 scale per 32 elements (ALIGN = 64 keeps every tensor and every
        # shard slice block-aligned, so slices quantise independently, with no amax reduction); the
        # fp8 convolutions consume the pulled e4m3 weights + scales directly (install_fp8_weights)
        self.pull_mx = self.pull_fp8 and feature("fp8_mx") and self.is_cuda
        if self.pull_fp8:
            self.p8 = torch.zeros(self.total, dtype=torch.float8_e4m3fn, device=dev)
            self.p8_scale = torch.ones(len(buckets) * self.P, dtype=torch.float32, device=dev)
            self.p8_amax = torch.zeros(len(buckets) * self.P, dtype=torch.float32, device=dev)
            self.p8_mx = torch.full((self.total // 32,), 127, dtype=torch.uint8, device=dev) if self.pull_mx else None

        # Modules that can write their parameter gradients straight into our flat buffer (fused BN)
        # get a grad sink; their params keep .grad = None so autograd adopts the written view
        # instead of launching an accumulate kernel.
        self._grad_views = {}
        self._direct = set()
        for m in model.modules():
            if hasattr(m, "psd_direct_grad_params"):
                for dp in m.psd_direct_grad_params():
                    if dp is not None and dp.requires_grad:
                        self._direct.add(id(dp))
                m._psd_grad_sink = self._sink
        # re-point the model at the flat buffers
        for b in buckets:
            for _, p, o, _n in b.params:
                p.data = _flat_view(self.params_flat, o, p)
                self._grad_views[id(p)] = _flat_view(self.grads_flat, o, p)
                p.grad = None if id(p) in self._direct else self._grad_views[id(p)]
        self._direct_params = [p for b in buckets for (_, p, _o, _n) in b.params if id(p) in self._direct]
        # grad-sink views are overwritten every step: only the accumulated ones need zeroing (a sink
        # param that gets no gradient in a step is zeroed when its bucket is flushed)
        self._zero_plan = zero_plan([(o, p.numel()) for b in buckets for (_, p, o, _n) in b.params
                                     if id(p) not in self._direct], self.grads_flat.numel())
        self._arrived: set = set()
        self._hooks = []
        self._p2b = {}
        for b in buckets:
            for _, p, _o, _n in b.params:
                self._p2b[id(p)] = b
        for b in buckets:
            for _, p, _o, _n in b.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        if self.is_cuda:
            self.comm_stream = torch.cuda.Stream(device=dev)
            self.ready_events = [torch.cuda.Event() for _ in buckets]
        self._advanced = False
        self._next = 0
        self.tracer = None  # utils.trace.StepTracer (set by the Trainer)
        self._sync_init()
        if self.pull_mx:
            install_fp8_weights(model, lambda: (self.p8, self.p8_mx, self.params_flat))

    # ------------------------------------------------------------------ setup
    def _sync_init(self):
        """Make every rank start from the owners' master values (pull v0)."""
        if self.pull_fp8:
            for b in self.buckets:
                for j, k in enumerate(self.my_shards):
                    self._quant_slice(b, k, self.master.narrow(0, b.local_offset + j * b.slice_numel, b.slice_numel))
            for b in self.buckets:
                self._pull(b)
            return
        if self._trivial:
            return
        for b in self.buckets:
            self._pull(b)
        if self.is_cuda:
            torch.cuda.synchronize(self.device)

    def _sink(self, p):
        """Flat-gradient view a fused op may write ``p``'s gradient into (or None)."""
        if id(p) not in self._direct:
            return None
        v = self._grad_views[id(p)]
        # a fresh view (refcount 1) so autograd's AccumulateGrad adopts it instead of cloning
        return v.view(v.shape)

    def memory_bytes(self) -> dict:
        eb = lambda t: 0 if t is None else t.numel() * t.element_size()  # noqa: E731
        return {"params_bf16": eb(self.params_flat), "grads": eb(self.grads_flat), "master": eb(self.master),
                "state": eb(self.state1) + eb(self.state2), "slots": sum(eb(s) for s in self.slots)}

    # ------------------------------------------------------------------ per-step protocol
    def begin_step(self, track: bool = True):
        """Call before forward: zero the gradient buffer and reset bucket bookkeeping."""
        if track:
            self.account_begin()
        zero_grads_(self.grads_flat, self._zero_plan)
        self._arrived = set()
        for p in self._direct_params:
            p.grad = None
        for b in self.buckets:
            b.pending = len(b.params)
            b.launched = False
        self._next = 0
        self._advanced = False

    def account_begin(self):
        """Host bookkeeping of a step's pull (runs per step, also under graph replay)."""
        t = self.step_idx
        for k in self.my_shards:  # in-flight gradient t is tracked as virtual worker t % (S+1)
            self.tracker.on_pull(t % (self.S + 1), k)

    def account_finish(self):
        t = self.step_idx
        if t >= self.S:
            for k in self.my_shards:
                self.tracker.on_apply((t - self.S) % (self.S + 1), k)
        self.step_idx += 1

    def idle_step(self):
        """A PS-only rank's step: zero contribution to the push, apply + publish its shards."""
        self.begin_step()
        self.finish_step()

    def _on_grad(self, p):
        self._arrived.add(id(p))
        if id(p) in self._direct:
            v = self._grad_views[id(p)]
            if p.grad is not None and p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)  # producer did not use the sink (reference / CPU path)
        b = self._p2b[id(p)]
        b.pending -= 1
        if not self.overlap:
            return
        # Launch strictly in bucket order so every rank enqueues the same collective sequence
        # (an out-of-order ready bucket waits for its predecessors).
        while self._next < len(self.buckets) and self.buckets[self._next].pending <= 0:
            self._launch(self.buckets[self._next])
            self._next += 1

    def finish_step(self, track: bool = True):
        """Call after backward: flush buckets whose hooks did not fire and join the comm stream."""
        while self._next < len(self.buckets):
            self._launch(self.buckets[self._next])
            self._next += 1
        if self.is_cuda:
            torch.cuda.current_stream(self.device).wait_stream(self.comm_stream)
        if track:
            self.account_finish()

    def _launch(self, b: Bucket):
        b.launched = True
        if b.pending > 0 and self._zero_plan is not None:  # flushed with gradients missing
            for _, p, _o, _n in b.params:
                if id(p) in self._direct and id(p) not in self._arrived:
                    self._grad_views[id(p)].zero_()
        if self.is_cuda:
            ev = self.ready_events[b.index]
            ev.record(torch.cuda.current_stream(self.device))
            self.comm_stream.wait_event(ev)
            with torch.cuda.stream(self.comm_stream):
                if self.tracer is not None:
                    with self.tracer.comm_span(self.comm_stream):
                        self._push_apply_pull(b)
                else:
                    self._push_apply_pull(b)
        elif self.tracer is not None:
            with self.tracer.comm_span():
                self._push_apply_pull(b)
        else:
            self._push_apply_pull(b)

    # ------------------------------------------------------------------ push / apply / pull
    def _owned_grad_views(self, b: Bucket, slot: int | None):
        """Where the reduced gradient of my owned slices of bucket b lives."""
        out = []
        for j, k in enumerate(self.my_shards):
            if slot is None:  # in-place in the gradient buffer
                out.append(self.grads_flat.narrow(0, b.offset + k * b.slice_numel, b.slice_numel))
            else:
                out.append(self.slots[slot].narrow(0, b.local_offset + j * b.slice_numel, b.slice_numel))
        return out

    def _inbox_views(self, b: Bucket, j: int):
        n = b.slice_numel
        base = (b.local_offset + j * n) * len(self.remote_workers)
        return [self.inbox.narrow(0, base + i * n, n) for i in range(len(self.remote_workers))]

    def _push_p2p(self, b: Bucket, slot: int | None):
        """Workers send slice k to owner k; owners receive one slice per remote worker."""
        g = self.grads_flat.narrow(0, b.offset, b.numel)
        sends, recvs = [], []
        if self.is_worker:
            for k, owner in enumerate(self.owners):
                if owner != self.rank:
                    sends.append((g.narrow(0, k * b.slice_numel, b.slice_numel), owner))
        for j, k in enumerate(self.my_shards):
            recvs += list(zip(self._inbox_views(b, j), self.remote_workers))
        self.t.exchange(sends, recvs)
        self._p2p_sources = {}
        for j, k in enumerate(self.my_shards):
            srcs = self._inbox_views(b, j)
            if self.is_worker:
                srcs.append(g.narrow(0, k * b.slice_numel, b.slice_numel))
            if slot is None:
                self._p2p_sources[j] = srcs  # S = 0: summed inside the fused apply
            else:
                multi_reduce_(self.slots[slot].narrow(0, b.local_offset + j * b.slice_numel, b.slice_numel), srcs)

    def _push(self, b: Bucket, slot: int | None):
        g = self.grads_flat.narrow(0, b.offset, b.numel)
        if self.push_p2p:
            return self._push_p2p(b, slot)
        if self._trivial:
            if slot is not None:
                self._owned_grad_views(b, slot)[0].copy_(g)
            return
        if self.collective_rs:
            dst = self._owned_grad_views(b, slot)[0] if slot is not None else \
                g.narrow(0, self.rank * b.slice_numel, b.slice_numel)
            self.t.reduce_scatter(g, dst)
        else:
            for k, owner in enumerate(self.owners):
                sl = g.narrow(0, k * b.slice_numel, b.slice_numel)
                self.t.reduce(sl, owner)
            if slot is not None:
                for dst, src in zip(self._owned_grad_views(b, slot), self._owned_grad_views(b, None)):
                    dst.copy_(src)

    def _apply(self, b: Bucket, slot: int | None):
        if not self._advanced:
            advance_(self.cfg, self.dyn)
            self._advanced = True
        for j, (k, gv) in enumerate(zip(self.my_shards, self._owned_grad_views(b, slot))):
            if self.push_p2p and slot is None:
                gv = self._p2p_sources[j]
            lo = b.local_offset + j * b.slice_numel
            m = self.master.narrow(0, lo, b.slice_numel)
            s1 = None if self.state1 is None else self.state1.narrow(0, lo, b.slice_numel)
            s2 = None if self.state2 is None else self.state2.narrow(0, lo, b.slice_numel)
            shadow = self.params_flat.narrow(0, b.offset + k * b.slice_numel, b.slice_numel)
            if self.pull_fp8:
                apply_no_advance_(self.cfg, self.dyn, m, gv, s1, s2, None)
                self._quant_slice(b, k, m)
            elif self.param_dtype == torch.bfloat16:  # the kernel writes the bf16 working copy itself
                apply_no_advance_(self.cfg, self.dyn, m, gv, s1, s2, shadow)
            else:  # fp32 working copy (CPU / fp32 runs): publish the master slice
                apply_no_advance_(self.cfg, self.dyn, m, gv, s1, s2, None)
                shadow.copy_(m)

    def _quant_slice(self, b: Bucket, k: int, src: torch.Tensor):
        C = native()
        if self.pull_mx:
            lo = b.offset + k * b.slice_numel
            C.quant_mx_(src, self.p8.narrow(0, lo, b.slice_numel), self.p8_mx.narrow(0, lo // 32, b.slice_numel // 32))
            return
        i = b.index * self.P + k
        amax = self.p8_amax.narrow(0, i, 1)
        amax.zero_()
        C.amax_(src, amax)
        C.quant_fp8_(src, amax, 448.0, self.p8.narrow(0, b.offset + k * b.slice_numel, b.slice_numel),
                     self.p8_scale.narrow(0, i, 1))

    def _pull_fp8(self, b: Bucket):
        C = native()
        if self.pull_mx:
            q = self.p8.narrow(0, b.offset, b.numel)
            mx = self.p8_mx.narrow(0, b.offset // 32, b.numel // 32)
            if not self._trivial:
                q8 = q.view(torch.uint8)
                sl, sl32 = b.slice_numel, b.slice_numel // 32
                if self.collective_rs:
                    self.t.all_gather(q8.narrow(0, self.rank * sl, sl), q8)
                    self.t.all_gather(mx.narrow(0, self.rank * sl32, sl32), mx)
                else:
                    for k, owner in enumerate(self.owners):
                        self.t.broadcast(q8.narrow(0, k * sl, sl), owner)
                        self.t.broadcast(mx.narrow(0, k * sl32, sl32), owner)
            C.dequant_mx_(q, mx, self.params_flat.narrow(0, b.offset, b.numel))
            return
        q = self.p8.narrow(0, b.offset, b.numel).view(torch.uint8)
        sc = self.p8_scale.narrow(0, b.index * self.P, self.P)
        if not self._trivial:
            if self.collective_rs:
                self.t.all_gather(q.narrow(0, self.rank * b.slice_numel, b.slice_numel), q)
                self.t.all_gather(sc.narrow(0, self.rank, 1), sc)
            else:
                for k, owner in enumerate(self.owners):
                    self.t.broadcast(q.narrow(0, k * b.slice_numel, b.slice_numel), owner)
                    self.t.broadcast(sc.narrow(0, k, 1), owner)
        for k in range(self.P):
            lo = b.offset + k * b.slice_numel
            C.dequant_fp8_(self.p8.narrow(0, lo, b.slice_numel), sc.narrow(0, k, 1),
                           self.params_flat.narrow(0, lo, b.slice_numel))

    def _pull(self, b: Bucket):
        if self.pull_fp8:
            return self._pull_fp8(b)
        w = self.params_flat.narrow(0, b.offset, b.numel)
        if self._trivial:
            return
        if self.collective_rs:
            self.t.all_gather(w.narrow(0, self.rank * b.slice_numel, b.slice_numel), w)
        elif self.push_p2p:
            # each owner sends its slice to every other rank directly (one xGMI link per peer)
            sends, recvs = [], []
            for k, owner in enumerate(self.owners):
                sl = w.narrow(0, k * b.slice_numel, b.slice_numel)
                if owner == self.rank:
                    sends += [(sl, r) for r in range(self.world) if r != self.rank]
                else:
                    recvs.append((sl, owner))
            self.t.exchange(sends, recvs)
        else:
            for k, owner in enumerate(self.owners):
                self.t.broadcast(w.narrow(0, k * b.slice_numel, b.slice_numel), owner)

    def _push_apply_pull(self, b: Bucket):
        t = self.step_idx
        if self.S == 0:
            self._push(b, None)
            self._apply(b, None)
        else:
            self._push(b, t % (self.S + 1))
            if t >= self.S:
                self._apply(b, (t - self.S) % (self.S + 1))
        self._pull(b)

    # ------------------------------------------------------------------ reporting / state
    def staleness_histogram(self):
        return list(self.tracker.histogram())

    def staleness_p50(self) -> int:
        return int(self.tracker.percentile(50.0))

    def set_lr(self, lr: float):
        self.dyn.set(lr=lr)

    def state_dict(self) -> dict:
        return {"master": self.master.detach().cpu(), "state1": None if self.state1 is None else self.state1.cpu(),
                "state2": None if self.state2 is None else self.state2.cpu(), "dyn": self.dyn.t.cpu(),
                "slots": [sl.cpu() for sl in self.slots],
                "step_idx": self.step_idx, "rank": self.rank, "world": self.world, "P": self.P,
                "layout": [(b.offset, b.numel, b.local_offset) for b in self.buckets]}

    def load_state_dict(self, sd: dict):
        self.master.copy_(sd["master"])
        if self.state1 is not None:
            self.state1.copy_(sd["state1"])
        if self.state2 is not None:
            self.state2.copy_(sd["state2"])
        self.dyn.t.copy_(sd["dyn"])
        # in-flight (reduced, not yet applied) gradients of the last S steps
        for dst, src in zip(self.slots, sd.get("slots") or []):
            dst.copy_(src)
        self.step_idx = int(sd["step_idx"])
        # re-publish the working copy from the masters (fp8 pull: re-quantise the owned slices,
        # the published fp8 buffers still hold the pre-load weights)
        for b in self.buckets:
            for j, k in enumerate(self.my_shards):
                lo = b.local_offset + j * b.slice_numel
                m = self.master.narrow(0, lo, b.slice_numel)
                if self.pull_fp8:
                    self._quant_slice(b, k, m)
                else:
                    self.params_flat.narrow(0, b.offset + k * b.slice_numel, b.slice_numel).copy_(m)
        for b in self.buckets:
            self._pull(b)

    # ------------------------------------------------------------------ sharded checkpoint
    def _manifest(self) -> dict:
        return {"format": "psd-collective-v1", "world": self.world, "P": self.P, "owners": self.owners,
                "worker_ranks": self.worker_ranks, "staleness": self.S, "step_idx": self.step_idx,
                "optimizer": self.cfg.to_dict(), "total": self.total,
                "buckets": [{"offset": b.offset, "numel": b.numel, "slice": b.slice_numel,
                             "params": [(n, list(p.shape), o, k) for (n, p, o, k) in b.params]}
                            for b in self.buckets]}

    def save(self, prefix: str, blocking: bool = True):
        """Write this rank's PS shards (fp32 masters, optimizer state, step scalars) to
        ``{prefix}.rank{r}.psd`` (atomic, CRC-checked; csrc/checkpoint.cpp) plus rank 0's JSON
        manifest. The device->host copies run on a side stream into pinned memory and, with
        ``blocking=False``, the file write happens on a host thread while training continues.
        Returns the writer thread (or None)."""
        import json
        import threading

        C = native()
        tensors = [self.master, self.dyn.t] + [t for t in (self.state1, self.state2) if t is not None] \
            + list(self.slots)
        if self.is_cuda:
            # Snapshot on the current stream first (HBM->HBM, ~50 us for ResNet-50's state): the
            # next step's fused apply (comm stream, or the replayed graph on this stream) is
            # ordered after it, so the file holds exactly this step. The slow device->host copy
            # then reads the snapshot on a side stream while training continues.
            cur = torch.cuda.current_stream(self.device)
            if getattr(self, "_ckpt_done", None) is not None:
                cur.wait_event(self._ckpt_done)  # the previous D2H still reads the snapshot
            if getattr(self, "_ckpt_snap", None) is None or len(self._ckpt_snap) != len(tensors):
                self._ckpt_snap = [torch.empty_like(t) for t in tensors]
            for s, t in zip(self._ckpt_snap, tensors):
                s.copy_(t)
            side = torch.cuda.Stream(device=self.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                host = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in tensors]
                for h, s in zip(host, self._ckpt_snap):
                    h.copy_(s, non_blocking=True)
            done = torch.cuda.Event()
            done.record(side)
            self._ckpt_done = done
        else:
            host = [t.detach().clone() for t in tensors]
            done = None
        man = self._manifest()
        man["rank"] = self.rank
        man["my_shards"] = self.my_shards
        man_s = json.dumps(man)
        path = f"{prefix}.rank{self.rank}.psd"

        def write():
            if done is not None:
                done.synchronize()
            C.save_native_ckpt(path, man_s, host)
            if self.rank == 0:
                with open(f"{prefix}.manifest.json.tmp", "w") as f:
                    f.write(man_s)
                os.replace(f"{prefix}.manifest.json.tmp", f"{prefix}.manifest.json")

        if blocking:
            write()
            return None
        th = threading.Thread(target=write, name="psd-ckpt", daemon=True)
        th.start()
        return th

    def load(self, prefix: str):
        """Restore this rank's shards from ``save(prefix)`` (same world / shard layout) and
        re-publish the working parameters."""
        import json

        man, ts = native().load_native_ckpt(f"{prefix}.rank{self.rank}.psd")
        m = json.loads(man)
        if m["world"] != self.world or m["owners"] != self.owners or m["total"] != self.total:
            raise ValueError(f"checkpoint layout (world {m['world']}, owners {m['owners']}) does not match this "
                             f"run (world {self.world}, owners {self.owners})")
        sd = {"master": ts[0], "dyn": ts[1], "step_idx": m["step_idx"]}
        k = 2
        if self.state1 is not None:
            sd["state1"] = ts[k]
            k += 1
        if self.state2 is not None:
            sd["state2"] = ts[k]
            k += 1
        sd["slots"] = ts[k:]
        self.load_state_dict(sd)
        if self.is_cuda:
            torch.cuda.synchronize(self.device)

    def export_reference(self, path: str, epoch: int, iteration: int = 0):
        """Gather the fp32 masters and write the reference's binary checkpoint layout on rank 0
        (collective: every rank must call)."""
        full = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        for b in self.buckets:
            for j, k in enumerate(self.my_shards):
                full.narrow(0, b.offset + k * b.slice_numel, b.slice_numel).copy_(
                    self.master.narrow(0, b.local_offset + j * b.slice_numel, b.slice_numel))
        if self.world > 1:
            for b in self.buckets:
                for k, owner in enumerate(self.owners):
                    self.t.broadcast(full.narrow(0, b.offset + k * b.slice_numel, b.slice_numel), owner)
        if self.rank != 0:
            return
        names, shapes, tensors = [], [], []
        for b in self.buckets:
            for (n, p, o, k) in b.params:
                names.append(n)
                shapes.append(list(p.shape))
                tensors.append(full.narrow(0, o, k).cpu())
        native().save_reference_ckpt(path, epoch, iteration, names, shapes, tensors)

    # ------------------------------------------------------------------ elastic resize
    def close(self):
        """Detach from the model (grad hooks, grad sinks) so a new CollectivePS over a different
        world can take it over; the model keeps its current parameter values."""
        for h in self._hooks:
            h.remove()
        self._hooks = []
        for m in self.model.modules():
            if getattr(m, "_psd_grad_sink", None) == self._sink:
                del m._psd_grad_sink
        for p in self.model.parameters():
            p.grad = None
            p.data = p.data.clone()

    def drain(self):
        """Apply the up-to-S reduced gradients still in flight (steps t-S .. t-1) and publish the
        result, so the shard state is complete at a membership change (no update is dropped).
        Collective: every rank of the current world calls it at the same step boundary."""
        t = self.step_idx
        stream = self.comm_stream if self.is_cuda else None
        if stream is not None:
            stream.wait_stream(torch.cuda.current_stream(self.device))
        ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
        with ctx:
            for j in range(max(0, t - self.S), t):  # pending: the gradient of step j is in slot j % (S+1)
                self._advanced = False
                for b in self.buckets:
                    self._apply(b, j % (self.S + 1))
                    self._pull(b)
                for k in self.my_shards:
                    self.tracker.on_apply(j % (self.S + 1), k)
            for s in self.slots:
                s.zero_()
        if stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(stream)

    def _canon_index(self):
        """(flat offset, canonical offset, numel) per parameter, canonical = model.named_parameters
        order without padding -- a layout independent of world size, shard count and buckets."""
        where = {id(p): (o, n) for b in self.buckets for (_, p, o, n) in b.params}
        out, c = [], 0
        for _, p in self.model.named_parameters():
            if id(p) in where:
                o, n = where[id(p)]
                out.append((o, c, n))
                c += n
        return out, c

    def canonical_state(self, root: int) -> dict:
        """Gather the fp32 masters + optimizer state of every shard onto rank ``root`` in the
        canonical layout (collective). Returns the tensors on ``root``, None elsewhere."""
        idx, n = self._canon_index()
        out = {}
        for key, src in (("master", self.master), ("state1", self.state1), ("state2", self.state2)):
            if src is None:
                continue
            full = torch.zeros(self.total, dtype=torch.float32, device=self.device)
            for b in self.buckets:
                for j, k in enumerate(self.my_shards):
                    full.narrow(0, b.offset + k * b.slice_numel, b.slice_numel).copy_(
                        src.narrow(0, b.local_offset + j * b.slice_numel, b.slice_numel))
            if self.world > 1:
                self.t.reduce(full, root)  # owners hold disjoint slices: the sum is the gather
            if self.rank == root:
                canon = torch.empty(n, dtype=torch.float32, device=self.device)
                for o, c, k in idx:
                    canon.narrow(0, c, k).copy_(full.narrow(0, o, k))
                out[key] = canon
        if self.rank != root:
            return None
        out["dyn"] = self.dyn.t.detach().clone()
        return out

    def load_canonical_state(self, sd: dict):
        """Inverse of ``canonical_state`` for this (possibly different) world: every rank passes the
        full canonical tensors; owners keep their slices and every rank publishes the weights."""
        idx, n = self._canon_index()
        for key, dst in (("master", self.master), ("state1", self.state1), ("state2", self.state2)):
            if dst is None or key not in sd:
                continue
            canon = sd[key].to(self.device)
            if canon.numel() != n:
                raise ValueError(f"canonical {key} has {canon.numel()} elements, model has {n}")
            full = torch.zeros(self.total, dtype=torch.float32, device=self.device)
            for o, c, k in idx:
                full.narrow(0, o, k).copy_(canon.narrow(0, c, k))
            for b in self.buckets:
                for j, k in enumerate(self.my_shards):
                    dst.narrow(0, b.local_offset + j * b.slice_numel, b.slice_numel).copy_(
                        full.narrow(0, b.offset + k * b.slice_numel, b.slice_numel))
            if key == "master":
                if self.pull_fp8:
                    for b in self.buckets:
                        for j, k in enumerate(self.my_shards):
                            self._quant_slice(b, k, self.master.narrow(0, b.local_offset + j * b.slice_numel,
                                                                       b.slice_numel))
                        self._pull(b)
                else:
                    self.params_flat.copy_(full)
        if "dyn" in sd:
            self.dyn.t.copy_(sd["dyn"].to(self.dyn.t.device))
            # step count / bias corrections / lr carry over; the 1/W averaging is this world's
            self.dyn.set(grad_scale=1.0 / len(self.worker_ranks))
        for s in self.slots:
            s.zero_()
        self.step_idx = 0

    def full_params_fp32(self) -> dict:
        """Gather the fp32 masters of every shard (for checkpoints / inspection)."""
        return {n: p.detach().float().clone() for n, p in self.model.named_parameters()}

    def num_params(self) -> int:
        return sum(n for b in self.buckets for (_, _, _, n) in b.params)

    def describe(self) -> str:
        return (f"CollectivePS(world={self.world}, shards={self.P} on ranks {self.owners}, staleness={self.S}, "
                f"buckets={len(self.buckets)}, params={self.num_params() / 1e6:.2f}M, transport={self.t.name})")
