"""Asynchronous parameter server: apply-on-arrival with a stale-synchronous bound, over peer memory.

The collective data plane (``collective_ps.CollectivePS``) moves every rank in lock-step: its
"asynchrony" is a fixed S-step gradient delay. This one is the real thing (BASELINE.json config 3,
SURVEY 7.5.2): each PS shard applies each worker's push the moment it lands, versions advance per
push, and a worker blocks only when it would lead the slowest worker by more than S steps.

Per step of a worker (``begin_step`` / grad hooks / ``finish_step``):

  pull    SSP wait (every worker's clock at every shard >= step - S), then DMA-copy each shard's
          latest published snapshot into the working weights (pinned while the copy runs)
  fwd/bwd on the current stream; as each gradient bucket completes (post-accumulate-grad hook) its
          slices are DMA-copied over xGMI straight into this worker's inbox slot on the owning GPU
          (comm stream, overlapped with the rest of backward)
  commit  once the copies have landed, a message (step, pulled versions) is posted to each shard's
          single-producer ring in the shared control block

The owner's native engine thread (``csrc/async_ps.cpp``) applies each message with the fused gfx950
optimizer kernel, writes the bf16 snapshot
into a free publish buffer and advances the shard version, the worker's clock and the staleness
histogram (staleness = shard version at apply - version the gradient was computed on).

Optimizer semantics (``semantics``):

  "round" (default): K-batch asynchronous SGD with K = W. Each shard takes the pushes
          in arrival order, from whichever workers, and every K of them make ONE optimizer step on
          their average with the synchronous hyperparameters (the K inbox slots are summed inside
          the fused apply kernel; above 16, in groups of 16 into fp32 partials first). A worker's clock advances when the round holding its push has
          been applied. At SSP bound 0 the rounds are exactly the synchronous steps (a worker
          cannot push step t+1 before every step-t push is applied), so the trajectory equals the
          synchronous one; at S >= 1 a round may mix steps (stale gradients, bounded by S).
  "push": every push is applied on arrival as its own step, with the per-push hyperparameters of
          ``csrc/async_hyper.h`` (SGD grad x 1/W; momentum beta^(1/W) and a rescaled lr; Adam/AdamW
          beta^(1/W), lr/W), which keep the synchronous per-round EMA horizons and steady-state
          displacement -- lower latency, approximate. Both are pinned against the synchronous
          trajectory in tests/test_async_ps.py.

Layout: the parameters live in one flat working buffer (``.data`` views, reverse registration
order, 64-element aligned) split into P contiguous shards; gradients alternate between two flat
buffers so the next step never waits for the previous step's push copies. One node, one process
per GPU (the control block is POSIX shared memory); ``device=cpu`` runs the identical protocol on
host shared memory (CPU CI / gloo plumbing).

Reference parity: ``ParameterServerCore::receive_gradients`` (src/parameter_server.cpp:18-75)
buffers every push and applies only at the all-worker barrier (:37); there is no async mode and no
version, so none of this has a counterpart beyond the push/pull/apply roles.
"""
from __future__ import annotations

import os
import time
import uuid
from dataclasses import dataclass, field

import torch
import torch.distributed as dist
import torch.nn as nn

from .. import native
from ..ops.optim import OptimConfig, OptimDyn
from ..utils.config import fault, feature
from .collective_ps import ALIGN, _flat_view, _round, install_fp8_weights, zero_grads_, zero_plan




class _NoTransport:
    """The async plane moves tensors by peer-memory DMA, not through a Transport; ``abort`` is the
    hook a failure detector (runtime/elastic.py _Watchdog) calls to fail every blocked wait."""

    name = "ipc"
    capturable = False

    def __init__(self, ps=None):
        self.ps = ps

    def abort(self):
        if self.ps is not None and self.ps.engine is not None:
            self.ps.engine.inject_error("aborted by a failure detector (a peer was declared dead)")


@dataclass
class _Bucket:
    index: int
    params: list = field(default_factory=list)  # (name, param, offset, numel)
    lo: int = 0
    hi: int = 0
    pending: int = 0


def _store_and_group():
    if dist.is_available() and dist.is_initialized():
        return dist.distributed_c10d._get_default_store(), dist.get_rank(), dist.get_world_size()
    return dist.HashStore(), 0, 1


class AsyncPS:
    def __init__(self, model: nn.Module, optim: OptimConfig, num_shards: int | None = None, staleness: int = 1,
                 bucket_mb: float = 16.0, device: torch.device | None = None, ps_ranks: list[int] | None = None,
                 worker_ranks: list[int] | None = None, param_dtype: torch.dtype = torch.bfloat16, nbuf: int = 4,
                 timeout_s: float | None = None, overlap: bool = True, store=None, log: bool = False,
                 semantics: str = "round", pull_dtype: str = "bf16", schedule: str = "free", xfer: str = "auto"):
        """``semantics``: "round" (K-batch async, default) or "push" (apply-on-arrival with the
        per-push hyperparameters of csrc/async_hyper.h); see the module docstring.
        ``schedule`` "fixed" ("round" semantics only): round r holds exactly every worker's step-r
        push and the pull of step t takes exactly version max(t - S, 0) -- every gradient is
        S rounds stale whatever the timing, so an S >= 1 run is bit-for-bit reproducible and equals
        synchronous SGD with S-step-delayed gradients (csrc/async_ps.h set_fixed_schedule). "free"
        (default): rounds in arrival order, pulls of the latest admissible snapshot.
        ``pull_dtype`` "fp8" (the Wide-ResNet fp8-weights config): each owner also publishes the MX
        e4m3 copy of its snapshot (one E8M0 scale per 32 elements, quantised from the fp32 master
        right after the apply, csrc/async_ps.cpp quant_publish); workers pull 1.03 bytes/parameter
        instead of 2, dequantise the bf16 working copy locally and hand the e4m3 weights + scales to
        the fp8 convolutions (no per-step weight quantisation on the worker).
        ``xfer`` (GPU): how pushes and pulls cross to the owners' memory -- "kernel": one scatter /
        gather kernel per bucket push / pull that reads or writes every owner's peer-mapped memory
        at once, one xGMI link per owner (kernels/xfer.hip); "copy": one hipMemcpyAsync per shard
        (one link at a time); "auto" (default): the kernel, falling back to the copies (on every
        rank together, logged in ``xfer_mode``) if its start-up self-test fails."""
        if xfer not in ("auto", "kernel", "copy"):
            raise ValueError(f"xfer must be auto, kernel or copy, got {xfer!r}")
        self.xfer = xfer
        self.model = model
        self.cfg = optim
        st, self.rank, self.world = _store_and_group()
        self.store = store or st
        self.t = _NoTransport(self)
        self.worker_ranks = list(worker_ranks) if worker_ranks is not None else list(range(self.world))
        self.is_worker = self.rank in self.worker_ranks
        self.W = len(self.worker_ranks)
        if ps_ranks is not None:
            self.owners = list(ps_ranks)
        else:
            P = num_shards or self.world
            if not 1 <= P <= self.world:
                raise ValueError(f"num_shards must be in [1, world={self.world}], got {P}")
            self.owners = [k * self.world // P for k in range(P)]
        self.P = len(self.owners)
        self.my_shards = [k for k, r in enumerate(self.owners) if r == self.rank]
        self.S = int(staleness)
        self.overlap = overlap
        self.device = device or next(model.parameters()).device
        self.is_cuda = self.device.type == "cuda"
        if param_dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("AsyncPS publishes bf16 or fp32 weights")
        if pull_dtype not in ("bf16", "fp8"):
            raise ValueError(f"pull_dtype must be bf16 or fp8, got {pull_dtype}")
        self.pull_mx = pull_dtype == "fp8" and param_dtype == torch.bfloat16 and self.is_cuda
        self.param_dtype = param_dtype
        self.step_idx = 0
        if schedule not in ("free", "fixed") or (schedule == "fixed" and semantics != "round"):
            raise ValueError(f"schedule must be 'free' or 'fixed' (fixed: round semantics), got {schedule!r}")
        self.schedule = schedule
        if schedule == "fixed":
            nbuf = max(nbuf, self.S + 2)  # the last S + 1 versions stay published
        self.pulled = [0] * self.P
        timeout_s = float(os.environ.get("PSD_ASYNC_TIMEOUT", timeout_s or 600.0))

        # ---- flat layout (same conventions as CollectivePS: reverse registration, 64-aligned)
        params = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        params.reverse()
        off = 0
        layout = []
        for n, p in params:
            layout.append((n, p, off, p.numel()))
            off += _round(p.numel(), ALIGN)
        total = _round(max(off, ALIGN), self.P * ALIGN)
        self.total = total
        # P contiguous shards, 64-element aligned, balanced by size
        bounds = [_round(total * k // self.P, ALIGN) for k in range(self.P)] + [total]
        self.shard_off = bounds[:-1]
        self.shard_len = [bounds[k + 1] - bounds[k] for k in range(self.P)]
        self._build_buckets(layout, bucket_mb)

        dev = self.device
        init = torch.zeros(total, dtype=torch.float32, device=dev)
        for n, p, o, k in layout:
            _flat_view(init, o, p).copy_(p.detach().float())
        # working weights: with S >= 1 two buffers alternate per step, so the pull of step t+1 (DMA
        # from the owners' publish buffers) runs on a side stream while step t computes
        # (world 1: the pull is one local device copy, so pulling straight into the working weights at
        # the step start costs less than the prefetch + working-buffer copy -- feature async_direct_pull)
        self.prefetch = self.S >= 1 and not (self.world == 1 and feature("async_direct_pull"))
        self.pbufs = [init.to(param_dtype)]
        if self.prefetch:
            self.pbufs.append(self.pbufs[0].clone())
        # the model's parameters view ONE working buffer; each step copies its pulled buffer into it
        # on the compute stream (_to_work: a ~70 us device copy for BERT-base) instead of re-pointing
        # every parameter from Python (~200 `p.data =` per step: ~1 ms of host time at the step
        # boundary, where the GPU waited for it -- profiles/r5/bert_base_b256_r5_kernels.md)
        self.pwork = self.pbufs[0].clone() if self.prefetch else self.pbufs[0]
        self.cb = 0
        # MX pull targets (one per working buffer): e4m3 [total] + E8M0 scales [total / 32]
        self.q8s = [torch.zeros(total, dtype=torch.float8_e4m3fn, device=dev) for _ in self.pbufs] if self.pull_mx else []
        self.sc8s = [torch.full((total // 32,), 127, dtype=torch.uint8, device=dev) for _ in self.pbufs] \
            if self.pull_mx else []
        self.grads = [torch.zeros(total, dtype=param_dtype, device=dev) for _ in range(2)]
        self.gb = 0
        f32 = dict(dtype=torch.float32, device=dev)
        # per-push hyperparameters (module docstring)
        if semantics not in ("round", "push"):
            raise ValueError(f"semantics must be 'round' or 'push', got {semantics!r}")
        self.semantics = semantics
        # K = W: every round completes (a cap below W would strand a partial round at W > 16 and
        # hold a worker's clock back forever); the engine pre-reduces above 16 sources
        self.round = self.W if semantics == "round" else 1
        if semantics == "push":
            self.hyper = native().async_hyper(optim.code, self.W, optim.momentum, optim.beta1, optim.beta2,
                                              optim.weight_decay)
        else:
            self.hyper = dict(lr_factor=1.0, grad_scale=1.0 / self.round, momentum=optim.momentum, beta1=optim.beta1,
                              beta2=optim.beta2, weight_decay=optim.weight_decay)
        self.master, self.state1, self.state2, self.dyn = {}, {}, {}, {}
        for k in self.my_shards:
            self.master[k] = init.narrow(0, self.shard_off[k], self.shard_len[k]).clone()
            if optim.num_states >= 1:
                self.state1[k] = torch.zeros(self.shard_len[k], **f32)
            if optim.num_states >= 2:
                self.state2[k] = torch.zeros(self.shard_len[k], **f32)
            self.dyn[k] = OptimDyn(dev, lr=optim.lr * self.hyper["lr_factor"], grad_scale=self.hyper["grad_scale"])
        del init

        # grad sinks (fused BN / MFMA linear write their parameter gradients straight into the buffer)
        self._direct = set()
        for m in model.modules():
            if hasattr(m, "psd_direct_grad_params"):
                for dp in m.psd_direct_grad_params():
                    if dp is not None and dp.requires_grad:
                        self._direct.add(id(dp))
                m._psd_grad_sink = self._sink
        self._layout = layout
        self._zero_plan = zero_plan([(o, p.numel()) for (_n, p, o, _k) in layout if id(p) not in self._direct], total)
        self._arrived: set = set()
        for (n, p, o, k) in layout:
            p.data = _flat_view(self.pwork, o, p)
        self._gview_cache = {}
        self._set_grad_views()
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for _, p, _o, _n in layout]
        self._next = 0
        if self.is_cuda:
            # ONE push stream: HIP maps a process's streams onto GPU_MAX_HW_QUEUES = 4 hardware
            # queues, and compute + engine apply + push + pull already take four -- a fifth stream
            # shares a queue with one of them and serialises behind its work (ResNet-50 b1024 async
            # S = 1: 91-95 ms/step with two push streams vs 78 ms synchronous,
            # profiles/async_push_streams_r4.md). The owners' links overlap inside one launch
            # instead (kernels/xfer.hip).
            self.comm_stream = torch.cuda.Stream(device=dev)
            self.comm_streams = [self.comm_stream]
            self.pull_stream = torch.cuda.Stream(device=dev)
            self.push_done = [None, None]
            self.step_done = [None, None]  # end of a step's work on the compute stream, per buffer
            self.pull_done = [None, None]
        self._prefetched = None  # (step, pulled versions) of the pull issued ahead

        # ---- native engine: control block (rank 0 creates), memory exchange, initial publish
        # instance sequence number from the store itself (a per-rank counter key): every rank
        # agrees on it for any store lifetime -- an id(store)-keyed local count could collide when
        # a freed elastic generation's store address is reused on some ranks only
        n = int(self.store.add(f"psd/async/seq/{self.rank}", 1))
        key = f"psd/async/{n}"
        if self.rank == 0:
            self.store.set(f"{key}/shm", f"/psd_{os.getpid()}_{uuid.uuid4().hex[:12]}")
        shm = self.store.get(f"{key}/shm").decode()
        C = native()
        devidx = dev.index if (self.is_cuda and dev.index is not None) else (torch.cuda.current_device()
                                                                            if self.is_cuda else -1)
        if self.rank != 0:
            self.store.wait([f"{key}/ctl"])
        self.engine = C.AsyncEngine(self.rank, self.world, self.owners, self.worker_ranks, self.shard_off,
                                    self.shard_len, self.S, nbuf, shm, self.rank == 0, devidx, timeout_s,
                                    torch.finfo(param_dtype).bits // 8, self.pull_mx)
        if self.rank == 0:
            self.store.set(f"{key}/ctl", b"1")
        try:
            self._connect(key, optim, log)
        except Exception:
            # release this rank's shared memory / IPC mappings before the (collective) error escapes
            self.engine.stop()
            self.engine.close_peers()
            self.engine.free_local()
            self.engine = None
            raise
        self.tracer = None
        self.closed = False
        self._ckpt_seq = 0
        if self.pull_mx:  # the fp8 convolutions read the pulled e4m3 weights of the current buffer
            install_fp8_weights(model, lambda: (self.q8s[self.cb], self.sc8s[self.cb], self.pwork))

    def _connect(self, key, optim, log):
        """Exchange memory descriptors, map the peers, publish version 0, self-test, start."""
        self._key = key
        self.store.set(f"{key}/desc/{self.rank}", self.engine.local_desc())
        err = ""
        try:
            for r in range(self.world):
                self.engine.attach_peer(r, self.store.get(f"{key}/desc/{r}"))
        except Exception as e:  # noqa: BLE001 -- reported collectively below
            err = f"rank {self.rank}: {e}"
        self._agree("attach", err)
        for k in self.my_shards:
            h = self.hyper
            self.engine.set_shard_state(k, self.master[k], self.state1.get(k), self.state2.get(k), self.dyn[k].t,
                                        optim.code, h["momentum"], optim.dampening, optim.nesterov,
                                        h["weight_decay"], h["beta1"], h["beta2"], optim.eps)
            self.engine.publish_initial(k)
        self.engine.set_round(self.round)
        self.engine.set_fixed_schedule(self.schedule == "fixed")
        if log:
            self.engine.enable_log(True)
        self._barrier("init")
        self.xfer_fallback = None
        if self.is_cuda:
            self.engine.set_xfer(self.xfer != "copy")
        try:
            self.selftest("kernel" if self.is_cuda and self.xfer != "copy" else "copy")
        except RuntimeError as e:  # collective: every rank sees the same failure
            if not (self.is_cuda and self.xfer == "auto"):
                raise
            self.xfer_fallback = str(e)[:300]
            self.engine.set_xfer(False)
            self.selftest("copy")
        self.xfer_mode = self.engine.xfer_mode()
        self.engine.start()

    def selftest(self, attempt: str = "copy"):
        """Collective start-up check of the peer-memory paths on this node (before any training):
        every worker DMA-writes a known pattern into its inbox on every shard owner, and every
        owner verifies what landed; every worker pulls the version-0 snapshots and compares each
        shard with its owner's published checksum (the ranks' weights need not agree yet: an elastic
        joiner's are replaced by load_canonical_state next). Raises on any mismatch on any rank (so a
        caller can fall back to the collective plane instead of training on a broken path).

        ``attempt`` ("kernel" / "copy": the transport under test) tags every store key of this
        attempt -- checksums, barrier, verdict -- so a retry after a failed kernel-path attempt never
        meets the first attempt's counters (a reused barrier key is already at world size and would
        let an owner check its inbox before the workers' second pushes landed)."""
        dev = self.device
        tag = f"{attempt}"
        ok, why = True, ""
        for k in self.my_shards:  # the snapshot each owner published: bf16/fp32(master)
            v = self.master[k].to(self.param_dtype).double()
            self.store.set(f"{self._key}/ck/{tag}/{k}", f"{float(v.sum())!r} {float(v.abs().sum())!r}")
        if self.is_worker:
            pat = (torch.arange(self.total, device=dev) % 251 + (self.rank + 1)).to(self.param_dtype)
            self.engine.push(0, pat, 0, self.total, self._stream_ptr())
            got = torch.empty_like(self.params_flat)
            self.engine.pull(0, got, self._stream_ptr())
            if self.is_cuda:
                torch.cuda.synchronize(dev)
            for k in range(self.P):
                self.store.wait([f"{self._key}/ck/{tag}/{k}"])
                want_s, want_a = (float(x) for x in self.store.get(f"{self._key}/ck/{tag}/{k}").decode().split())
                sl = got.narrow(0, self.shard_off[k], self.shard_len[k]).double()
                if abs(float(sl.sum()) - want_s) > 1e-6 * max(want_a, 1.0) or \
                        abs(float(sl.abs().sum()) - want_a) > 1e-6 * max(want_a, 1.0):
                    ok, why = False, f"rank {self.rank}: pulled shard {k} != its owner's snapshot"
        if fault("selftest_fail_rank") == self.rank:  # fault injection (tests)
            ok, why = False, f"rank {self.rank}: injected self-test failure"
        if attempt == "kernel" and fault("selftest_fail_kernel") == self.rank:  # fails the kernel path only
            ok, why = False, f"rank {self.rank}: injected kernel-transport self-test failure"
        self._barrier(f"selftest-push/{tag}")
        for k in self.my_shards:
            for wi, w in enumerate(self.worker_ranks):
                v = self.engine.inbox_view(k, wi, 0)
                want = (torch.arange(self.shard_off[k], self.shard_off[k] + self.shard_len[k], device=dev) % 251
                        + (w + 1)).to(self.param_dtype)
                if not torch.equal(v, want):
                    ok, why = False, f"rank {self.rank}: shard {k} inbox of worker {w} holds wrong data"
                v.zero_()
        if self.is_cuda:
            torch.cuda.synchronize(dev)
        self._agree("selftest", "" if ok else why, attempt=tag)
        self.selftest_ok = True

    def _agree(self, tag: str, err: str, attempt: str = ""):
        """Collective status exchange through the store: every rank raises if any rank failed.
        ``attempt`` keeps the keys of a retried exchange apart from the earlier ones."""
        key = f"{self._key}/{tag}" + (f"/{attempt}" if attempt else "")
        self.store.set(f"{key}/{self.rank}", err or "ok")
        errs = []
        for r in range(self.world):
            self.store.wait([f"{key}/{r}"])
            v = self.store.get(f"{key}/{r}").decode()
            if v != "ok":
                errs.append(v)
        if errs:
            raise RuntimeError(f"AsyncPS {tag} failed: " + "; ".join(errs))

    # ------------------------------------------------------------------ helpers
    @property
    def params_flat(self) -> torch.Tensor:
        """The working weights of the current step (the buffer the model's parameters view)."""
        return self.pwork

    def _barrier(self, tag: str):
        if self.world == 1:
            return
        k = f"{self._key}/bar/{tag}"
        self.store.add(k, 1)
        import time

        t0 = time.time()
        while int(self.store.add(k, 0)) < self.world:
            if time.time() - t0 > 600:
                raise RuntimeError(f"AsyncPS barrier {tag} timed out")
            time.sleep(0.001)

    def _stream_ptr(self, s=None) -> int:
        if not self.is_cuda:
            return 0
        s = s or torch.cuda.current_stream(self.device)
        return s.cuda_stream

    def _set_grad_views(self):
        views = self._gview_cache.get(self.gb)
        if views is None:  # built once per gradient buffer (two alternate)
            g = self.grads[self.gb]
            views = {id(p): _flat_view(g, o, p) for (_n, p, o, _k) in self._layout}
            self._gview_cache[self.gb] = views
        self._grad_views = views
        for n, p, o, k in self._layout:
            p.grad = None if id(p) in self._direct else views[id(p)]

    def _to_work(self):
        """The pulled buffer of this step into the working weights (stream-ordered on the current
        stream: after the previous step's kernels, before this step's)."""
        if self.pwork is not self.pbufs[self.cb]:
            self.pwork.copy_(self.pbufs[self.cb])

    def _sink(self, p):
        if id(p) not in self._direct:
            return None
        v = self._grad_views[id(p)]
        return v.view(v.shape)

    def memory_bytes(self) -> dict:
        eb = lambda t: t.numel() * t.element_size()  # noqa: E731
        work = eb(self.pwork) if all(self.pwork is not b for b in self.pbufs) else 0
        return {"params": sum(eb(b) for b in self.pbufs) + work, "grads": 2 * eb(self.grads[0]),
                "master": sum(eb(t) for t in self.master.values()),
                "state": sum(eb(t) for t in list(self.state1.values()) + list(self.state2.values()))}

    # ------------------------------------------------------------------ per-step protocol
    def begin_step(self, track: bool = True):
        if not self.is_worker:
            return
        t = self.step_idx
        self.gb = t % 2
        if self.is_cuda and self.push_done[self.gb] is not None:
            # the push copies of step t-2 read this gradient buffer
            torch.cuda.current_stream(self.device).wait_event(self.push_done[self.gb])
        zero_grads_(self.grads[self.gb], self._zero_plan)
        self._arrived = set()
        self._set_grad_views()
        for b in self.buckets:
            b.pending = len(b.params)
        self._next = 0
        if self.prefetch:
            self.cb = t % 2
            if self._prefetched is not None and self._prefetched[0] == t:
                self.pulled = self._prefetched[1]
                if self.is_cuda:
                    torch.cuda.current_stream(self.device).wait_event(self.pull_done[self.cb])
                self._to_work()
                return
        self.pulled = self._pull_into(t, self.cb, None)
        self._to_work()

    def _pull_into(self, t: int, nb: int, stream) -> list:
        """Pull of step t into working buffer ``nb`` on ``stream`` (None: the current stream): the
        bf16 snapshots, or with MX the e4m3 + scales and their bf16 dequantisation."""
        sptr = stream.cuda_stream if stream is not None else self._stream_ptr()
        if not self.pull_mx:
            return list(self.engine.pull(t, self.pbufs[nb], sptr))
        # the engine dequantises into the bf16 buffer on the same stream (fused into the gather)
        return list(self.engine.pull_mx(t, self.q8s[nb], self.sc8s[nb], self.pbufs[nb], sptr))

    def _prefetch_pull(self, t: int):
        """Issue the pull of step t (the next one) now: the SSP wait happens on the host here, the
        DMA on the pull stream, after the step that last used that buffer (t-2) is done with it."""
        nb = t % 2
        if self.is_cuda:
            if self.step_done[nb] is not None:
                self.pull_stream.wait_event(self.step_done[nb])
            pulled = self._pull_into(t, nb, self.pull_stream)
            ev = torch.cuda.Event()
            ev.record(self.pull_stream)
            self.pull_done[nb] = ev
        else:
            pulled = self.engine.pull(t, self.pbufs[nb], 0)
        self._prefetched = (t, list(pulled))

    def _on_grad(self, p):
        self._arrived.add(id(p))
        if id(p) in self._direct:
            v = self._grad_views[id(p)]
            if p.grad is not None and p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)
        b = self._p2b[id(p)]
        b.pending -= 1
        if not self.overlap:
            return
        while self._next < len(self.buckets) and self.buckets[self._next].pending <= 0:
            self._push(self.buckets[self._next])
            self._next += 1

    def _push(self, b: _Bucket):
        g = self.grads[self.gb]
        if b.pending > 0 and self._zero_plan is not None:  # flushed with gradients missing
            for _n, p, _o, _k in b.params:
                if id(p) in self._direct and id(p) not in self._arrived:
                    self._grad_views[id(p)].zero_()
        if self.is_cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            cs = self.comm_streams[b.index % len(self.comm_streams)]
            cs.wait_event(ev)
            self.engine.push(self.step_idx, g, b.lo, b.hi, cs.cuda_stream)
        else:
            self.engine.push(self.step_idx, g, b.lo, b.hi, 0)

    def finish_step(self, track: bool = True):
        if not self.is_worker:
            return
        while self._next < len(self.buckets):
            self._push(self.buckets[self._next])
            self._next += 1
        if self.is_cuda:
            for cs in self.comm_streams[1:]:  # the commit posts after every push copy has landed
                ev = torch.cuda.Event()
                ev.record(cs)
                self.comm_stream.wait_event(ev)
            self.engine.commit(self.step_idx, self.pulled, self.comm_stream.cuda_stream)
            ev = torch.cuda.Event()
            ev.record(self.comm_stream)
            self.push_done[self.gb] = ev
            done = torch.cuda.Event()
            done.record(torch.cuda.current_stream(self.device))
            self.step_done[self.cb] = done
        else:
            self.engine.commit(self.step_idx, self.pulled, 0)
        self.step_idx += 1
        if self.prefetch:
            self._prefetch_pull(self.step_idx)

    def idle_step(self):
        pass

    # ------------------------------------------------------------------ end of run / reporting
    def drain(self):
        """Block until every worker's pushes so far are applied everywhere (collective: all ranks)."""
        steps = torch.tensor([self.step_idx if self.is_worker else 0], dtype=torch.int64)
        if self.world > 1 and dist.is_initialized():
            steps = steps.to(self.device) if dist.get_backend() == "nccl" else steps
            dist.all_reduce(steps, op=dist.ReduceOp.MAX)
        self.engine.wait_all_applied(int(steps.item()))
        if self.is_cuda:
            torch.cuda.synchronize(self.device)

    def refresh_weights(self):
        """After ``drain``: the working weights (the model's parameter views) = the latest applied
        snapshot. Workers otherwise hold the weights of their last pull, one round behind."""
        if self.is_worker and self.engine is not None:
            self.pulled = self._pull_into(0, self.cb, None)
            self._to_work()
            if self.is_cuda:
                torch.cuda.synchronize(self.device)

    def _build_buckets(self, layout, bucket_mb: float):
        """Push buckets: consecutive parameter ranges of ~``bucket_mb`` (the tail padding travels
        with the last bucket)."""
        elem = torch.finfo(self.param_dtype).bits // 8
        cap = max(ALIGN, int(bucket_mb * (1 << 20)) // elem)
        self.buckets: list[_Bucket] = []
        cur = _Bucket(0, lo=0)
        for n, p, o, k in layout:
            cur.params.append((n, p, o, k))
            cur.hi = o + _round(k, ALIGN)
            if cur.hi - cur.lo >= cap:
                self.buckets.append(cur)
                cur = _Bucket(len(self.buckets), lo=cur.hi)
        if cur.params:
            self.buckets.append(cur)
        self.buckets[-1].hi = self.total
        self.bucket_mb = float(bucket_mb)
        self._p2b = {id(p): b for b in self.buckets for _n, p, _o, _k in b.params}

    def rebucket(self, bucket_mb: float):
        """Rebuild the push buckets at another size (between steps; every rank the same size)."""
        self._build_buckets(self._layout, bucket_mb)

    def probe_push_sizes(self, sizes_mb=(1, 2, 4, 8, 16, 32, 64), reps: int = 3) -> dict:
        """The bandwidth of THIS plane's push transport vs bucket size, measured before training
        (collective, every rank): each worker DMA-copies its whole gradient buffer into its inbox
        slot on every owner in chunks of ``size`` MB -- one engine push per chunk on alternating
        push streams, exactly what a step's bucket pushes do (no commit: nothing is applied) --
        and the max over ranks of the time gives {MB: GB/s}. The RCCL send/recv probe
        (parallel/bucketing.py probe_p2p) measures the collective plane's transport, not this one."""
        out = {}
        g = self.grads[0]
        elem = g.element_size()
        for mb in sizes_mb:
            n = max(ALIGN, int(mb * (1 << 20)) // elem // ALIGN * ALIGN)  # chunk ends stay 16-B aligned
            el, err = 0.0, None
            if self.is_worker:
                def run():
                    for i, lo in enumerate(range(0, self.total, n)):
                        cs = self.comm_streams[i % len(self.comm_streams)] if self.is_cuda else None
                        self.engine.push(self.step_idx, g, lo, min(lo + n, self.total),
                                         cs.cuda_stream if cs is not None else 0)
                    if self.is_cuda:
                        for cs in self.comm_streams:
                            cs.synchronize()

                try:  # a failure here must reach every rank (below), not strand them in the all_reduce
                    run()
                    t0 = time.perf_counter()
                    for _ in range(reps):
                        run()
                    el = (time.perf_counter() - t0) / reps
                except Exception as e:  # noqa: BLE001
                    err = e
            t = torch.tensor([el, 1.0 if err is not None else 0.0], dtype=torch.float64)
            if self.world > 1 and dist.is_initialized():
                if dist.get_backend() == "nccl":
                    t = t.to(self.device)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
            if float(t[1]) > 0:
                raise RuntimeError(f"push-size probe failed on a rank{f': {err}' if err is not None else ''}")
            el = float(t[0])
            out[mb] = round(self.total * elem * self.P / max(el, 1e-9) / 1e9, 1) if el > 0 else None
        return out

    def probe_xfer_blocks(self, caps=(8, 16, 24, 32, 48, 64, 96), reps: int = 3, keep: float = 0.9) -> dict:
        """The scatter kernel's workgroup budget (collective, every rank; before training): each
        worker pushes its whole gradient buffer into its inbox slot on every owner in one launch per
        cap, timed (max over ranks). Returns {"GBps": {cap: GB/s}, "chosen": cap}: the SMALLEST cap
        within ``keep`` of the best bandwidth -- the fewest CUs the push takes from the backward
        pass running beside it for (nearly) the same link throughput -- and sets it on the engine.
        Only meaningful where the kernel transport runs (a remote owner); otherwise returns {}."""
        if not (self.is_cuda and self.xfer_mode == "kernel") or all(o == self.rank for o in self.owners):
            remote = False
        else:
            remote = True
        t = torch.tensor([1.0 if remote else 0.0], dtype=torch.float64)
        if self.world > 1 and dist.is_initialized():
            if dist.get_backend() == "nccl":
                t = t.to(self.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if float(t[0]) == 0.0 or not self.is_cuda:
            return {}
        g = self.grads[0]
        old = self.engine.xfer_blocks_cap()
        res = {}
        for cap in caps:
            self.engine.set_xfer_blocks(int(cap))
            el, err = 0.0, None
            if self.is_worker:
                try:
                    st = self.comm_streams[0]
                    self.engine.push(self.step_idx, g, 0, self.total, st.cuda_stream)
                    st.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(reps):
                        self.engine.push(self.step_idx, g, 0, self.total, st.cuda_stream)
                    st.synchronize()
                    el = (time.perf_counter() - t0) / reps
                except Exception as e:  # noqa: BLE001 -- reported collectively below
                    err = e
            t = torch.tensor([el, 1.0 if err is not None else 0.0], dtype=torch.float64)
            if self.world > 1 and dist.is_initialized():
                if dist.get_backend() == "nccl":
                    t = t.to(self.device)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
            if float(t[1]) > 0:
                self.engine.set_xfer_blocks(old)
                raise RuntimeError(f"xfer workgroup probe failed on a rank{f': {err}' if err is not None else ''}")
            el = float(t[0])
            res[int(cap)] = round(self.total * g.element_size() / max(el, 1e-9) / 1e9, 1) if el > 0 else None
        ok = {c: v for c, v in res.items() if v}
        if not ok:  # no worker timed anything (a pure-owner world): keep the default
            self.engine.set_xfer_blocks(old)
            return {"GBps": res, "chosen": old}
        best = max(ok.values())
        chosen = min(c for c, v in ok.items() if v >= keep * best)
        self.engine.set_xfer_blocks(chosen)
        return {"GBps": res, "chosen": chosen}

    def probe_bandwidth(self, reps: int = 3) -> dict:
        """After ``drain``: time this worker's full push (DMA of the whole gradient into its inbox slot
        on every owner, no commit) and a full pull (latest snapshots into a scratch buffer) -- the
        peer-memory data plane's achieved bandwidth on this node (xGMI links at N > 1)."""
        if not (self.is_worker and self.is_cuda):
            return {}
        g = self.grads[0]
        tmp = torch.empty_like(self.params_flat)
        st = torch.cuda.current_stream(self.device)
        out = {}
        for name, fn in (("push", lambda: self.engine.push(self.step_idx, g, 0, self.total, st.cuda_stream)),
                         # step_idx: the latest admissible snapshot under both schedules (a fixed
                         # schedule keeps only the last S + 1 versions; step 0's is long gone)
                         ("pull", lambda: self.engine.pull(self.step_idx, tmp, st.cuda_stream))):
            fn()
            torch.cuda.synchronize(self.device)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                fn()
            e.record()
            e.synchronize()
            ms = s.elapsed_time(e) / reps
            out[f"{name}_GBps"] = round(self.total * g.element_size() / (ms * 1e-3) / 1e9, 1)
        return out

    def abort(self):
        """Non-collective teardown after a failure (a dead peer would never reach close()'s
        barriers): raise the shared error so every peer's waits fail, stop the engine, unmap the
        peers' memory and free this rank's. Pushes not yet applied are lost; recovery restarts from
        a checkpoint (runtime/elastic.py)."""
        if self.closed or self.engine is None:
            return
        try:
            self.engine.inject_error(f"rank {self.rank} aborted")
        except Exception:  # noqa: BLE001
            pass
        self.engine.stop()
        hist, vers, log = self.staleness_histogram(), self.versions(), self.apply_log()
        self._final = (hist, vers, log)
        self.engine.close_peers()
        self.engine.free_local()
        self.engine = None
        self._release_model()
        self.closed = True

    def _release_model(self):
        for h in self._hooks:
            h.remove()
        for m in self.model.modules():
            if getattr(m, "_psd_grad_sink", None) == self._sink:
                del m._psd_grad_sink

    def close(self):
        """Collective: stop the engine, unmap the peers' memory, free this rank's (all ranks call).
        After a failure (the shared error is set) this is ``abort``: no barriers with dead peers."""
        if self.closed:
            return
        if self.engine.error():
            self.abort()
            return
        self.engine.stop()
        self._barrier("stop")
        self.engine.close_peers()
        self._barrier("unmapped")
        hist, vers, log = self.staleness_histogram(), self.versions(), self.apply_log()
        self._final = (hist, vers, log)
        self.engine.free_local()
        self.engine = None
        self._release_model()
        self.closed = True

    def staleness_histogram(self):
        if self.engine is None:
            return list(self._final[0])
        return list(self.engine.histogram())

    def staleness_p50(self) -> int:
        h = self.staleness_histogram()
        tot, acc = sum(h), 0
        for i, c in enumerate(h):
            acc += c
            if tot and acc * 2 >= tot:
                return i
        return -1

    def versions(self) -> list[int]:
        if self.engine is None:
            return list(self._final[1])
        return [int(self.engine.version(k)) for k in range(self.P)]

    def apply_log(self):
        if self.engine is None:
            return list(self._final[2])
        return [tuple(x) for x in self.engine.apply_log()]

    def set_lr(self, lr: float):
        """``lr``: the synchronous (per-round) learning rate; each push runs with its async share."""
        for d in self.dyn.values():
            d.set(lr=lr * self.hyper["lr_factor"])

    def num_params(self) -> int:
        return sum(k for (_, _, _, k) in self._layout)

    def state_dict(self) -> dict:
        """This rank's shard state (call after ``drain``)."""
        return {"master": {k: v.detach().cpu() for k, v in self.master.items()},
                "state1": {k: v.cpu() for k, v in self.state1.items()},
                "state2": {k: v.cpu() for k, v in self.state2.items()},
                "dyn": {k: d.t.cpu() for k, d in self.dyn.items()}, "versions": self.versions(),
                "step_idx": self.step_idx}

    # ------------------------------------------------------------------ checkpoint / resume
    def _quiesce(self):
        """Collective: every push so far applied at every shard, so the masters, optimizer state,
        versions and clocks form one consistent cut."""
        self.drain()

    def _layout_meta(self) -> dict:
        return {"world": self.world, "owners": self.owners, "workers": self.worker_ranks, "P": self.P,
                "shard_off": self.shard_off, "shard_len": self.shard_len, "total": self.total,
                "staleness": self.S, "semantics": self.semantics, "round": self.round,
                "optimizer": self.cfg.to_dict(), "params": [(n, list(p.shape), o, k) for (n, p, o, k) in self._layout]}

    def save(self, prefix: str, blocking: bool = True):
        """Sharded checkpoint (collective: every rank calls at the same step). After a drain, each
        shard owner writes ``{prefix}.rank{r}.psd`` (atomic, CRC-checked: csrc/checkpoint.cpp) with
        its fp32 masters, optimizer state and step scalars, plus the shard versions and every
        worker's SSP clock; rank 0 writes ``{prefix}.manifest.json``. The device state is
        snapshotted (HBM->HBM) before any rank returns, so the engines' next applies cannot race
        the copy; with ``blocking=False`` the device->host copy and the file write run on a host
        thread while training continues. Returns that thread (or None).

        Reference: the periodic checkpoint thread (src/parameter_server_service.cpp:150-169) and
        ParameterServerCore::save_checkpoint (src/parameter_server.cpp:112-144), which kept no
        optimizer state, versions or worker iteration."""
        import json
        import threading

        self._quiesce()
        C = native()
        snap = []
        meta = {"step_idx": self.step_idx if self.is_worker else None, "shards": {}}
        for k in self.my_shards:
            ts = [self.master[k], self.dyn[k].t] + [d[k] for d in (self.state1, self.state2) if k in d]
            snap.extend(t.detach().clone() for t in ts)
            meta["shards"][str(k)] = {"version": int(self.engine.version(k)), "clocks": list(self.engine.clocks(k)),
                                      "n": len(ts)}
        # the workers' step (the owners that are not workers learn it from the store)
        steps = torch.tensor([self.step_idx if self.is_worker else 0], dtype=torch.int64)
        if self.world > 1 and dist.is_initialized():
            steps = steps.to(self.device) if dist.get_backend() == "nccl" else steps
            dist.all_reduce(steps, op=dist.ReduceOp.MAX)
        meta["step_idx"] = int(steps.item())
        if self.is_cuda:
            torch.cuda.synchronize(self.device)
        self._barrier(f"ckpt-snap-{self._ckpt_seq}")  # every owner's snapshot taken before anyone pushes
        self._ckpt_seq += 1
        man = {"format": "psd-async-v1", **self._layout_meta(), **meta, "rank": self.rank}
        man_s = json.dumps(man)
        path = f"{prefix}.rank{self.rank}.psd"

        def write():
            host = [t.cpu() for t in snap]
            C.save_native_ckpt(path, man_s, host)
            if self.rank == 0:
                m0 = {k: v for k, v in man.items() if k not in ("shards", "rank")}
                with open(f"{prefix}.manifest.json.tmp", "w") as f:
                    f.write(json.dumps(m0))
                os.replace(f"{prefix}.manifest.json.tmp", f"{prefix}.manifest.json")

        if blocking:
            write()
            return None
        th = threading.Thread(target=write, name="psd-async-ckpt", daemon=True)
        th.start()
        return th

    def load(self, prefix: str):
        """Resume from ``save(prefix)`` with the same layout (collective, before the first step):
        every owner restores its shards' masters, optimizer state and step scalars and re-publishes
        them as the saved shard versions with the saved SSP clocks; every worker continues at the
        saved step (its first pull waits on the restored clocks)."""
        import json

        man, ts = native().load_native_ckpt(f"{prefix}.rank{self.rank}.psd")
        m = json.loads(man)
        mine = self._layout_meta()
        for key in ("world", "owners", "workers", "shard_off", "shard_len", "total", "round"):
            if m[key] != mine[key]:
                raise ValueError(f"checkpoint {prefix}: {key} {m[key]} does not match this run's {mine[key]}")
        if m["optimizer"]["kind"] != self.cfg.kind:
            raise ValueError(f"checkpoint optimizer {m['optimizer']['kind']} != {self.cfg.kind}")
        self.engine.stop()
        i = 0
        for k in self.my_shards:
            sh = m["shards"][str(k)]
            self.master[k].copy_(ts[i])
            self.dyn[k].t.copy_(ts[i + 1])
            j = i + 2
            for d in (self.state1, self.state2):
                if k in d:
                    d[k].copy_(ts[j])
                    j += 1
            i += sh["n"]
            self.engine.publish_initial(k, sh["version"], sh["clocks"])
        self.step_idx = int(m["step_idx"])
        self._prefetched = None
        self.engine.start()
        if self.is_cuda:
            torch.cuda.synchronize(self.device)
        self._barrier(f"ckpt-load-{self._ckpt_seq}")
        self._ckpt_seq += 1
        if self.is_worker:  # working weights = the restored snapshot (forward hooks, eval before a step);
            # with MX pulls the e4m3 copy the fp8 convolutions read (install_fp8_weights) is pulled too
            self.pulled = self._pull_into(0, self.cb, None)
            self._to_work()
            if self.is_cuda:
                torch.cuda.synchronize(self.device)

    def _canon_index(self):
        """(flat offset, canonical offset, numel) per parameter, canonical = model.named_parameters
        order without padding (the layout CollectivePS.canonical_state uses too)."""
        where = {id(p): (o, k) for (_n, p, o, k) in self._layout}
        out, c = [], 0
        for _, p in self.model.named_parameters():
            if id(p) in where:
                o, k = where[id(p)]
                out.append((o, c, k))
                c += k
        return out, c

    def canonical_keys(self) -> list:
        return ["master", "state1", "state2"][: 1 + self.cfg.num_states]

    def dyn_template(self) -> torch.Tensor:
        """A tensor shaped like the step-scalar block (the receive buffer of a broadcast)."""
        return torch.zeros(8, dtype=torch.int32, device=self.device)

    def canonical_state(self, root: int) -> dict | None:
        """Collective: drain, then gather every shard's fp32 master + optimizer state onto rank
        ``root`` in the layout-independent canonical order (owners hold disjoint ranges: a sum
        reduce is the gather). Returns the tensors on ``root``, None elsewhere."""
        self._quiesce()
        idx, n = self._canon_index()
        out = {}
        for key, src in (("master", self.master), ("state1", self.state1), ("state2", self.state2)):
            if (key == "state1" and self.cfg.num_states < 1) or (key == "state2" and self.cfg.num_states < 2):
                continue
            full = torch.zeros(self.total, dtype=torch.float32, device=self.device)
            for k, t in src.items():
                full.narrow(0, self.shard_off[k], self.shard_len[k]).copy_(t)
            if self.world > 1 and dist.is_initialized():
                dist.reduce(full, root)
            if self.rank == root:
                canon = torch.empty(n, dtype=torch.float32, device=self.device)
                for o, c, k in idx:
                    canon.narrow(0, c, k).copy_(full.narrow(0, o, k))
                out[key] = canon
        # step scalars: every shard advanced in lock-step (one apply per round), take shard 0's
        d = self.dyn[0].t.detach().clone() if 0 in self.dyn else torch.zeros(8, dtype=torch.int32, device=self.device)
        if self.world > 1 and dist.is_initialized():
            if self.owners[0] != root:
                if self.rank == self.owners[0]:
                    dist.send(d, root)
                elif self.rank == root:
                    dist.recv(d, self.owners[0])
        if self.rank != root:
            return None
        out["dyn"] = d
        return out

    def load_canonical_state(self, sd: dict):
        """Inverse of ``canonical_state`` for this (possibly different) world and shard layout:
        every rank passes the full canonical tensors; owners keep their ranges and re-publish them
        (version 0 of this plane), workers take the weights."""
        idx, n = self._canon_index()
        full = {}
        for key in ("master", "state1", "state2"):
            if key not in sd:
                continue
            canon = sd[key].to(self.device)
            if canon.numel() != n:
                raise ValueError(f"canonical {key} has {canon.numel()} elements, model has {n}")
            f = torch.zeros(self.total, dtype=torch.float32, device=self.device)
            for o, c, k in idx:
                f.narrow(0, o, k).copy_(canon.narrow(0, c, k))
            full[key] = f
        self.engine.stop()
        for k in self.my_shards:
            for key, dst in (("master", self.master), ("state1", self.state1), ("state2", self.state2)):
                if key in full and k in dst:
                    dst[k].copy_(full[key].narrow(0, self.shard_off[k], self.shard_len[k]))
            if "dyn" in sd:
                self.dyn[k].t.copy_(sd["dyn"].to(self.dyn[k].t.device))
                # lr / grad scale of THIS plane's semantics and worker count
                self.dyn[k].set(lr=self.cfg.lr * self.hyper["lr_factor"], grad_scale=self.hyper["grad_scale"])
            self.engine.publish_initial(k)
        self.engine.start()
        self.params_flat.copy_(full["master"].to(self.param_dtype))
        for b in self.pbufs:
            if b is not self.pwork:
                b.copy_(self.params_flat)
        for q, sc, b in zip(self.q8s, self.sc8s, self.pbufs):
            # MX pulls: the e4m3 weights the fp8 convolutions read, and the working bf16 copy as a
            # pull would leave it (dequantised)
            native().quant_mx_(full["master"], q, sc)
            native().dequant_mx_(q, sc, b)
        self._to_work()
        self.step_idx = 0
        self._prefetched = None
        if self.is_cuda:
            torch.cuda.synchronize(self.device)
        self._barrier(f"canon-load-{self._ckpt_seq}")
        self._ckpt_seq += 1

    def export_reference(self, path: str, epoch: int, iteration: int = 0):
        """The reference's binary checkpoint layout (src/parameter_server.cpp:112-144: fp32 params by
        name) on rank 0, from the drained fp32 masters (collective)."""
        sd = self.canonical_state(root=0)
        if self.rank != 0:
            return
        names, shapes, vals = [], [], []
        idx, _ = self._canon_index()
        params = [(n, p) for n, p in self.model.named_parameters() if p.requires_grad]
        for (n, p), (_o, c, k) in zip(params, idx):
            names.append(n)
            shapes.append(list(p.shape))
            vals.append(sd["master"].narrow(0, c, k).view(p.shape).cpu())
        native().save_reference_ckpt(path, epoch, iteration, names, shapes, vals)

    def describe(self) -> str:
        return (f"AsyncPS(world={self.world}, shards={self.P} on ranks {self.owners}, workers={self.worker_ranks}, "
                f"SSP bound={self.S}, buckets={len(self.buckets)}, params={self.num_params() / 1e6:.2f}M, "
                f"memory={self.engine.memory_kind()}, xfer={self.xfer_mode})")
