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

  "round" (default): K-batch asynchronous SGD with K = W (min(W, 16)). Each shard takes the pushes
          in arrival order, from whichever workers, and every K of them make ONE optimizer step on
          their average with the synchronous hyperparameters (the K inbox slots are summed inside
          the fused apply kernel). A worker's clock advances when the round holding its push has
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
import uuid
from dataclasses import dataclass, field

import torch
import torch.distributed as dist
import torch.nn as nn

from .. import native
from ..ops.optim import OptimConfig, OptimDyn
from .collective_ps import ALIGN, _flat_view, _round, zero_grads_, zero_plan

_INSTANCE = [0]


class _NoTransport:
    name = "ipc"
    capturable = False


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
                 semantics: str = "round"):
        """``semantics``: "round" (K-batch async, default) or "push" (apply-on-arrival with the
        per-push hyperparameters of csrc/async_hyper.h); see the module docstring."""
        self.model = model
        self.cfg = optim
        st, self.rank, self.world = _store_and_group()
        self.store = store or st
        self.t = _NoTransport()
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
        self.param_dtype = param_dtype
        self.step_idx = 0
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
        # push buckets: consecutive parameter ranges of ~bucket_mb
        elem = torch.finfo(param_dtype).bits // 8
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
        self.buckets[-1].hi = total  # the tail padding travels with the last bucket

        dev = self.device
        init = torch.zeros(total, dtype=torch.float32, device=dev)
        for n, p, o, k in layout:
            _flat_view(init, o, p).copy_(p.detach().float())
        # working weights: with S >= 1 two buffers alternate per step, so the pull of step t+1 (DMA
        # from the owners' publish buffers) runs on a side stream while step t computes
        self.prefetch = self.S >= 1
        self.pbufs = [init.to(param_dtype)]
        if self.prefetch:
            self.pbufs.append(self.pbufs[0].clone())
        self.cb = 0
        self.grads = [torch.zeros(total, dtype=param_dtype, device=dev) for _ in range(2)]
        self.gb = 0
        f32 = dict(dtype=torch.float32, device=dev)
        # per-push hyperparameters (module docstring)
        if semantics not in ("round", "push"):
            raise ValueError(f"semantics must be 'round' or 'push', got {semantics!r}")
        self.semantics = semantics
        self.round = min(self.W, 16) if semantics == "round" else 1
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
        self._p2b = {}
        for b in self.buckets:
            for _, p, _o, _n in b.params:
                self._p2b[id(p)] = b
        self._pviews = [[_flat_view(b, o, p) for (_n, p, o, _k) in layout] for b in self.pbufs]
        for (n, p, o, k), v in zip(layout, self._pviews[0]):
            p.data = v
        self._set_grad_views()
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for _, p, _o, _n in layout]
        self._next = 0
        if self.is_cuda:
            self.comm_stream = torch.cuda.Stream(device=dev)
            self.pull_stream = torch.cuda.Stream(device=dev)
            self.push_done = [None, None]
            self.step_done = [None, None]  # end of a step's work on the compute stream, per buffer
            self.pull_done = [None, None]
        self._prefetched = None  # (step, pulled versions) of the pull issued ahead

        # ---- native engine: control block (rank 0 creates), memory exchange, initial publish
        _INSTANCE[0] += 1
        key = f"psd/async/{_INSTANCE[0]}"
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
                                    torch.finfo(param_dtype).bits // 8)
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
        if log:
            self.engine.enable_log(True)
        self._barrier("init")
        self.selftest()
        self.engine.start()

    def selftest(self):
        """Collective start-up check of the peer-memory paths on this node (before any training):
        every worker DMA-writes a known pattern into its inbox on every shard owner, and every
        owner verifies what landed; every worker pulls the version-0 snapshots and compares them
        with its own initial weights. Raises on any mismatch on any rank (so a caller can fall
        back to the collective plane instead of training on a broken path)."""
        dev = self.device
        ok, why = True, ""
        if self.is_worker:
            pat = (torch.arange(self.total, device=dev) % 251 + (self.rank + 1)).to(self.param_dtype)
            self.engine.push(0, pat, 0, self.total, self._stream_ptr())
            got = torch.empty_like(self.params_flat)
            self.engine.pull(0, got, self._stream_ptr())
            if self.is_cuda:
                torch.cuda.synchronize(dev)
            if not torch.equal(got, self.params_flat):
                ok, why = False, f"rank {self.rank}: pulled snapshot != initial weights"
        if os.environ.get("PSD_ASYNC_SELFTEST_FAIL_RANK") == str(self.rank):  # fault injection (tests)
            ok, why = False, f"rank {self.rank}: injected self-test failure"
        self._barrier("selftest-push")
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
        self._agree("selftest", "" if ok else why)
        self.selftest_ok = True

    def _agree(self, tag: str, err: str):
        """Collective status exchange through the store: every rank raises if any rank failed."""
        self.store.set(f"{self._key}/{tag}/{self.rank}", err or "ok")
        errs = []
        for r in range(self.world):
            self.store.wait([f"{self._key}/{tag}/{r}"])
            v = self.store.get(f"{self._key}/{tag}/{r}").decode()
            if v != "ok":
                errs.append(v)
        if errs:
            raise RuntimeError(f"AsyncPS {tag} failed: " + "; ".join(errs))

    # ------------------------------------------------------------------ helpers
    @property
    def params_flat(self) -> torch.Tensor:
        """The working weights of the current step."""
        return self.pbufs[self.cb]

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
        g = self.grads[self.gb]
        self._grad_views = {}
        for n, p, o, k in self._layout:
            v = _flat_view(g, o, p)
            self._grad_views[id(p)] = v
            p.grad = None if id(p) in self._direct else v

    def _sink(self, p):
        if id(p) not in self._direct:
            return None
        v = self._grad_views[id(p)]
        return v.view(v.shape)

    def memory_bytes(self) -> dict:
        eb = lambda t: t.numel() * t.element_size()  # noqa: E731
        return {"params": sum(eb(b) for b in self.pbufs), "grads": 2 * eb(self.grads[0]),
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
            for (_n, p, _o, _k), v in zip(self._layout, self._pviews[self.cb]):
                p.data = v
            if self._prefetched is not None and self._prefetched[0] == t:
                self.pulled = self._prefetched[1]
                if self.is_cuda:
                    torch.cuda.current_stream(self.device).wait_event(self.pull_done[self.cb])
                return
        self.pulled = list(self.engine.pull(t, self.params_flat, self._stream_ptr()))

    def _prefetch_pull(self, t: int):
        """Issue the pull of step t (the next one) now: the SSP wait happens on the host here, the
        DMA on the pull stream, after the step that last used that buffer (t-2) is done with it."""
        nb = t % 2
        if self.is_cuda:
            if self.step_done[nb] is not None:
                self.pull_stream.wait_event(self.step_done[nb])
            pulled = self.engine.pull(t, self.pbufs[nb], self.pull_stream.cuda_stream)
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
            self.comm_stream.wait_event(ev)
            self.engine.push(self.step_idx, g, b.lo, b.hi, self.comm_stream.cuda_stream)
        else:
            self.engine.push(self.step_idx, g, b.lo, b.hi, 0)

    def finish_step(self, track: bool = True):
        if not self.is_worker:
            return
        while self._next < len(self.buckets):
            self._push(self.buckets[self._next])
            self._next += 1
        if self.is_cuda:
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
                         ("pull", lambda: self.engine.pull(0, tmp, st.cuda_stream))):
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

    def close(self):
        """Collective: stop the engine, unmap the peers' memory, free this rank's (all ranks call)."""
        if self.closed:
            return
        self.engine.stop()
        self._barrier("stop")
        self.engine.close_peers()
        self._barrier("unmapped")
        hist, vers, log = self.staleness_histogram(), self.versions(), self.apply_log()
        self._final = (hist, vers, log)
        self.engine.free_local()
        self.engine = None
        for h in self._hooks:
            h.remove()
        for m in self.model.modules():
            if getattr(m, "_psd_grad_sink", None) == self._sink:
                del m._psd_grad_sink
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

    def describe(self) -> str:
        return (f"AsyncPS(world={self.world}, shards={self.P} on ranks {self.owners}, workers={self.worker_ranks}, "
                f"SSP bound={self.S}, buckets={len(self.buckets)}, params={self.num_params() / 1e6:.2f}M, "
                f"memory={self.engine.memory_kind()})")
