"""Worker training step over the collective PS data plane, optionally captured as hipGraphs.

One step = begin (zero grads) -> forward -> backward (per-bucket push/apply/pull launched from
grad hooks onto the comm stream) -> join. With ``use_graph`` the whole step -- forward, backward,
every RCCL collective and every fused-apply kernel -- is captured once per staleness phase
(``t mod (S+1)`` selects the gradient slot, so S+1 graphs) and replayed; the host then only does
the version / staleness bookkeeping. This replaces a tracing compiler: the step's ~500 kernel
launches become one graph launch.

Reference parity: ``Worker::run_iteration`` (src/worker.cpp:331-406) is a pull -> compute ->
push -> poll loop with 500 ms sleeps; here pull/push are collectives inside the step and there is
no polling.
"""
from __future__ import annotations

import os
import time

import torch

from ..parallel.collective_ps import CollectivePS


class Trainer:
    def __init__(self, model, loss_fn, ps: CollectivePS, batch, use_graph: bool = False, graph_warmup: int = 3,
                 tracer=None, checkpoint_prefix: str | None = None, checkpoint_every: int = 0):
        self.model = model
        self.loss_fn = loss_fn
        self.ps = ps
        self.x, self.y = batch
        self.use_graph = use_graph and ps.is_cuda and ps.t.capturable
        self.graph_warmup = graph_warmup
        self.graphs: dict[int, torch.cuda.CUDAGraph] = {}
        self.static_loss = None
        self.step_count = 0
        self.graph_error = None
        self.tracer = tracer
        # periodic sharded PS checkpoint (reference: checkpoint thread every ckpt_interval,
        # src/parameter_main.cpp): device->host on a side stream, file write on a host thread
        self.checkpoint_prefix = checkpoint_prefix
        self.checkpoint_every = int(checkpoint_every)
        # PSD_STEP_LOG=1: (begin, forward, backward, finish) host seconds of every eager step
        self.host_phases = [] if os.environ.get("PSD_STEP_LOG", "0") == "1" else None
        self.boundary_evs = []  # (previous step's end, this step's forward start) events, with host_phases
        self._ckpt_thread = None
        if tracer is not None:
            self.use_graph = False  # per-phase timing needs eager steps
            ps.tracer = tracer

    # eager step ---------------------------------------------------------------
    def _body(self):
        if not self.ps.is_worker:  # disjoint placement: PS-only rank
            self.ps.begin_step()
            self.ps.finish_step()
            return torch.zeros((), device=self.ps.device)
        tr = self.tracer
        if tr is None and self.host_phases is not None:  # PSD_STEP_LOG=1: host time per phase (diagnosis)
            t0 = time.perf_counter()
            # drained: the compute stream had already run out of queued work when the host got here
            # (the GPU waits for the host at this step boundary)
            drained = bool(self.ps.is_cuda and torch.cuda.current_stream(self.ps.device).query())
            self.ps.begin_step()
            t1 = time.perf_counter()
            # ... or had finished the previous step's work by the time begin_step (its pull wait) let
            # the host go on (the event was recorded after the previous step's last kernel)
            ev = getattr(self, "_end_ev", None)
            drained_after = bool(ev is not None and ev.query())
            if self.ps.is_cuda:  # GPU time of the step boundary: previous step's end -> this forward's start
                self._fwd_ev = torch.cuda.Event(enable_timing=True)
                self._fwd_ev.record(torch.cuda.current_stream(self.ps.device))
            out = self.model(self.x)
            loss = self.loss_fn(out, self.y)
            t2 = time.perf_counter()
            loss.backward()
            t3 = time.perf_counter()
            self.ps.finish_step()
            t4 = time.perf_counter()
            if self.ps.is_cuda:
                self._end_ev = torch.cuda.Event(enable_timing=True)
                self._end_ev.record(torch.cuda.current_stream(self.ps.device))
                self.boundary_evs.append((ev, self._fwd_ev))
            self.host_phases.append((t1 - t0, t2 - t1, t3 - t2, t4 - t3, drained, drained_after))
            return loss
        if tr is None:
            self.ps.begin_step()
            out = self.model(self.x)
            loss = self.loss_fn(out, self.y)
            loss.backward()
            self.ps.finish_step()
            return loss
        with tr.phase("begin"):
            self.ps.begin_step()
        with tr.phase("forward"):
            out = self.model(self.x)
            loss = self.loss_fn(out, self.y)
        with tr.phase("backward"):
            loss.backward()
        with tr.phase("finish"):
            self.ps.finish_step()
        tr.end_step(self.step_count, version=self.ps.step_idx)
        return loss

    def eager_step(self):
        loss = self._body()
        self.step_count += 1
        return loss

    # graph capture ------------------------------------------------------------
    def _capture(self, phase: int):
        ps = self.ps
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=ps.device)
        s.wait_stream(torch.cuda.current_stream(ps.device))
        saved_idx = ps.step_idx
        # the captured body must see the slot indices of this phase (and be past the first S
        # apply-free steps): same residue mod S+1, >= S
        ps.step_idx = phase + (ps.S + 1)
        try:
            with torch.cuda.graph(g, stream=s, pool=self._pool):
                loss = self._body_captured()
        finally:
            ps.step_idx = saved_idx
        torch.cuda.current_stream(ps.device).wait_stream(s)
        return g, loss

    def _body_captured(self):
        # identical device work to _body, but the host bookkeeping (tracker, step counter) is done
        # per replay by `step()`, not at capture time
        ps = self.ps
        if not ps.is_worker:
            ps.begin_step(track=False)
            ps.finish_step(track=False)
            return torch.zeros((), device=ps.device)
        ps.begin_step(track=False)
        out = self.model(self.x)
        loss = self.loss_fn(out, self.y)
        loss.backward()
        ps.finish_step(track=False)
        return loss

    def step(self):
        """One training step (eager until the graphs are built, then graph replay)."""
        loss = self._step()
        if self.checkpoint_every > 0 and self.checkpoint_prefix and self.step_count % self.checkpoint_every == 0:
            self.checkpoint()
        return loss

    def checkpoint(self, blocking: bool = False):
        """Snapshot the PS shards to ``checkpoint_prefix`` (waits for the previous write first)."""
        if self._ckpt_thread is not None:
            self._ckpt_thread.join()
        self._ckpt_thread = self.ps.save(self.checkpoint_prefix, blocking=blocking)

    def wait_checkpoint(self):
        if self._ckpt_thread is not None:
            self._ckpt_thread.join()
            self._ckpt_thread = None

    def _step(self):
        ps = self.ps
        if not self.use_graph:
            return self.eager_step()
        phases = ps.S + 1
        # eager warmup: MIOpen/allocator/autotune must settle before capture; the first S steps
        # (no apply yet) are also eager
        if self.step_count < max(self.graph_warmup, ps.S) or self.graph_error is not None:
            return self.eager_step()
        key = ps.step_idx % phases
        if key not in self.graphs:
            try:
                if not hasattr(self, "_pool"):
                    self._pool = torch.cuda.graph_pool_handle()
                torch.cuda.synchronize(ps.device)
                g, loss = self._capture(key)
                self.graphs[key] = (g, loss)
            except Exception as e:  # capture unsupported by some library kernel: stay eager
                self.graph_error = repr(e)
                torch.cuda.synchronize(ps.device)
                return self.eager_step()
        g, loss = self.graphs[key]
        ps.account_begin()
        g.replay()
        ps.account_finish()
        self.step_count += 1
        return loss

    def run(self, steps: int) -> float:
        t0 = time.perf_counter()
        for _ in range(steps):
            self.step()
        self.wait_checkpoint()
        if self.ps.is_cuda:
            torch.cuda.synchronize(self.ps.device)
        return time.perf_counter() - t0
