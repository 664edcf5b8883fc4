"""Worker role over the gRPC data plane (the reference's architecture, with real gradients).

Reference parity (src/worker.cpp, include/worker.h:21-69):
  discover_parameter_server :141-157 / register_with_coordinator :159-186 -> ``initialize``
  query_with_retry :129-139 (5 tries, 100*2^k ms)                        -> ``_retry``
  heartbeat_loop :231-238 (every 5 s, IDLE/TRAINING status)              -> ``_heartbeat_loop``
  pull_parameters :240-252 / push_gradients :254-272 / check_sync_ready :274-287
  run_iteration :331-406 (pull -> compute -> push -> poll)               -> ``run_iteration``
  compute_gradients :316-329 (constant 0.01 stub)                        -> a real forward/backward
  load_checkpoint_from_server :289-314                                   -> returns (epoch, iteration)
  reconnect :124-127 (dead code in the reference)                        -> ``reconnect`` (used on
                                                                            heartbeat rejection)
Differences: one persistent channel per peer; the sync wait is a server-side long-poll
(``PullRequest.wait_ms``) instead of 200x50 ms client polling with 500 ms retry sleeps; the
coordinator returns a consistent host:port (D1); initial parameters come from worker 0's seeded
model through ``InitParameters`` (the reference let the first averaged gradient *become* the
parameters, src/parameter_server.cpp:78-81 -- kept only in ``reference_compat`` mode).

Fault injection (env): PSD_FAULT="stop_heartbeat_after=n,exit_after_push=k,push_delay_ms=ms"
(utils/config.py FAULTS).
"""
from __future__ import annotations

import os
import socket
import threading
import time

import torch

from .. import models
from ..rpc import schema, service
from ..utils.config import fault
from ..utils.log import get_logger

cpb = schema.coordinator
ppb = schema.parameter_server


class Worker:
    def __init__(self, coordinator: str, worker_id: int, worker_addr: str = "", worker_port: int = 0,
                 model: str = "mlp", batch: int = 64, device: str = "cpu", heartbeat_s: float = 5.0,
                 rpc_timeout: float = 60.0, sync_wait_s: float = 30.0, seed: int = 0, bf16_wire: bool = False,
                 raw_wire: bool = True, mode: str = "sync"):
        self.log = get_logger(f"worker{worker_id}")
        self.coordinator_addr = coordinator
        self.worker_id = int(worker_id)
        self.mode = mode
        self.worker_addr, self.worker_port = worker_addr, int(worker_port)
        self.heartbeat_s = heartbeat_s
        self.rpc_timeout = rpc_timeout
        self.sync_wait_ms = int(sync_wait_s * 1000)
        self.bf16_wire, self.raw_wire = bf16_wire, raw_wire
        self.device = torch.device(device)
        torch.manual_seed(seed)  # identical init on every worker (only worker 0's is used)
        dtype = torch.float32 if self.device.type == "cpu" else torch.bfloat16
        self.spec = models.build(model, self.device, dtype)
        self.model = self.spec.model
        if dtype != torch.float32:  # parameters only: fused-BN running stats stay fp32
            for prm in self.model.parameters():
                prm.data = prm.data.to(dtype)
        self.batch = self.spec.make_batch(batch, self.device, seed=1000 + self.worker_id)
        self.status = cpb.IDLE
        self._status_lock = threading.Lock()
        self._initialized = threading.Event()
        self._stop = threading.Event()
        self.coord = service.Stub(coordinator, cpb, timeout=rpc_timeout)
        self.ps = None
        self.ps_address = None
        self.membership_epoch = 0
        self.version = -1
        self.pushes = 0
        self._cached = None  # params fetched by the sync wait, reused by the next iteration
        self.hb = threading.Thread(target=self._heartbeat_loop, name=f"hb{worker_id}", daemon=True)
        self.hb.start()

    # ------------------------------------------------------------------ control plane
    def _retry(self, fn, attempts: int = 5, base_ms: int = 100):
        err = None
        for k in range(attempts):
            try:
                return fn()
            except Exception as e:  # noqa: BLE001 - retried like the reference's query_with_retry
                err = e
                time.sleep(base_ms * (2 ** k) / 1000.0)
        raise RuntimeError(f"worker {self.worker_id}: RPC failed after {attempts} attempts: {err}")

    def initialize(self):
        r = self._retry(lambda: self.coord.GetParameterServerAddress(cpb.GetPSAddressRequest()))
        self.ps_address = r.address if ":" in r.address else f"{r.address}:{r.port}"
        self._register()
        self.ps = service.Stub(self.ps_address, ppb, timeout=self.rpc_timeout)
        # seed the PS with this worker's initial parameters (first caller wins)
        init = ppb.GradientUpdate(worker_id=self.worker_id, iteration=-1)
        init.gradients.extend(service.tensors_to_protos(self._named_params(), raw=True))
        ir = self._retry(lambda: self.ps.InitParameters(init))
        # elastic join: start at the oldest iteration the PS has not aggregated yet
        self.start_iteration = 0
        if not ir.success:
            st = self.stats()
            cur = int(st.current_iteration)
            if st.version > 0:
                ss = self.ps.CheckSyncStatus(ppb.SyncStatusRequest(iteration=cur))
                self.start_iteration = cur + 1 if ss.ready else cur
        self.log.info("PS at %s (%s); membership epoch %d; starting at iteration %d", self.ps_address, ir.message,
                      self.membership_epoch, self.start_iteration)
        self._initialized.set()
        return True

    def _register(self):
        info = cpb.WorkerInfo(worker_id=self.worker_id, address=self.worker_addr or "localhost",
                              port=self.worker_port, hostname=f"worker-{self.worker_id}@{socket.gethostname()}")
        r = self._retry(lambda: self.coord.RegisterWorker(info))
        self.membership_epoch = r.membership_epoch
        return r

    def reconnect(self):
        """Re-register after the coordinator expired us (dead code in the reference)."""
        self.log.warning("re-registering with the coordinator")
        self._register()

    def set_status(self, s):
        with self._status_lock:
            self.status = s

    def _heartbeat_loop(self):
        n = 0
        stop_after = fault("stop_heartbeat_after")
        while not self._stop.wait(self.heartbeat_s):
            if not self._initialized.is_set():
                continue
            if 0 <= stop_after <= n:
                continue  # fault injection: go silent, the coordinator will expire us
            n += 1
            with self._status_lock:
                st = self.status
            try:
                r = self.coord.Heartbeat(cpb.HeartbeatRequest(worker_id=self.worker_id, status=st), timeout=5.0,
                                         wait_for_ready=False)
                self.membership_epoch = r.membership_epoch
                if not r.success:
                    self.reconnect()
            except Exception as e:  # noqa: BLE001
                self.log.debug("heartbeat failed: %s", e)

    # ------------------------------------------------------------------ data plane (gRPC)
    def _named_params(self):
        return [(n, p.detach()) for n, p in self.model.named_parameters()]

    def _load(self, update):
        params = dict(service.protos_to_tensors(update.parameters))
        with torch.no_grad():
            for n, p in self.model.named_parameters():
                if n in params:
                    p.copy_(params[n].to(p.dtype).reshape(p.shape))
        self.version = update.version

    def pull(self, iteration: int, wait: bool = False):
        req = ppb.PullRequest(worker_id=self.worker_id, iteration=iteration, wait_ms=self.sync_wait_ms if wait else 0,
                              accept_raw=self.raw_wire)
        return self._retry(lambda: self.ps.ServeParameters(req))

    def compute_gradients(self):
        for p in self.model.parameters():
            p.grad = None
        x, y = self.batch
        loss = self.spec.loss(self.model(x), y)
        loss.backward()
        return float(loss.detach().float()), [(n, p.grad.detach()) for n, p in self.model.named_parameters()]

    def push(self, iteration: int, grads):
        delay = fault("push_delay_ms")
        if delay:
            time.sleep(delay / 1000.0)
        up = ppb.GradientUpdate(worker_id=self.worker_id, iteration=iteration, pulled_version=max(self.version, 0))
        up.gradients.extend(service.tensors_to_protos(grads, raw=self.raw_wire, bf16=self.bf16_wire))
        r = self._retry(lambda: self.ps.ReceiveGradients(up))
        self.pushes += 1
        k = fault("exit_after_push")
        if 0 < k <= self.pushes:
            self.log.error("fault injection: exiting after push %d", self.pushes)
            os._exit(3)
        return r

    def run_iteration(self, iteration: int):
        """One pull -> compute -> push step. Returns (done, loss, push_response)."""
        self.set_status(cpb.TRAINING)
        try:
            if self.mode == "async":  # SSP: the PS holds the pull while we lead the slowest by > S
                upd = self.pull(iteration, wait=True)
            elif self._cached is not None:
                upd, self._cached = self._cached, None
            else:
                upd = self.pull(iteration - 1, wait=False)
            if not upd.parameters:
                raise RuntimeError("parameter server returned no parameters")
            self._load(upd)
            loss, grads = self.compute_gradients()
            r = self.push(iteration, grads)
            if not r.success:
                self.log.warning("iter %d push rejected: %s", iteration, r.message)
                return False, loss, r
            done = r.aggregation_complete
            if not done:  # sync barrier: long-poll until every live worker pushed this iteration
                upd = self.pull(iteration, wait=True)
                done = upd.ready
                self._cached = upd if done else None
            return done, loss, r
        finally:
            self.set_status(cpb.IDLE)

    def load_checkpoint_from_server(self, path: str):
        self.set_status(cpb.CHECKPOINTING)
        try:
            r = self._retry(lambda: self.ps.LoadCheckpoint(ppb.LoadCheckpointRequest(path=path, accept_raw=True)))
            if not r.success:
                raise RuntimeError(f"LoadCheckpoint({path}) failed: {r.message}")
            return r.epoch, r.iteration
        finally:
            self.set_status(cpb.IDLE)

    def stats(self):
        return self.ps.GetStats(ppb.SyncStatusRequest())

    def shutdown(self, deregister: bool = True):
        self._stop.set()
        if deregister:
            try:
                self.coord.Deregister(cpb.WorkerInfo(worker_id=self.worker_id), timeout=5.0, wait_for_ready=False)
            except Exception:  # noqa: BLE001
                pass
