"""Coordinator role: worker registry, heartbeat expiry, PS address / shard map, rendezvous kv.

Reference parity:
  coordinator_service_impl (src/coordinator_service.cpp:26-112) -> CoordinatorService
    RegisterWorker :39-61, Heartbeat :63-72 (unix-seconds timestamp), ListWorkers :74-88,
    GetParameterServerAddress :90-99
  cleanup_loop (:102-107, every 10 s remove_stale_workers(30)) -> ``_expiry_loop`` with the same
    defaults (sweep_s=10, expiry_s=30)
  run_coordinator_server (:114-126) -> ``serve``
The registry itself is the native C++ ``Registry`` (csrc/registry.cpp).

Fixed defects: D1/D2 -- the PS address is always returned as one consistent ``host:port`` in both
RegisterResponse and GetPSAddressResponse; D3 -- every join/leave/expiry bumps a membership epoch
that the PS and workers observe (RegisterResponse/HeartbeatResponse/ListWorkersResponse).
"""
from __future__ import annotations

import threading
import time

from .. import native
from ..rpc import schema, service
from ..utils.log import get_logger

pb = schema.coordinator
log = get_logger("coordinator")


def split_host_port(addr: str, default_port: int) -> tuple[str, int]:
    """``host:port`` / ``host`` / ``[v6]:port`` -> (host, port)."""
    addr = addr.strip()
    if addr.startswith("["):
        host, _, rest = addr[1:].partition("]")
        return host, int(rest[1:]) if rest.startswith(":") else default_port
    if addr.count(":") == 1:
        host, port = addr.split(":")
        return host, int(port)
    return addr, default_port


class CoordinatorService:
    def __init__(self, ps_host: str, ps_port: int, expiry_s: float = 30.0, sweep_s: float = 10.0,
                 shard_addresses: list[str] | None = None):
        C = native()
        self.reg = C.Registry(ps_host, ps_port)
        self.expiry_s, self.sweep_s = expiry_s, sweep_s
        self.shards = list(shard_addresses or [])
        for i, a in enumerate(self.shards):
            self.reg.set_shard(i, a, -1)
        self._stop = threading.Event()
        self._thr = threading.Thread(target=self._expiry_loop, name="coord-expiry", daemon=True)
        self._thr.start()

    # ---- reference RPCs
    def RegisterWorker(self, req, ctx):
        r = self.reg.register_worker(req.worker_id, req.address, req.port, req.hostname)
        log.info("worker %d %s (%s:%d) epoch=%d total=%d", req.worker_id, r.message, req.address or "localhost",
                 req.port, r.membership_epoch, r.total_workers)
        return pb.RegisterResponse(success=r.success, message=r.message, parameter_server_address=r.ps_address,
                                   total_workers=r.total_workers, membership_epoch=r.membership_epoch,
                                   ps_shard_addresses=self._shard_list())

    def Heartbeat(self, req, ctx):
        ok = self.reg.heartbeat(req.worker_id, int(req.status))
        return pb.HeartbeatResponse(success=ok, timestamp=int(time.time()),
                                    membership_epoch=self.reg.membership_epoch())

    def ListWorkers(self, req, ctx):
        ws = self.reg.list_workers()
        out = pb.ListWorkersResponse(total_workers=len(ws), membership_epoch=self.reg.membership_epoch())
        for w in ws:
            out.workers.add(worker_id=w.worker_id, address=w.address, port=w.port, hostname=w.hostname,
                            status=w.status)
        return out

    def GetParameterServerAddress(self, req, ctx):
        host, port = self.reg.ps_address()
        return pb.GetPSAddressResponse(address=f"{host}:{port}", port=port, shard_addresses=self._shard_list())

    # ---- additive RPCs
    def Deregister(self, req, ctx):
        ok = self.reg.deregister(req.worker_id)
        log.info("worker %d left (%s) epoch=%d", req.worker_id, "ok" if ok else "unknown", self.reg.membership_epoch())
        return pb.RegisterResponse(success=ok, message="deregistered" if ok else "unknown worker",
                                   total_workers=len(self.reg.live_ids()),
                                   membership_epoch=self.reg.membership_epoch())

    def KvSet(self, req, ctx):
        self.reg.kv_set(req.key, req.value)
        return pb.KvResponse(found=True)

    def KvGet(self, req, ctx):
        found, val = self.reg.kv_get(req.key, max(req.timeout_ms, 0) / 1000.0)
        return pb.KvResponse(found=found, value=val)

    # ---- internals
    def _shard_list(self):
        if self.shards:
            return self.shards
        host, port = self.reg.ps_address()
        return [f"{host}:{port}"]

    def _expiry_loop(self):
        while not self._stop.wait(self.sweep_s):
            gone = self.reg.remove_stale(self.expiry_s)
            if gone:
                log.warning("expired workers %s (no heartbeat for %.0f s); epoch=%d", gone, self.expiry_s,
                            self.reg.membership_epoch())

    def stop(self):
        self._stop.set()


STORE_KEY = "psd/store_port"


def host_store(svc: CoordinatorService, port: int = 0):
    """Host the rendezvous TCPStore of the elastic collective data plane (runtime/elastic.py) in
    the coordinator process, so it outlives any worker, and advertise its port in the kv."""
    import torch.distributed as dist

    store = dist.TCPStore("0.0.0.0", port, is_master=True, wait_for_workers=False)
    svc.reg.kv_set(STORE_KEY, str(store.port).encode())
    log.info("rendezvous store on port %d", store.port)
    return store


def serve(listen: str, ps_address: str, expiry_s: float = 30.0, sweep_s: float = 10.0,
          shard_addresses: list[str] | None = None, block: bool = True, store_port: int | None = 0):
    """``store_port``: port of the elastic rendezvous store (0: any free port; None: no store)."""
    host, port = split_host_port(ps_address, 50051)
    svc = CoordinatorService(host, port, expiry_s, sweep_s, shard_addresses)
    svc.store = host_store(svc, store_port) if store_port is not None else None
    server = service.make_server()
    service.add_service(server, pb, svc)
    bound = server.add_insecure_port(listen)
    if bound == 0:
        raise RuntimeError(f"coordinator: cannot bind {listen}")
    server.start()
    log.info("coordinator listening on %s (port %d); parameter server at %s:%d", listen, bound, host, port)
    if block:
        try:
            server.wait_for_termination()
        finally:
            svc.stop()
    return server, svc, bound
