"""Data-plane transports for the PS push/pull.

* ``RcclTransport`` -- the MI355X path: the native C++ ``RcclComm`` (csrc/comm.cpp) on explicit
  HIP streams. Collectives are enqueued on the stream that is current when called (the PS comm
  stream), never block the host and are legal inside hipGraph capture. The 128-byte RCCL unique
  id is bootstrapped through the rendezvous store (torch TCPStore or the coordinator's kv).
* ``TorchDistTransport`` -- ``torch.distributed`` process group: ``gloo`` for the CPU plumbing
  config / CI (BASELINE config 1) and the several-ranks-on-one-GPU rehearsal. Device tensors over
  an nccl process group always go through ``RcclTransport`` (one RCCL path, no torch-PG detour).
* ``LocalTransport`` -- world size 1: push/pull are identities (the colocated shard *is* the
  worker's buffer), so no copy is issued.

Reference parity: ``NCCLManager::allreduce_float`` (src/nccl_manager.cpp:102-121) was the only
collective; push = reduce-scatter and pull = all-gather replace the reference's
host-gradient -> gRPC -> host-average path (src/worker.cpp:254-272, src/parameter_server.cpp:38-63).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .. import native


class Transport:
    name = "base"
    world: int = 1
    rank: int = 0

    def reduce_scatter(self, inp: torch.Tensor, out: torch.Tensor) -> None:
        raise NotImplementedError

    def all_gather(self, inp: torch.Tensor, out: torch.Tensor) -> None:
        raise NotImplementedError

    def reduce(self, t: torch.Tensor, root: int) -> None:
        raise NotImplementedError

    def broadcast(self, t: torch.Tensor, root: int) -> None:
        raise NotImplementedError

    def send(self, t: torch.Tensor, peer: int) -> None:
        raise NotImplementedError

    def recv(self, t: torch.Tensor, peer: int) -> None:
        raise NotImplementedError

    def exchange(self, sends, recvs) -> None:
        """Grouped point-to-point: every (tensor, peer) in ``sends`` / ``recvs`` in one batch."""
        with self.group():
            for t, p in sends:
                self.send(t, p)
            for t, p in recvs:
                self.recv(t, p)

    def group(self):
        return _NullCtx()

    @property
    def capturable(self) -> bool:
        return False


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class LocalTransport(Transport):
    name = "local"

    def __init__(self):
        self.world, self.rank = 1, 0

    def reduce_scatter(self, inp, out):
        if out.data_ptr() != inp.data_ptr():
            out.copy_(inp)

    def all_gather(self, inp, out):
        if out.data_ptr() != inp.data_ptr():
            out.copy_(inp)

    def reduce(self, t, root):
        pass

    def broadcast(self, t, root):
        pass

    @property
    def capturable(self) -> bool:
        return True


class TorchDistTransport(Transport):
    """``torch.distributed`` collectives; synchronous w.r.t. the current stream."""

    name = "torch"

    def __init__(self, group=None):
        self.group_ = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = dist.get_backend(group)

    def _g(self, r):
        # group-local rank -> global rank
        return r if self.group_ is None else dist.get_global_rank(self.group_, r)

    def reduce_scatter(self, inp, out):
        if self.backend == "gloo":
            # gloo has no reduce_scatter_tensor: all-reduce then take our slice (CPU CI path)
            tmp = inp.clone()
            dist.all_reduce(tmp, group=self.group_)
            n = out.numel()
            out.copy_(tmp[self.rank * n:(self.rank + 1) * n])
        else:
            dist.reduce_scatter_tensor(out, inp, group=self.group_)

    def all_gather(self, inp, out):
        if self.backend == "gloo":
            chunks = list(out.chunk(self.world))
            src = inp.clone() if inp.data_ptr() == chunks[self.rank].data_ptr() else inp
            dist.all_gather(chunks, src, group=self.group_)
        else:
            dist.all_gather_into_tensor(out, inp, group=self.group_)

    def reduce(self, t, root):
        if self.backend == "gloo" and t.is_cuda:
            # gloo has no device reduce: all-reduce (only the root's copy is consumed). Rehearsal
            # path for several ranks sharing one GPU (bench.py --backend gloo), not a data plane.
            dist.all_reduce(t, group=self.group_)
            return
        dist.reduce(t, dst=self._g(root), group=self.group_)

    def broadcast(self, t, root):
        dist.broadcast(t, src=self._g(root), group=self.group_)

    def send(self, t, peer):
        dist.send(t, dst=self._g(peer), group=self.group_)

    def recv(self, t, peer):
        dist.recv(t, src=self._g(peer), group=self.group_)

    def exchange(self, sends, recvs):
        ops = [dist.P2POp(dist.isend, t, self._g(p), self.group_) for t, p in sends] + \
              [dist.P2POp(dist.irecv, t, self._g(p), self.group_) for t, p in recvs]
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()


class RcclTransport(Transport):
    """Native RCCL communicator driven from C++ on the current HIP stream."""

    name = "rccl"

    def __init__(self, rank: int, world: int, device: int, store=None, key: str = "psd/rccl_uid"):
        C = native()
        self.world, self.rank, self.device = world, rank, device
        if store is None:
            store = dist.distributed_c10d._get_default_store()
        if rank == 0:
            uid = C.RcclComm.unique_id()
            store.set(key, uid)
        else:
            store.wait([key])
            uid = store.get(key)
        self.comm = C.RcclComm(rank, world, bytes(uid), device)

    def reduce_scatter(self, inp, out):
        self.comm.reduce_scatter(inp, out, "sum", 0)

    def all_gather(self, inp, out):
        self.comm.all_gather(inp, out, 0)

    def reduce(self, t, root):
        self.comm.reduce(t, t, root, "sum", 0)

    def broadcast(self, t, root):
        self.comm.broadcast(t, root, 0)

    def send(self, t, peer):
        self.comm.send(t, peer, 0)

    def recv(self, t, peer):
        self.comm.recv(t, peer, 0)

    def group(self):
        C = native()

        class _G:
            def __enter__(self_):
                C.RcclComm.group_start()

            def __exit__(self_, *a):
                C.RcclComm.group_end()
                return False

        return _G()

    @property
    def capturable(self) -> bool:
        return True

    def abort(self):
        self.comm.abort()


def transport_kind(world: int, backend: str | None, kind: str = "auto", device_type: str = "cuda") -> str:
    """Which transport a process uses (pure policy, unit-tested): world 1 -> ``local``; device
    tensors over an nccl (= RCCL) process group -> the native ``rccl`` communicator on the PS comm
    stream (graph-capturable); gloo / CPU tensors -> ``torch``. ``kind`` (or ``PSD_TRANSPORT``)
    overrides the automatic choice."""
    kind = os.environ.get("PSD_TRANSPORT", kind)
    if world <= 1:
        if kind not in ("auto", "local"):
            return kind  # tests: drive RCCL / torch collectives even at world size 1
        return "local"
    if kind == "local":
        raise ValueError("local transport requires world size 1")
    if kind != "auto":
        return kind
    if backend == "nccl" and device_type == "cuda":
        return "rccl"
    return "torch"


def make_transport(kind: str = "auto", device: torch.device | None = None) -> Transport:
    """The transport for the current process group and device (see ``transport_kind``)."""
    init = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size() if init else 1
    backend = dist.get_backend() if init else None
    dtype_ = device.type if device is not None else ("cuda" if torch.cuda.is_available() else "cpu")
    k = transport_kind(world, backend, kind, dtype_)
    if k == "local":
        return LocalTransport()
    if k == "rccl":
        dev = device.index if device is not None and device.index is not None else torch.cuda.current_device()
        if not init:
            return RcclTransport(0, 1, dev, store=dist.HashStore())
        return RcclTransport(dist.get_rank(), world, dev)
    return TorchDistTransport()
