"""grpcio plumbing for the two services: generic handlers, persistent client stubs, tensor codec.

Fixes of the reference's transport: one persistent channel per peer (the
reference opened a new channel for *every* RPC, src/worker.cpp:143-275), deadlines on every call,
raised message limits (the reference's 4 MiB default caps a push at ~1M floats), and a bulk
``raw`` bytes payload per tensor instead of element-by-element ``add_data`` loops.
"""
from __future__ import annotations

from concurrent import futures

import grpc
import numpy as np
import torch

from . import schema

MAX_MSG = 1 << 30
CHANNEL_OPTS = [("grpc.max_send_message_length", MAX_MSG), ("grpc.max_receive_message_length", MAX_MSG),
                ("grpc.keepalive_time_ms", 30000)]

DTYPE_F32, DTYPE_F64, DTYPE_BF16 = 0, 1, 2


def make_server(max_workers: int = 32) -> grpc.Server:
    return grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers), options=CHANNEL_OPTS)


def add_service(server: grpc.Server, ns, impl) -> None:
    """Register ``impl.<Method>(request, context)`` for every method of namespace ``ns``."""
    handlers = {}
    for meth in ns.methods:
        fn = getattr(impl, meth)
        handlers[meth] = grpc.unary_unary_rpc_method_handler(
            fn, request_deserializer=ns.request_type(meth).FromString,
            response_serializer=ns.response_type(meth).SerializeToString)
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(ns.service_name, handlers),))


class Stub:
    """Persistent client for one service: ``stub.Method(request, timeout=...)``."""

    def __init__(self, address: str, ns, timeout: float = 30.0):
        self.address = address
        self.ns = ns
        self.timeout = timeout
        self.channel = grpc.insecure_channel(address, options=CHANNEL_OPTS)
        for meth in ns.methods:
            call = self.channel.unary_unary(f"/{ns.service_name}/{meth}",
                                            request_serializer=ns.request_type(meth).SerializeToString,
                                            response_deserializer=ns.response_type(meth).FromString)
            setattr(self, meth, self._wrap(call))

    def _wrap(self, call):
        def f(req, timeout=None, wait_for_ready=True):
            return call(req, timeout=timeout or self.timeout, wait_for_ready=wait_for_ready)

        return f

    def close(self):
        self.channel.close()


# --------------------------------------------------------------------------------- tensor codec
def tensor_to_proto(name: str, t: torch.Tensor, raw: bool = True, bf16: bool = False):
    """Encode a tensor. ``raw`` (default) uses the bulk bytes field; ``raw=False`` produces the
    reference's ``repeated float data`` encoding (what a reference C++ peer reads)."""
    msg = schema.parameter_server.Tensor(name=name, shape=list(t.shape))
    t = t.detach()
    if raw:
        if bf16:
            msg.dtype = DTYPE_BF16
            msg.raw = t.to(torch.bfloat16).contiguous().cpu().view(torch.int16).numpy().tobytes()
        else:
            msg.dtype = DTYPE_F32
            msg.raw = t.to(torch.float32).contiguous().cpu().numpy().tobytes()
    else:
        msg.dtype = DTYPE_F32
        msg.data.extend(t.to(torch.float32).reshape(-1).cpu().tolist())
    return msg


def proto_to_tensor(msg) -> torch.Tensor:
    shape = tuple(msg.shape)
    if msg.raw:
        if msg.dtype == DTYPE_BF16:
            a = np.frombuffer(msg.raw, dtype=np.int16).copy()
            return torch.from_numpy(a).view(torch.bfloat16).float().reshape(shape)
        if msg.dtype == DTYPE_F64:
            return torch.from_numpy(np.frombuffer(msg.raw, dtype=np.float64).copy()).float().reshape(shape)
        return torch.from_numpy(np.frombuffer(msg.raw, dtype=np.float32).copy()).reshape(shape)
    a = np.asarray(msg.data, dtype=np.float32)
    return torch.from_numpy(a).reshape(shape) if a.size else torch.zeros(shape)


def tensors_to_protos(named, raw=True, bf16=False):
    return [tensor_to_proto(n, t, raw, bf16) for n, t in named]


def protos_to_tensors(msgs):
    return [(m.name, proto_to_tensor(m)) for m in msgs]
