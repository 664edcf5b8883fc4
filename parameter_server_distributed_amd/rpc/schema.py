"""Wire schema of the control plane: ``proto/psd_coordinator.proto`` and
``proto/psd_parameter_server.proto`` are the source of truth, parsed at import time by
``rpc/protoparse.py`` into descriptors and message classes (no protoc in this image).

The two services keep the reference's package names, service names, method names, message names,
field numbers and field types (the reference's proto/coordinator.proto, proto/parameter_server.proto),
so a reference C++ client/server can talk to ours. Everything we add is *additive*: new fields carry
new numbers and new methods new names, which proto3 peers ignore.

Additions (all optional on the wire):
  coordinator.WorkerInfo            5 status, 6 gpu
  coordinator.RegisterResponse      5 membership_epoch, 6 ps_shard_addresses
  coordinator.HeartbeatResponse     3 membership_epoch
  coordinator.ListWorkersResponse   3 membership_epoch
  coordinator.GetPSAddressResponse  3 shard_addresses
  coordinator.Coordinator           Deregister, KvSet, KvGet (RCCL unique-id bootstrap)
  parameter_server.Tensor           5 raw (bulk little-endian payload; dtype 2 = bfloat16)
  parameter_server.GradientUpdate   4 pulled_version
  parameter_server.PushResponse     7 version, 8 staleness
  parameter_server.PullRequest      3 wait_ms, 4 accept_raw (reply with bulk bytes, not repeated float)
  parameter_server.LoadCheckpointRequest 2 accept_raw; LoadCheckpointResponse 5 iteration
  parameter_server.ParameterUpdate  4 version
  parameter_server.ParameterServer  InitParameters, GetStats, SetTotalWorkers

``emit_proto(dir)`` copies the .proto files for non-Python peers.
"""
from __future__ import annotations

import os

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from . import protoparse

PROTO_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "proto")
PROTO_FILES = {"coordinator": "psd_coordinator.proto", "parameter_server": "psd_parameter_server.proto"}

_POOL = descriptor_pool.DescriptorPool()
FILES: dict[str, descriptor_pb2.FileDescriptorProto] = {}
for _pkg, _fname in PROTO_FILES.items():
    _fd = protoparse.parse_file(os.path.join(PROTO_DIR, _fname))
    if _fd.package != _pkg:
        raise ValueError(f"{_fname}: package {_fd.package!r}, expected {_pkg!r}")
    FILES[_pkg] = _fd
    _POOL.Add(_fd)


class _Namespace:
    def __init__(self, fd: descriptor_pb2.FileDescriptorProto):
        self.package = fd.package
        svc = fd.service[0]
        self.service_name = f"{fd.package}.{svc.name}"
        self.methods = {m.name: (m.input_type.split(".")[-1], m.output_type.split(".")[-1]) for m in svc.method}
        for m in fd.message_type:
            desc = _POOL.FindMessageTypeByName(f"{fd.package}.{m.name}")
            setattr(self, m.name, message_factory.GetMessageClass(desc))
        for e in fd.enum_type:
            for v in e.value:
                setattr(self, v.name, v.number)

    def request_type(self, method):
        return getattr(self, self.methods[method][0])

    def response_type(self, method):
        return getattr(self, self.methods[method][1])


coordinator = _Namespace(FILES["coordinator"])
parameter_server = _Namespace(FILES["parameter_server"])


def emit_proto(out_dir: str) -> list[str]:
    """Copy the schema (proto/psd_*.proto) for non-Python peers: protoc --cpp_out on these files
    gives a reference-compatible C++ client/server."""
    import shutil

    os.makedirs(out_dir, exist_ok=True)
    paths = []
    for fname in PROTO_FILES.values():
        dst = os.path.join(out_dir, fname)
        shutil.copyfile(os.path.join(PROTO_DIR, fname), dst)
        paths.append(dst)
    return paths


if __name__ == "__main__":
    import sys

    print("\n".join(emit_proto(sys.argv[1] if len(sys.argv) > 1 else "proto_out")))
