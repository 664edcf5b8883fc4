"""Wire schema of the control plane, built at import time (no protoc in this image).

The two services keep the reference's package names, service names, method names, message names
and field numbers (proto/coordinator.proto, proto/parameter_server.proto of the reference), so a
reference C++ client/server can talk to ours. Everything we add is *additive*: new fields carry new
numbers and new methods new names, which proto3 peers ignore.

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

``emit_proto(dir)`` writes equivalent .proto text for non-Python peers.
"""
from __future__ import annotations

import os

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto
T = {"int32": F.TYPE_INT32, "int64": F.TYPE_INT64, "bool": F.TYPE_BOOL, "string": F.TYPE_STRING,
     "float": F.TYPE_FLOAT, "double": F.TYPE_DOUBLE, "bytes": F.TYPE_BYTES}

# (message, [(field, number, type, repeated)]); type "." = message/enum reference in-package
COORDINATOR = {
    "package": "coordinator",
    "enums": {"WorkerStatus": [("IDLE", 0), ("TRAINING", 1), ("CHECKPOINTING", 2), ("ERROR", 3)]},
    "messages": [
        ("WorkerInfo", [("worker_id", 1, "int32", False), ("address", 2, "string", False), ("port", 3, "int32", False),
                        ("hostname", 4, "string", False), ("status", 5, ".WorkerStatus", False),
                        ("gpu", 6, "int32", False)]),
        ("RegisterResponse", [("success", 1, "bool", False), ("message", 2, "string", False),
                              ("parameter_server_address", 3, "string", False), ("total_workers", 4, "int32", False),
                              ("membership_epoch", 5, "int64", False), ("ps_shard_addresses", 6, "string", True)]),
        ("HeartbeatRequest", [("worker_id", 1, "int32", False), ("status", 2, ".WorkerStatus", False)]),
        ("HeartbeatResponse", [("success", 1, "bool", False), ("timestamp", 2, "int64", False),
                               ("membership_epoch", 3, "int64", False)]),
        ("ListWorkersRequest", []),
        ("ListWorkersResponse", [("workers", 1, ".WorkerInfo", True), ("total_workers", 2, "int32", False),
                                 ("membership_epoch", 3, "int64", False)]),
        ("GetPSAddressRequest", []),
        ("GetPSAddressResponse", [("address", 1, "string", False), ("port", 2, "int32", False),
                                  ("shard_addresses", 3, "string", True)]),
        ("KvRequest", [("key", 1, "string", False), ("value", 2, "bytes", False), ("timeout_ms", 3, "int32", False)]),
        ("KvResponse", [("found", 1, "bool", False), ("value", 2, "bytes", False)]),
    ],
    "service": ("Coordinator", [
        ("RegisterWorker", "WorkerInfo", "RegisterResponse"),
        ("Heartbeat", "HeartbeatRequest", "HeartbeatResponse"),
        ("ListWorkers", "ListWorkersRequest", "ListWorkersResponse"),
        ("GetParameterServerAddress", "GetPSAddressRequest", "GetPSAddressResponse"),
        ("Deregister", "WorkerInfo", "RegisterResponse"),
        ("KvSet", "KvRequest", "KvResponse"),
        ("KvGet", "KvRequest", "KvResponse"),
    ]),
}

PARAMETER_SERVER = {
    "package": "parameter_server",
    "enums": {},
    "messages": [
        ("GradientUpdate", [("worker_id", 1, "int32", False), ("iteration", 2, "int32", False),
                            ("gradients", 3, ".Tensor", True), ("pulled_version", 4, "int64", False)]),
        ("Tensor", [("name", 1, "string", False), ("shape", 2, "int32", True), ("data", 3, "float", True),
                    ("dtype", 4, "int32", False), ("raw", 5, "bytes", False)]),
        ("PushResponse", [("success", 1, "bool", False), ("message", 2, "string", False),
                          ("iteration", 3, "int32", False), ("aggregation_complete", 4, "bool", False),
                          ("workers_received", 5, "int32", False), ("total_workers", 6, "int32", False),
                          ("version", 7, "int64", False), ("staleness", 8, "int64", False)]),
        ("PullRequest", [("worker_id", 1, "int32", False), ("iteration", 2, "int32", False),
                         ("wait_ms", 3, "int32", False), ("accept_raw", 4, "bool", False)]),
        ("ParameterUpdate", [("iteration", 1, "int32", False), ("parameters", 2, ".Tensor", True),
                             ("ready", 3, "bool", False), ("version", 4, "int64", False)]),
        ("SyncStatusRequest", [("iteration", 1, "int32", False)]),
        ("SyncStatusResponse", [("iteration", 1, "int32", False), ("ready", 2, "bool", False),
                                ("workers_received", 3, "int32", False), ("total_workers", 4, "int32", False)]),
        ("SaveCheckpointRequest", [("epoch", 1, "int32", False), ("path", 2, "string", False)]),
        ("SaveCheckpointResponse", [("success", 1, "bool", False), ("message", 2, "string", False),
                                    ("checkpoint_path", 3, "string", False)]),
        ("LoadCheckpointRequest", [("path", 1, "string", False), ("accept_raw", 2, "bool", False)]),
        ("LoadCheckpointResponse", [("success", 1, "bool", False), ("message", 2, "string", False),
                                    ("epoch", 3, "int32", False), ("parameters", 4, ".Tensor", True),
                                    ("iteration", 5, "int32", False)]),
        ("StatsResponse", [("version", 1, "int64", False), ("current_iteration", 2, "int32", False),
                           ("total_workers", 3, "int32", False), ("staleness_histogram", 4, "int64", True),
                           ("counters_json", 5, "string", False)]),
        ("SetTotalWorkersRequest", [("total_workers", 1, "int32", False)]),
    ],
    "service": ("ParameterServer", [
        ("ReceiveGradients", "GradientUpdate", "PushResponse"),
        ("ServeParameters", "PullRequest", "ParameterUpdate"),
        ("CheckSyncStatus", "SyncStatusRequest", "SyncStatusResponse"),
        ("SaveCheckpoint", "SaveCheckpointRequest", "SaveCheckpointResponse"),
        ("LoadCheckpoint", "LoadCheckpointRequest", "LoadCheckpointResponse"),
        ("InitParameters", "GradientUpdate", "PushResponse"),
        ("GetStats", "SyncStatusRequest", "StatsResponse"),
        ("SetTotalWorkers", "SetTotalWorkersRequest", "PushResponse"),
    ]),
}


def _file_proto(spec: dict, name: str) -> descriptor_pb2.FileDescriptorProto:
    pkg = spec["package"]
    fd = descriptor_pb2.FileDescriptorProto(name=name, package=pkg, syntax="proto3")
    for ename, vals in spec["enums"].items():
        e = fd.enum_type.add(name=ename)
        for vn, vv in vals:
            e.value.add(name=vn, number=vv)
    for mname, fields in spec["messages"]:
        m = fd.message_type.add(name=mname)
        for fname, num, ftype, rep in fields:
            f = m.field.add(name=fname, number=num, label=F.LABEL_REPEATED if rep else F.LABEL_OPTIONAL)
            if ftype.startswith("."):
                tname = ftype[1:]
                f.type = F.TYPE_ENUM if tname in spec["enums"] else F.TYPE_MESSAGE
                f.type_name = f".{pkg}.{tname}"
            else:
                f.type = T[ftype]
    sname, methods = spec["service"]
    s = fd.service.add(name=sname)
    for meth, req, resp in methods:
        s.method.add(name=meth, input_type=f".{pkg}.{req}", output_type=f".{pkg}.{resp}")
    return fd


_POOL = descriptor_pool.DescriptorPool()
_FILES = {}
for _spec, _name in ((COORDINATOR, "psd_coordinator.proto"), (PARAMETER_SERVER, "psd_parameter_server.proto")):
    _FILES[_spec["package"]] = _POOL.Add(_file_proto(_spec, _name))


class _Namespace:
    def __init__(self, spec):
        self.package = spec["package"]
        self.service_name = f"{spec['package']}.{spec['service'][0]}"
        self.methods = {m: (req, resp) for (m, req, resp) in spec["service"][1]}
        for mname, _ in spec["messages"]:
            desc = _POOL.FindMessageTypeByName(f"{spec['package']}.{mname}")
            setattr(self, mname, message_factory.GetMessageClass(desc))
        for ename, vals in spec["enums"].items():
            for vn, vv in vals:
                setattr(self, vn, vv)

    def request_type(self, method):
        return getattr(self, self.methods[method][0])

    def response_type(self, method):
        return getattr(self, self.methods[method][1])


coordinator = _Namespace(COORDINATOR)
parameter_server = _Namespace(PARAMETER_SERVER)


def emit_proto(out_dir: str) -> list[str]:
    """Write .proto text equivalent to the runtime descriptors (for non-Python peers)."""
    os.makedirs(out_dir, exist_ok=True)
    paths = []
    for spec, fname in ((COORDINATOR, "coordinator.proto"), (PARAMETER_SERVER, "parameter_server.proto")):
        lines = ['syntax = "proto3";', "", f"package {spec['package']};", ""]
        sname, methods = spec["service"]
        lines.append(f"service {sname} {{")
        for m, req, resp in methods:
            lines.append(f"  rpc {m}({req}) returns ({resp});")
        lines += ["}", ""]
        for ename, vals in spec["enums"].items():
            lines.append(f"enum {ename} {{")
            lines += [f"  {vn} = {vv};" for vn, vv in vals]
            lines += ["}", ""]
        for mname, fields in spec["messages"]:
            lines.append(f"message {mname} {{")
            for fname_, num, ftype, rep in fields:
                t = ftype[1:] if ftype.startswith(".") else ftype
                lines.append(f"  {'repeated ' if rep else ''}{t} {fname_} = {num};")
            lines += ["}", ""]
        p = os.path.join(out_dir, fname)
        with open(p, "w") as f:
            f.write("\n".join(lines))
        paths.append(p)
    return paths


if __name__ == "__main__":
    import sys

    print("\n".join(emit_proto(sys.argv[1] if len(sys.argv) > 1 else "proto_out")))
