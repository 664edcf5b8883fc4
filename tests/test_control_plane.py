"""Control plane: wire schema compatibility, coordinator registry, PS core semantics, checkpoints."""
import json
import os
import struct
import threading

import pytest
import torch

from parameter_server_distributed_amd.ops.optim import OptimConfig
from parameter_server_distributed_amd.rpc import schema, service
from parameter_server_distributed_amd.runtime.coordinator import split_host_port
from parameter_server_distributed_amd.runtime.parameter_server import make_config

# Field numbers of the reference's proto/coordinator.proto and proto/parameter_server.proto.
REFERENCE_FIELDS = {
    ("coordinator", "WorkerInfo"): {"worker_id": 1, "address": 2, "port": 3, "hostname": 4},
    ("coordinator", "RegisterResponse"): {"success": 1, "message": 2, "parameter_server_address": 3,
                                          "total_workers": 4},
    ("coordinator", "HeartbeatRequest"): {"worker_id": 1, "status": 2},
    ("coordinator", "HeartbeatResponse"): {"success": 1, "timestamp": 2},
    ("coordinator", "ListWorkersResponse"): {"workers": 1, "total_workers": 2},
    ("coordinator", "GetPSAddressResponse"): {"address": 1, "port": 2},
    ("parameter_server", "GradientUpdate"): {"worker_id": 1, "iteration": 2, "gradients": 3},
    ("parameter_server", "Tensor"): {"name": 1, "shape": 2, "data": 3, "dtype": 4},
    ("parameter_server", "PushResponse"): {"success": 1, "message": 2, "iteration": 3, "aggregation_complete": 4,
                                           "workers_received": 5, "total_workers": 6},
    ("parameter_server", "PullRequest"): {"worker_id": 1, "iteration": 2},
    ("parameter_server", "ParameterUpdate"): {"iteration": 1, "parameters": 2, "ready": 3},
    ("parameter_server", "SyncStatusRequest"): {"iteration": 1},
    ("parameter_server", "SyncStatusResponse"): {"iteration": 1, "ready": 2, "workers_received": 3,
                                                 "total_workers": 4},
    ("parameter_server", "SaveCheckpointRequest"): {"epoch": 1, "path": 2},
    ("parameter_server", "SaveCheckpointResponse"): {"success": 1, "message": 2, "checkpoint_path": 3},
    ("parameter_server", "LoadCheckpointRequest"): {"path": 1},
    ("parameter_server", "LoadCheckpointResponse"): {"success": 1, "message": 2, "epoch": 3, "parameters": 4},
}
REFERENCE_METHODS = {
    "coordinator.Coordinator": ["RegisterWorker", "Heartbeat", "ListWorkers", "GetParameterServerAddress"],
    "parameter_server.ParameterServer": ["ReceiveGradients", "ServeParameters", "CheckSyncStatus", "SaveCheckpoint",
                                         "LoadCheckpoint"],
}


@pytest.mark.parametrize("key", list(REFERENCE_FIELDS), ids=lambda k: f"{k[0]}.{k[1]}")
def test_wire_field_numbers_match_reference(key):
    ns = getattr(schema, key[0])
    desc = getattr(ns, key[1]).DESCRIPTOR
    got = {f.name: f.number for f in desc.fields}
    for name, num in REFERENCE_FIELDS[key].items():
        assert got[name] == num, f"{key}.{name}"


def test_service_and_method_names():
    for ns in (schema.coordinator, schema.parameter_server):
        for m in REFERENCE_METHODS[ns.service_name]:
            assert m in ns.methods
    assert schema.coordinator.TRAINING == 1 and schema.coordinator.ERROR == 3


def test_tensor_codec_raw_and_reference_encoding():
    t = torch.randn(3, 5)
    for raw in (True, False):
        m = service.tensor_to_proto("w", t, raw=raw)
        m2 = schema.parameter_server.Tensor.FromString(m.SerializeToString())
        torch.testing.assert_close(service.proto_to_tensor(m2), t)
    b = service.proto_to_tensor(service.tensor_to_proto("w", t, raw=True, bf16=True))
    torch.testing.assert_close(b, t.to(torch.bfloat16).float())


def test_emit_proto(tmp_path):
    paths = schema.emit_proto(str(tmp_path))
    txt = open(paths[1]).read()
    assert "rpc ReceiveGradients(GradientUpdate) returns (PushResponse);" in txt
    assert "repeated float data = 3;" in txt


REF_PROTO = os.environ.get("PSD_REFERENCE_PROTO_DIR", "/root/reference/proto")


@pytest.mark.skipif(not os.path.isdir(REF_PROTO), reason="reference .proto files not present")
@pytest.mark.parametrize("pkg,fname", [("coordinator", "coordinator.proto"),
                                       ("parameter_server", "parameter_server.proto")])
def test_schema_is_a_wire_superset_of_the_reference_proto(pkg, fname):
    """Parse the reference's own .proto (read-only) and require every message, field name, field
    number, scalar/enum/message type, label (repeated or not), enum value and rpc signature to be
    identical in our proto/psd_*.proto -- names, numbers *and* types (the old test
    checked hand-copied numbers only)."""
    from parameter_server_distributed_amd.rpc import protoparse

    ref = protoparse.describe(protoparse.parse_file(os.path.join(REF_PROTO, fname)))
    ours = protoparse.describe(schema.FILES[pkg])
    diff = {k: (v, ours.get(k)) for k, v in ref.items() if ours.get(k) != v}
    assert not diff, diff
    ref_fd = protoparse.parse_file(os.path.join(REF_PROTO, fname))
    assert ref_fd.package == schema.FILES[pkg].package
    # additions are additive: our extra fields never reuse a number the reference message has
    for m in schema.FILES[pkg].message_type:
        rm = next((x for x in ref_fd.message_type if x.name == m.name), None)
        if rm is None:
            continue
        ref_nums = {f.number: f.name for f in rm.field}
        for f in m.field:
            assert ref_nums.get(f.number, f.name) == f.name, (m.name, f.name, f.number)


def test_wire_types_of_reference_fields():
    """Types the reference relies on, pinned without the reference tree (e.g. timestamp int64,
    shape repeated int32, data repeated float)."""
    from google.protobuf.descriptor import FieldDescriptor as FD

    hb = schema.coordinator.HeartbeatResponse.DESCRIPTOR.fields_by_name["timestamp"]
    assert hb.type == FD.TYPE_INT64
    t = schema.parameter_server.Tensor.DESCRIPTOR.fields_by_name
    assert t["shape"].type == FD.TYPE_INT32 and t["shape"].is_repeated
    assert t["data"].type == FD.TYPE_FLOAT and t["data"].is_repeated
    assert schema.coordinator.HeartbeatRequest.DESCRIPTOR.fields_by_name["status"].enum_type.name == "WorkerStatus"
    g = schema.parameter_server.GradientUpdate.DESCRIPTOR.fields_by_name["gradients"]
    assert g.message_type.name == "Tensor" and g.is_repeated


def test_proto_parser_grammar_and_errors():
    from parameter_server_distributed_amd.rpc import protoparse

    fd = protoparse.parse('''
        syntax = "proto3";  /* block
        comment */ package demo;
        option cc_enable_arenas = true;
        enum E { A = 0; B = 1; }
        message M { repeated int64 xs = 1 [packed = true]; E e = 2; N n = 3; reserved 9; }
        message N {}
        service S { rpc Do(M) returns (N); rpc Opt(N) returns (M) {} }
    ''', "demo.proto")
    d = protoparse.describe(fd)
    assert d["M.xs"][0] == 1 and d["M.e"][3] == "E" and d["M.n"][3] == "N" and d["rpc S.Opt"] == ("N", "M")
    with pytest.raises(protoparse.ProtoSyntaxError):
        protoparse.parse('syntax = "proto3"; package p; message M { Unknown u = 1; }', "bad.proto")
    with pytest.raises(protoparse.ProtoSyntaxError):
        protoparse.parse('syntax = "proto3"; package p; extend M {}', "bad.proto")


def test_split_host_port():
    assert split_host_port("localhost:50051", 1) == ("localhost", 50051)
    assert split_host_port("10.0.0.5", 50051) == ("10.0.0.5", 50051)
    assert split_host_port("[::1]:7", 1) == ("::1", 7)


def test_registry_heartbeat_expiry_and_epochs(C):
    r = C.Registry("ps-host", 50051)
    r.use_manual_clock(100.0)
    res = r.register_worker(0, "", 0, "")
    assert res.success and res.ps_address == "ps-host:50051" and res.total_workers == 1
    e1 = res.membership_epoch
    r.register_worker(1, "10.0.0.2", 7000, "h1")
    assert r.membership_epoch() == e1 + 1
    r.register_worker(1, "10.0.0.2", 7000, "h1")  # re-register: no epoch bump
    assert r.membership_epoch() == e1 + 1
    r.advance_clock(20)
    assert r.heartbeat(1, 1)
    assert not r.heartbeat(9, 1)
    r.advance_clock(15)  # worker 0 silent 35 s > 30 s
    assert r.remove_stale(30.0) == [0]
    assert r.live_ids() == [1]
    assert r.membership_epoch() == e1 + 2
    ws = r.list_workers()
    assert ws[0].hostname == "h1" and ws[0].status == 1
    assert r.deregister(1) and r.live_ids() == []


def test_registry_kv_rendezvous(C):
    r = C.Registry("h", 1)
    out = {}

    def getter():
        out["v"] = r.kv_get("uid", 5.0)

    t = threading.Thread(target=getter)
    t.start()
    r.kv_set("uid", b"\x00\x01" * 64)
    t.join()
    assert out["v"] == (True, b"\x00\x01" * 64)
    assert r.kv_get("missing", 0.01) == (False, b"")


def _core(C, workers=2, mode="sync", staleness=-1, optim=None, compat=False):
    cfg = make_config(workers, optim or OptimConfig("sgd", lr=0.5, momentum=0.0), mode, staleness, compat)
    return C.PSCore(cfg, "cpu")


def test_sync_barrier_average_and_update(C):
    core = _core(C)
    core.init_params(["w"], [[4]], [torch.ones(4)])
    r0 = core.push(0, 0, ["w"], [torch.full((4,), 2.0)], -1)
    assert r0.success and not r0.aggregation_complete and r0.workers_received == 1
    assert core.sync_status(0) == (False, 1, 2)
    r0b = core.push(0, 0, ["w"], [torch.full((4,), 4.0)], -1)  # re-push overwrites (reference semantics)
    assert r0b.workers_received == 1
    r1 = core.push(1, 0, ["w"], [torch.full((4,), 6.0)], -1)
    assert r1.aggregation_complete and r1.workers_received == 2
    ready, _, ver, flat = core.pull(0, 0, 0.0)
    assert ready and ver == 1
    torch.testing.assert_close(flat[:4], torch.full((4,), 1.0 - 0.5 * 5.0))  # p -= lr * mean(4, 6)
    late = core.push(0, 0, ["w"], [torch.ones(4)], -1)
    assert late.aggregation_complete and "late" in late.message
    assert core.counters()["late_dropped"] == 1
    bad = core.push(0, 1, ["w"], [torch.ones(5)], -1)
    assert not bad.success and "mismatch" in bad.message


def test_reference_compat_first_aggregate_becomes_params(C):
    core = _core(C, compat=True)
    core.push(0, 0, ["weight"], [torch.full((10, 10), 0.01)], -1)
    r = core.push(1, 0, ["weight"], [torch.full((10, 10), 0.03)], -1)
    assert r.aggregation_complete
    _, _, _, flat = core.pull(0, 0, 0.0)
    torch.testing.assert_close(flat[:100], torch.full((100,), 0.02))
    core.push(0, 1, ["weight"], [torch.full((10, 10), 0.01)], -1)
    core.push(1, 1, ["weight"], [torch.full((10, 10), 0.01)], -1)
    _, _, _, flat = core.pull(0, 1, 0.0)
    torch.testing.assert_close(flat[:100], torch.full((100,), 0.01))  # p -= g with lr 1


def test_sync_pull_long_poll_and_membership_shrink(C):
    core = _core(C, workers=3)
    core.init_params(["w"], [[2]], [torch.zeros(2)])
    core.push(0, 0, ["w"], [torch.ones(2)], -1)
    core.push(1, 0, ["w"], [torch.ones(2)], -1)
    res = {}
    t = threading.Thread(target=lambda: res.setdefault("r", core.pull(0, 0, 5.0)))
    t.start()
    core.set_total_workers(2)  # worker 2 left: the pending iteration completes with 2 pushes
    t.join()
    assert res["r"][0] is True and core.version() == 1


def test_async_staleness_histogram_and_ssp_bound(C):
    core = _core(C, workers=2, mode="async", staleness=1, optim=OptimConfig("sgd", lr=1.0, momentum=0.0))
    core.init_params(["w"], [[2]], [torch.zeros(2)])
    # worker 0 pulls v0 and pushes twice before worker 1 pushes its v0 gradient
    assert core.pull(0, 0, 0.0)[0]
    r = core.push(0, 0, ["w"], [torch.ones(2)], 0)
    assert r.staleness == 0 and r.version == 1
    assert core.pull(0, 1, 0.0)[0]  # clock lead 1 <= S
    core.push(0, 1, ["w"], [torch.ones(2)], 1)
    # worker 0 now leads worker 1 (clock 0) by 2 > S=1: a pull for iteration 2 is held
    assert core.pull(0, 2, 0.05)[0] is False
    r1 = core.push(1, 0, ["w"], [torch.ones(2)], 0)
    assert r1.staleness == 2
    hist = core.staleness_histogram()
    assert hist[0] == 2 and hist[2] == 1
    # async grad scale 1/W: three unit gradients at lr 1 -> -1.5
    torch.testing.assert_close(core.pull(0, 1, 0.0)[3][:2], torch.full((2,), -1.5))


def _read_reference_ckpt(path):
    """Independent pure-Python reader of the reference layout (src/parameter_server.cpp:112-144)."""
    with open(path, "rb") as f:
        b = f.read()
    o = 0
    epoch, it = struct.unpack_from("<ii", b, o)
    o += 8
    (n,) = struct.unpack_from("<Q", b, o)
    o += 8
    out = []
    for _ in range(n):
        (nl,) = struct.unpack_from("<Q", b, o)
        o += 8
        name = b[o:o + nl].decode()
        o += nl
        (rank,) = struct.unpack_from("<Q", b, o)
        o += 8
        shape = list(struct.unpack_from(f"<{rank}i", b, o))
        o += 4 * rank
        (dt,) = struct.unpack_from("<i", b, o)
        o += 4
        (numel,) = struct.unpack_from("<Q", b, o)
        o += 8
        data = list(struct.unpack_from(f"<{numel}f", b, o))
        o += 4 * numel
        out.append((name, shape, dt, data))
    assert o == len(b)
    return epoch, it, out


def test_reference_checkpoint_layout_roundtrip(C, tmp_path):
    core = _core(C)
    core.init_params(["weight", "bias"], [[2, 3], [3]], [torch.arange(6.0).reshape(2, 3), torch.tensor([7.0, 8, 9])])
    p = str(tmp_path / "checkpoint_epoch_3.ckpt")
    assert core.save_reference(p, 3)
    epoch, it, ts = _read_reference_ckpt(p)
    assert epoch == 3 and it == 0
    assert ts[0] == ("weight", [2, 3], 0, [0.0, 1, 2, 3, 4, 5]) and ts[1][3] == [7.0, 8, 9]
    core2 = _core(C)
    assert core2.load_reference(p) == (True, 3)
    torch.testing.assert_close(core2.pull(0, 0, 0.0)[3][:6], torch.arange(6.0))


def test_reference_checkpoint_written_by_python_is_loadable(C, tmp_path):
    """A file in the reference's exact byte layout (as its C++ PS would write it) imports cleanly."""
    p = tmp_path / "ref.ckpt"
    with open(p, "wb") as f:
        f.write(struct.pack("<iiQ", 5, 42, 1))
        f.write(struct.pack("<Q", 6) + b"weight" + struct.pack("<Q", 2) + struct.pack("<ii", 10, 10))
        f.write(struct.pack("<iQ", 0, 100) + struct.pack("<100f", *([0.01] * 100)))
    epoch, it, names, shapes, dtypes, data = C.load_reference_ckpt(str(p))
    assert (epoch, it, names, shapes, dtypes) == (5, 42, ["weight"], [[10, 10]], [0])
    torch.testing.assert_close(data[0], torch.full((100,), 0.01))


def test_native_checkpoint_crc_and_atomicity(C, tmp_path):
    p = str(tmp_path / "shard0.psd")
    ts = [torch.randn(33), torch.arange(5, dtype=torch.int32), torch.randn(4, 4).to(torch.bfloat16)]
    C.save_native_ckpt(p, json.dumps({"k": 1}), ts)
    assert not os.path.exists(p + ".tmp")
    man, back = C.load_native_ckpt(p)
    assert json.loads(man) == {"k": 1}
    for a, b in zip(ts, back):
        assert torch.equal(a, b)
    raw = bytearray(open(p, "rb").read())
    raw[-3] ^= 0xFF
    open(p, "wb").write(bytes(raw))
    with pytest.raises(RuntimeError, match="checksum"):
        C.load_native_ckpt(p)


def test_run_config_yaml_and_json(tmp_path):
    import argparse

    from parameter_server_distributed_amd.utils.config import apply_config

    y = tmp_path / "r.yaml"
    y.write_text("ps-shards: 4\nstaleness: 2\n")
    ap = argparse.ArgumentParser()
    ap.add_argument("--ps-shards", type=int, default=2)
    ap.add_argument("--staleness", type=int, default=1)
    apply_config(ap, ["--config", str(y), "--staleness", "3"])
    a = ap.parse_args(["--config", str(y), "--staleness", "3"])
    assert (a.ps_shards, a.staleness) == (4, 3)  # file sets defaults, flags win
    j = tmp_path / "r.json"
    j.write_text('{"bogus": 1}')
    ap2 = argparse.ArgumentParser()
    with pytest.raises(SystemExit):
        apply_config(ap2, ["--config", str(j)])


def test_shipped_configs_parse():
    import glob
    import os

    from parameter_server_distributed_amd.utils.config import load_config

    files = glob.glob(os.path.join(os.path.dirname(__file__), "..", "configs", "*.yaml"))
    assert files
    for f in files:
        assert "model" in load_config(f)
