"""Collective PS data plane, multi-process on CPU (gloo, world size 2): push/apply/pull over
reduce-scatter/all-gather (P = world) and reduce/broadcast (P < world), sync and bounded-staleness,
checked against a single-process fp32 reference of the same SGD-momentum trajectory."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from parameter_server_distributed_amd import models
from parameter_server_distributed_amd.ops.optim import OptimConfig
from parameter_server_distributed_amd.parallel.collective_ps import CollectivePS
from parameter_server_distributed_amd.parallel.transport import TorchDistTransport
from parameter_server_distributed_amd.runtime.trainer import Trainer

STEPS = 4
CFG = dict(kind="momentum", lr=0.1, momentum=0.9, weight_decay=1e-3)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, shards, stale, out, disjoint=False, push_mode="auto"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.float32, hidden=64)
    kw = {}
    if disjoint:  # first half workers, second half PS shards
        kw = dict(worker_ranks=list(range(world // 2)), ps_ranks=list(range(world // 2, world)))
    ps = CollectivePS(spec.model, OptimConfig(**CFG), TorchDistTransport(), num_shards=shards, staleness=stale,
                      bucket_mb=0.0005, grad_dtype=torch.float32, param_dtype=torch.float32, push_mode=push_mode, **kw)
    assert len(ps.buckets) > 1
    tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(16, torch.device("cpu"), seed=rank))
    for _ in range(STEPS):
        tr.step()
    params = {n: p.detach().clone() for n, p in spec.model.named_parameters()}
    hist = ps.staleness_histogram()
    if rank == 0:
        torch.save({"params": params, "hist": hist}, out)
    dist.barrier()
    dist.destroy_process_group()


def _reference(world, stale):
    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.float32, hidden=64)
    m = spec.model
    opt = torch.optim.SGD(m.parameters(), lr=CFG["lr"], momentum=CFG["momentum"], weight_decay=CFG["weight_decay"])
    batches = [spec.make_batch(16, torch.device("cpu"), seed=r) for r in range(world)]
    pending = []
    for t in range(STEPS):
        grads = [torch.zeros_like(p) for p in m.parameters()]
        for x, y in batches:
            m.zero_grad()
            spec.loss(m(x), y).backward()
            for g, p in zip(grads, m.parameters()):
                g += p.grad / world
        pending.append(grads)
        if t >= stale:
            g = pending.pop(0)
            for p, gg in zip(m.parameters(), g):
                p.grad = gg
            opt.step()
    return {n: p.detach() for n, p in m.named_parameters()}


@pytest.mark.slow
@pytest.mark.parametrize("shards,stale", [(2, 0), (1, 0), (2, 1), (1, 2)])
def test_gloo_world2_matches_reference(tmp_path, shards, stale):
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(2, _port(), shards, stale, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    want = _reference(2, stale)
    for n in want:
        torch.testing.assert_close(got["params"][n], want[n], rtol=1e-5, atol=1e-6, msg=n)
    hist = got["hist"]
    applied = STEPS - stale
    if shards == 2 or True:
        # rank 0 owns one shard in both layouts; every apply is recorded with its staleness
        assert sum(hist) == applied
        if stale and applied > stale:
            assert hist[stale] >= 1


@pytest.mark.slow
@pytest.mark.parametrize("world", [4, 8])
def test_gloo_bench_layout_2_shards_async(tmp_path, world):
    """The driver's scaling layout (bench.py defaults at N = 4 / 8): 2 PS shards colocated on
    ranks 0 and N/2, every rank a worker, staleness bound 1, reduce/broadcast push/pull."""
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(world, _port(), 2, 1, out, False, "reduce"), nprocs=world, join=True)
    got = torch.load(out, weights_only=True)
    want = _reference(world, 1)
    for n in want:
        torch.testing.assert_close(got["params"][n], want[n], rtol=1e-5, atol=1e-6, msg=n)
    assert sum(got["hist"]) == STEPS - 1 and got["hist"][1] >= 1


@pytest.mark.slow
def test_gloo_disjoint_placement_2_workers_2_ps(tmp_path):
    """BASELINE config 4 layout in miniature: PS shards on ranks that do no compute."""
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(4, _port(), 2, 0, out, True), nprocs=4, join=True)
    got = torch.load(out, weights_only=True)
    want = _reference(2, 0)
    for n in want:
        torch.testing.assert_close(got["params"][n], want[n], rtol=1e-5, atol=1e-6, msg=n)
    assert sum(got["hist"]) == 0  # rank 0 is a pure worker: it owns no shard


@pytest.mark.slow
@pytest.mark.parametrize("disjoint,shards,stale", [(True, 2, 0), (True, 2, 1), (False, 1, 0), (False, 2, 2)])
def test_gloo_p2p_push_matches_reference(tmp_path, disjoint, shards, stale):
    """Grouped send/recv push into per-worker inboxes + multi-source fused apply."""
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(4, _port(), shards, stale, out, disjoint, "p2p"), nprocs=4, join=True)
    got = torch.load(out, weights_only=True)
    want = _reference(2 if disjoint else 4, stale)
    for n in want:
        torch.testing.assert_close(got["params"][n], want[n], rtol=1e-5, atol=1e-6, msg=n)


def test_world1_local_matches_reference():
    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.float32, hidden=64)
    ps = CollectivePS(spec.model, OptimConfig(**CFG), staleness=0, bucket_mb=0.0005, grad_dtype=torch.float32,
                      param_dtype=torch.float32)
    tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(16, torch.device("cpu"), seed=0))
    for _ in range(STEPS):
        tr.step()
    want = _reference(1, 0)
    for n, p in spec.model.named_parameters():
        torch.testing.assert_close(p.detach(), want[n], rtol=1e-5, atol=1e-6)


def test_fp8_pull_publishes_fp8_representable_weights():
    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.bfloat16, hidden=64)
    ps = CollectivePS(spec.model, OptimConfig(**CFG), staleness=0, bucket_mb=0.0005, pull_dtype="fp8")
    tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(16, torch.device("cpu"), seed=0))
    for _ in range(2):
        tr.step()
    for b in ps.buckets:
        m = ps.master.narrow(0, b.local_offset, b.slice_numel)
        scale = m.abs().max().clamp_min(1e-12) / 448.0
        q = (m / scale).clamp(-448, 448).to(torch.float8_e4m3fn)
        want = (q.float() * scale).to(torch.bfloat16)
        got = ps.params_flat.narrow(0, b.offset, b.slice_numel)
        torch.testing.assert_close(got.float(), want.float(), rtol=1e-2, atol=1e-6)


def test_tracer_records_phases(tmp_path):
    from parameter_server_distributed_amd.utils.trace import StepTracer

    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.float32, hidden=64)
    ps = CollectivePS(spec.model, OptimConfig(**CFG), staleness=0, bucket_mb=0.0005, grad_dtype=torch.float32,
                      param_dtype=torch.float32)
    p = str(tmp_path / "trace.jsonl")
    tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(16, torch.device("cpu")), tracer=StepTracer(p))
    for _ in range(3):
        tr.step()
    tr.tracer.close()
    import json

    recs = [json.loads(ln) for ln in open(p)]
    assert [r["step"] for r in recs] == [0, 1, 2]
    for k in ("forward_ms", "backward_ms", "finish_ms", "comm_ms"):
        assert k in recs[-1] and recs[-1][k] >= 0


def _ckpt_worker(rank, world, port, prefix, phase, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.float32, hidden=64)
    ps = CollectivePS(spec.model, OptimConfig(**CFG), TorchDistTransport(), staleness=1, bucket_mb=0.0005,
                      grad_dtype=torch.float32, param_dtype=torch.float32)
    tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(16, torch.device("cpu"), seed=rank))
    if phase == "save":
        for _ in range(2):
            tr.step()
        th = ps.save(prefix, blocking=False)
        th.join()
        ps.export_reference(prefix + ".ref.ckpt", epoch=1, iteration=2)
    else:
        ps.load(prefix)
    for _ in range(2):
        tr.step()
    if rank == 0:
        torch.save({n: p.detach().clone() for n, p in spec.model.named_parameters()}, out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
def test_sharded_checkpoint_resume_is_exact(tmp_path, C):
    prefix = str(tmp_path / "ck")
    mp.spawn(_ckpt_worker, args=(2, _port(), prefix, "save", str(tmp_path / "a.pt")), nprocs=2, join=True)
    mp.spawn(_ckpt_worker, args=(2, _port(), prefix, "load", str(tmp_path / "b.pt")), nprocs=2, join=True)
    a = torch.load(str(tmp_path / "a.pt"), weights_only=True)
    b = torch.load(str(tmp_path / "b.pt"), weights_only=True)
    for n in a:
        torch.testing.assert_close(a[n], b[n], rtol=0, atol=0, msg=n)
    epoch, it, names, shapes, _, data = C.load_reference_ckpt(prefix + ".ref.ckpt")
    assert (epoch, it) == (1, 2) and "fc1.weight" in names


def _fp8_run(prefix, phase):
    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.bfloat16, hidden=64)
    ps = CollectivePS(spec.model, OptimConfig(**CFG), staleness=1, bucket_mb=0.0005, pull_dtype="fp8")
    tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(16, torch.device("cpu"), seed=0))
    if phase == "save":
        for _ in range(3):
            tr.step()
        ps.save(prefix)
    else:
        ps.load(prefix)
    for _ in range(2):
        tr.step()
    return {n: p.detach().clone() for n, p in spec.model.named_parameters()}


def test_fp8_pull_resume_is_exact(tmp_path):
    """Resume of an fp8-published run re-quantises the restored masters: the first
    gradients after load must be computed on the checkpointed weights, not the initial ones."""
    prefix = str(tmp_path / "ck8")
    a = _fp8_run(prefix, "save")
    b = _fp8_run(prefix, "load")
    for n in a:
        torch.testing.assert_close(a[n], b[n], rtol=0, atol=0, msg=n)


@pytest.mark.gpu
def test_async_save_is_a_consistent_snapshot_gpu(tmp_path, gpu, C):
    """save(blocking=False) followed at once by more training steps must write exactly the state of
    the step it was called at (the snapshot is ordered before the next fused apply)."""
    torch.manual_seed(0)
    spec = models.build("resnet50", gpu, torch.bfloat16, image_size=32, num_classes=10)
    ps = CollectivePS(spec.model, OptimConfig("momentum", lr=0.05), staleness=1, bucket_mb=4, device=gpu)
    tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(8, gpu))
    for _ in range(3):
        tr.step()
    ref, live = str(tmp_path / "ref"), str(tmp_path / "live")
    ps.save(ref, blocking=True)
    th = ps.save(live, blocking=False)
    for _ in range(3):
        tr.step()
    th.join()
    _, a = C.load_native_ckpt(ref + ".rank0.psd")
    _, b = C.load_native_ckpt(live + ".rank0.psd")
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_transport_policy_native_rccl_at_n_gt_1(monkeypatch):
    """N > 1 over an nccl process group always selects the native RCCL communicator (no torch-PG
    detour for device tensors); gloo / CPU select torch; world 1 is local."""
    from parameter_server_distributed_amd.parallel.transport import transport_kind

    monkeypatch.delenv("PSD_TRANSPORT", raising=False)
    assert transport_kind(8, "nccl") == "rccl"
    assert transport_kind(2, "nccl") == "rccl"
    assert transport_kind(2, "gloo") == "torch"
    assert transport_kind(2, "nccl", device_type="cpu") == "torch"
    assert transport_kind(1, "nccl") == "local"
    assert transport_kind(1, None, "rccl") == "rccl"
    with pytest.raises(ValueError):
        transport_kind(2, "nccl", "local")


def test_zero_plan_merges_accumulated_ranges():
    """The PS zeroes only the gradient ranges that are accumulated into (not the grad-sink ones):
    adjacent / overlapping spans merge; too many ranges or most of the buffer -> one full zero."""
    from parameter_server_distributed_amd.parallel.collective_ps import zero_grads_, zero_plan

    assert zero_plan([(64, 64), (0, 64), (256, 10)], 4096) == [(0, 128), (256, 10)]
    assert zero_plan([(0, 3000)], 4096) is None  # most of the buffer
    assert zero_plan([(i * 100, 10) for i in range(20)], 4096) is None  # too many launches
    assert zero_plan([], 4096) == []
    g = torch.ones(512)
    zero_grads_(g, [(0, 128), (256, 10)])
    assert float(g[:128].sum()) == 0 and float(g[128:256].sum()) == 128 and float(g[256:266].sum()) == 0
    zero_grads_(g, None)
    assert float(g.sum()) == 0


def test_bert_sink_params_skip_the_zero_fill():
    """With MfmaLinear / LayerNorm grad sinks, only the embeddings (and the plain LayerNorms) are
    accumulated: the PS zero plan covers a small part of BERT's gradient buffer."""
    from parameter_server_distributed_amd.parallel.collective_ps import zero_plan

    spec = models.build("bert_base", torch.device("cpu"), torch.float32, layers=2)
    direct = set()
    for m in spec.model.modules():
        if hasattr(m, "psd_direct_grad_params"):
            direct.update(id(p) for p in m.psd_direct_grad_params() if p is not None)
    off, spans = 0, []
    for p in spec.model.parameters():
        if id(p) not in direct:
            spans.append((off, p.numel()))
        off += p.numel()
    plan = zero_plan(spans, off)
    assert plan is not None and sum(n for _, n in plan) < off // 2
