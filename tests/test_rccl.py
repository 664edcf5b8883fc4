"""Native RCCL communicator (csrc/comm.cpp) on one MI355X (world size 1: every collective is an
identity, which still exercises unique-id bootstrap, communicator init, dtype mapping and stream
placement), plus the RcclTransport driving the collective PS end to end."""
import pytest
import torch

from parameter_server_distributed_amd import native

pytestmark = pytest.mark.gpu


def test_rccl_world1_collectives(gpu):
    C = native()
    uid = C.RcclComm.unique_id()
    assert isinstance(uid, bytes) and len(uid) == 128
    assert C.RcclComm.version() > 0
    comm = C.RcclComm(0, 1, uid, gpu.index or 0)
    x = torch.arange(64, dtype=torch.float32, device=gpu)
    comm.all_reduce(x, "sum", 0)
    torch.testing.assert_close(x.cpu(), torch.arange(64.0))
    b = torch.randn(128, device=gpu).to(torch.bfloat16)
    out = torch.empty_like(b)
    comm.reduce_scatter(b, out, "sum", 0)
    torch.testing.assert_close(out, b)
    g = torch.empty_like(b)
    comm.all_gather(b, g, 0)
    torch.testing.assert_close(g, b)
    comm.broadcast(b, 0, 0)
    s = torch.cuda.Stream()
    y = torch.ones(32, device=gpu)
    with torch.cuda.stream(s):
        comm.all_reduce(y, "max", s.cuda_stream)
    s.synchronize()
    assert y.sum().item() == 32
    assert comm.async_error() == ""
    comm.abort()


def test_rccl_transport_drives_collective_ps(gpu):
    import torch.distributed as dist

    from parameter_server_distributed_amd import models
    from parameter_server_distributed_amd.ops.optim import OptimConfig
    from parameter_server_distributed_amd.parallel.collective_ps import CollectivePS
    from parameter_server_distributed_amd.parallel.transport import RcclTransport
    from parameter_server_distributed_amd.runtime.trainer import Trainer

    store = dist.HashStore()
    t = RcclTransport(0, 1, gpu.index or 0, store=store)
    torch.manual_seed(0)
    spec = models.build("mlp", gpu, torch.bfloat16)
    ps = CollectivePS(spec.model, OptimConfig("momentum", lr=0.05), t, staleness=1, bucket_mb=0.1, device=gpu)
    tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(256, gpu))
    losses = [float(tr.step()) for _ in range(6)]
    assert losses[-1] < losses[0]
    assert ps.staleness_p50() == 1


def test_rccl_transport_graph_capture_matches_local(gpu, monkeypatch):
    """A whole collective-PS step (fwd, bwd, RCCL reduce-scatter / all-gather, fused apply) captured
    in a hipGraph on the native transport and replayed: same weights as the local-transport graph."""
    import torch.distributed as dist

    from parameter_server_distributed_amd import models
    from parameter_server_distributed_amd.ops.optim import OptimConfig
    from parameter_server_distributed_amd.parallel.collective_ps import CollectivePS
    from parameter_server_distributed_amd.parallel.transport import LocalTransport, RcclTransport
    from parameter_server_distributed_amd.runtime.trainer import Trainer

    monkeypatch.setenv("PSD_FEATURES", "linear_tune=0")  # same GEMM kernels in both runs
    out = []
    for t in (LocalTransport(), RcclTransport(0, 1, gpu.index or 0, store=dist.HashStore())):
        torch.manual_seed(0)
        spec = models.build("mlp", gpu, torch.bfloat16)
        ps = CollectivePS(spec.model, OptimConfig("momentum", lr=0.05), t, staleness=1, bucket_mb=0.1, device=gpu)
        tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(256, gpu), use_graph=True)
        for _ in range(8):
            tr.step()
        torch.cuda.synchronize()
        assert tr.graphs and tr.graph_error is None, tr.graph_error
        out.append(ps.params_flat.clone())
    assert torch.equal(out[0], out[1])
