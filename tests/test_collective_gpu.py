"""The overlapped GPU data plane at world size 2: two ranks share cuda:0 over
gloo, every bucket's push / fused apply / pull runs on the PS comm stream from the gradient hooks
while backward continues, with several buckets and staleness S = 1. Checked against the fp32
single-process reference trajectory of the same delayed-gradient SGD-momentum (the CPU test's
``_reference``), and the ranks' published weights must be bit-identical after every step."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from parameter_server_distributed_amd import models
from parameter_server_distributed_amd.ops.optim import OptimConfig
from parameter_server_distributed_amd.parallel.collective_ps import CollectivePS
from parameter_server_distributed_amd.parallel.transport import TorchDistTransport
from parameter_server_distributed_amd.runtime.trainer import Trainer

from test_collective_ps import CFG, _port, _reference  # noqa: E402

STEPS = 4


def _fp(t: torch.Tensor):
    w = t.view(torch.int16 if t.element_size() == 2 else torch.int32).to(torch.int64)
    pos = torch.arange(w.numel(), device=w.device, dtype=torch.int64) % 1009 + 1
    return [int(w.sum().item()), int((w * pos).sum().item())]


def _worker(rank, world, port, model, stale, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    if model == "mlp":
        spec = models.build("mlp", dev, torch.float32, hidden=64)
        kw = dict(grad_dtype=torch.float32, param_dtype=torch.float32, bucket_mb=0.0005)
        batch = spec.make_batch(16, dev, seed=rank)
    else:
        spec = models.build("resnet50", dev, torch.bfloat16, image_size=32, num_classes=10)
        kw = dict(bucket_mb=2.0)
        batch = spec.make_batch(8, dev, seed=rank)
    ps = CollectivePS(spec.model, OptimConfig(**CFG), TorchDistTransport(), num_shards=2, staleness=stale,
                      device=dev, overlap=True, **kw)
    assert len(ps.buckets) > 1 and ps.is_cuda
    tr = Trainer(spec.model, spec.loss, ps, batch, use_graph=False)
    fps = []
    for _ in range(STEPS):
        tr.step()
        torch.cuda.synchronize()
        fps.append(_fp(ps.params_flat))
    got = [None] * world
    dist.all_gather_object(got, fps)
    if rank == 0:
        params = {n: p.detach().float().cpu().clone() for n, p in spec.model.named_parameters()}
        torch.save({"params": params, "fps": got}, out)
    dist.barrier()
    dist.destroy_process_group()


def _resnet_reference(world, stale, dev):
    """The same trajectory in one process on the same GPU kernels: bf16 working weights, each
    rank's gradient computed in turn, averaged in fp32, applied (S steps late) by torch SGD to an
    fp32 master. What the data plane may change is only the gradient summation (bf16 reduce)."""
    torch.manual_seed(0)
    spec = models.build("resnet50", dev, torch.bfloat16, image_size=32, num_classes=10)
    m = spec.model
    params = [p for p in m.parameters() if p.requires_grad]
    master = [p.detach().float().clone() for p in params]
    init = {n: p.detach().float().cpu().clone() for n, p in m.named_parameters()}
    for p, w in zip(params, master):
        p.data = w.to(torch.bfloat16)
    opt = torch.optim.SGD(master, lr=CFG["lr"], momentum=CFG["momentum"], weight_decay=CFG["weight_decay"])
    batches = [spec.make_batch(8, dev, seed=r) for r in range(world)]
    pending = []
    for t in range(STEPS):
        grads = [torch.zeros_like(w) for w in master]
        for x, y in batches:
            for p in params:
                p.grad = None
            spec.loss(m(x), y).backward()
            for g, p in zip(grads, params):
                g += p.grad.float() / world
        pending.append(grads)
        if t >= stale:
            for w, gg in zip(master, pending.pop(0)):
                w.grad = gg
            opt.step()
            for p, w in zip(params, master):
                p.data.copy_(w)
    names = [n for n, p in m.named_parameters() if p.requires_grad]
    return {n: w.detach().cpu() for n, w in zip(names, master)}, init


@pytest.mark.gpu
@pytest.mark.parametrize("stale", [1, 0])
def test_world2_overlapped_mlp_matches_fp32_reference(tmp_path, gpu, stale):
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(2, _port(), "mlp", stale, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    assert got["fps"][0] == got["fps"][1], "ranks hold different published weights"
    want = _reference(2, stale)
    for n in want:
        torch.testing.assert_close(got["params"][n], want[n], rtol=1e-4, atol=1e-5, msg=n)


@pytest.mark.gpu
def test_world2_overlapped_resnet_bf16_tracks_fp32_reference(tmp_path, gpu):
    """bf16 ResNet through the fused BN / conv kernels, 2 ranks, S = 1, several buckets: the
    weight *updates* (w_T - w_0) must agree with a single-process replay on the same kernels with an
    fp32 gradient average and fp32 master -- a dropped, doubled or torn bucket update would be off
    by ~100 %."""
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(2, _port(), "resnet", 1, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    assert got["fps"][0] == got["fps"][1], "ranks hold different published weights"
    want, init = _resnet_reference(2, 1, gpu)
    num = den = 0.0
    worst = []
    for n in want:
        g, w, i = got["params"][n], want[n], init[n]
        assert torch.isfinite(g).all(), n
        d_ref = w - i  # compare the updates (both runs start from the same init)
        d_gpu = g - i
        du_ref = d_ref.norm().item()
        du_err = (d_gpu - d_ref).norm().item()
        num += du_err ** 2
        den += du_ref ** 2
        if du_ref > 1e-3:
            worst.append((du_err / du_ref, n))
    assert (num / den) ** 0.5 < 0.1, ((num / den) ** 0.5, sorted(worst)[-5:])
