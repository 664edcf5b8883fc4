"""Stream census of the asynchronous data plane.

HIP maps a process's streams onto GPU_MAX_HW_QUEUES = 4 hardware queues: a fifth busy stream
shares a queue with one of the others and serialises behind its work (a second push stream cost
17 ms per ResNet-50 step, profiles/async_push_streams_r4.md). This test runs 2 ranks on one MI355X
(gloo process group, the async PS at SSP bound 1 -- prefetching pulls -- owning one shard each, a
ResNet-50 at 64x64 through the Trainer), profiles three steps after warmup on every rank with the
torch profiler, and counts the distinct HIP streams that ran GPU work (kernels and copies): the
compute stream, the push stream, the pull stream and the owner engine's apply stream -- at most 4.
"""
import json
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from parameter_server_distributed_amd import models
    from parameter_server_distributed_amd.ops.optim import OptimConfig
    from parameter_server_distributed_amd.parallel.async_ps import AsyncPS
    from parameter_server_distributed_amd.runtime.trainer import Trainer

    torch.manual_seed(0)
    spec = models.build("resnet50", dev, torch.bfloat16, image_size=64)
    ps = AsyncPS(spec.model, OptimConfig("momentum", lr=0.01, momentum=0.9), num_shards=world, staleness=1,
                 bucket_mb=4, device=dev)
    tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(16, dev, seed=rank))
    for _ in range(4):
        tr.step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(3):
            tr.step()
        torch.cuda.synchronize()
    path = os.path.join(out_dir, f"trace{rank}.json")
    prof.export_chrome_trace(path)
    ps.drain()
    ps.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_async_plane_uses_at_most_4_streams(tmp_path, gpu):
    world = 2
    mp.spawn(_rank, args=(world, _port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        with open(tmp_path / f"trace{r}.json") as f:
            ev = json.load(f)["traceEvents"]
        gpu_ev = [e for e in ev if e.get("ph") == "X" and e.get("cat") in ("kernel", "gpu_memcpy", "gpu_memset")]
        assert len(gpu_ev) > 100, (r, len(gpu_ev))
        streams = {e["args"].get("stream") for e in gpu_ev if isinstance(e.get("args"), dict)}
        streams.discard(None)
        assert streams, f"rank {r}: no stream ids in the profiler trace"
        per = {s: sum(1 for e in gpu_ev if e["args"].get("stream") == s) for s in streams}
        print(f"rank {r}: {len(streams)} streams, GPU ops per stream {per}")
        assert len(streams) <= 4, (r, per)


def _streams_of(trace_path):
    with open(trace_path) as f:
        ev = json.load(f)["traceEvents"]
    gpu_ev = [e for e in ev if e.get("ph") == "X" and e.get("cat") in ("kernel", "gpu_memcpy", "gpu_memset")]
    per = {}
    for e in gpu_ev:
        s = e["args"].get("stream") if isinstance(e.get("args"), dict) else None
        if s is not None:
            per[s] = per.get(s, 0) + 1
    rccl = {e["args"].get("stream") for e in gpu_ev if isinstance(e.get("args"), dict)
            and ("nccl" in e.get("name", "").lower() or "rccl" in e.get("name", "").lower())}
    return per, rccl


def _nccl_world1(out_dir, plane):
    """One rank with the bench's N > 1 setup at world 1: an eager RCCL process group bound to the
    device (bench.py init_process_group("nccl", device_id=...)), the PS plane, the Trainer; three
    profiled steps followed by the bench's post-timing all_reduce."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0", WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    from parameter_server_distributed_amd import models
    from parameter_server_distributed_amd.ops.optim import OptimConfig
    from parameter_server_distributed_amd.parallel.async_ps import AsyncPS
    from parameter_server_distributed_amd.parallel.collective_ps import CollectivePS
    from parameter_server_distributed_amd.parallel.transport import make_transport
    from parameter_server_distributed_amd.runtime.trainer import Trainer

    torch.manual_seed(0)
    spec = models.build("resnet50", dev, torch.bfloat16, image_size=64)
    opt = OptimConfig("momentum", lr=0.01, momentum=0.9)
    if plane == "async":
        ps = AsyncPS(spec.model, opt, num_shards=1, staleness=1, bucket_mb=4, device=dev)
    else:  # the collective plane on the native RCCL communicator (transport "auto" -> rccl)
        ps = CollectivePS(spec.model, opt, make_transport("rccl", dev), num_shards=1, staleness=1, bucket_mb=4,
                          device=dev)
    tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(16, dev, seed=0))
    for _ in range(4):
        tr.step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(3):
            tr.step()
        t = torch.ones(4, device=dev)
        dist.all_reduce(t)  # the bench's histogram / timing all_reduce (after the timed steps)
        torch.cuda.synchronize()
    prof.export_chrome_trace(os.path.join(out_dir, f"nccl_{plane}.json"))
    if plane == "async":
        ps.drain()
    ps.close() if hasattr(ps, "close") else None
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("plane", ["async", "collective"])
def test_nccl_world1_stream_census(tmp_path, gpu, plane):
    """the census of the N > 1 setup -- the eager RCCL process group bench.py
    creates with device_id, and on the collective plane the native RCCL communicator -- in one rank
    at world 1 (RCCL needs a GPU per rank, so this is the largest RCCL world one MI355X holds). The
    streams that carry the training steps' work stay within the 4 hardware queues; the RCCL process
    group's own stream is used only by the post-timing all_reduce."""
    mp.spawn(_nccl_world1_entry, args=(str(tmp_path), plane), nprocs=1, join=True)
    per, rccl = _streams_of(tmp_path / f"nccl_{plane}.json")
    print(f"{plane}: {len(per)} streams, GPU ops per stream {per}; RCCL kernels on {sorted(rccl)}")
    assert sum(per.values()) > 100, per
    post = {s for s in rccl if per.get(s) == 1}  # the stream whose only op is the post-timing all_reduce
    assert len(per) - len(post) <= 4, (per, sorted(rccl))


def _nccl_world1_entry(_i, out_dir, plane):
    _nccl_world1(out_dir, plane)
