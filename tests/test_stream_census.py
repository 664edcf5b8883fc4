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
