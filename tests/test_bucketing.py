"""Bucket-size policy (parallel/bucketing.py) on synthetic bandwidth tables, and the probe on a
2-rank gloo world (the policy input format; bandwidth numbers there are CPU, not xGMI)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from parameter_server_distributed_amd.parallel.bucketing import choose_bucket_mb


def test_knee_is_the_smallest_size_near_the_best_bandwidth():
    # xGMI-like curve: latency-bound below ~8 MB, flat above
    table = {1: 40.0, 2: 70.0, 4: 105.0, 8: 138.0, 16: 147.0, 32: 150.0, 64: 151.0}
    assert choose_bucket_mb(table, model_mb=50.0) == 8.0  # 138 >= 0.9 * 151
    assert choose_bucket_mb(table, model_mb=100.0, frac=0.97) == 16.0
    assert choose_bucket_mb(table, model_mb=50.0, frac=0.97) == 12.5  # capped: 4 buckets of the model


def test_cap_keeps_enough_buckets_to_overlap():
    table = {1: 10.0, 4: 40.0, 16: 100.0, 64: 150.0}
    assert choose_bucket_mb(table, model_mb=64.0) == 16.0  # knee 64 MB, but 64 / 4 buckets
    assert choose_bucket_mb(table, model_mb=1000.0) == 64.0
    assert choose_bucket_mb(table, model_mb=0.5) == 1.0  # never below the smallest measured size


def test_failed_or_empty_probes_fall_back():
    assert choose_bucket_mb({}, model_mb=100.0) == 16.0
    assert choose_bucket_mb({1: float("nan"), 4: -1, 16: "error"}, model_mb=100.0, default=8.0) == 8.0
    assert choose_bucket_mb({"4": 50.0, "16": 52.0}, model_mb=100.0) == 4.0  # JSON string keys


def _probe_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parameter_server_distributed_amd.parallel import bucketing

    # the probe's p2p pattern on CPU tensors (same code path as on GPUs apart from the sync)
    torch.cuda.synchronize = lambda *a, **k: None  # no GPU here
    t = bucketing.probe_p2p(torch.device("cpu"), sizes_mb=(0.25, 1), iters=2)
    if rank == 0:
        torch.save(t, out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
def test_probe_p2p_table_shape(tmp_path):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "t.pt")
    mp.spawn(_probe_worker, args=(2, port, out), nprocs=2, join=True)
    t = torch.load(out, weights_only=True)
    assert set(t) == {0.25, 1} and all(v > 0 for v in t.values())
    assert choose_bucket_mb(t, model_mb=100.0) in (0.25, 1.0)
