"""Gradient-bucket size from a measured bandwidth-vs-size table.

A push bucket is the unit the data plane moves while backward is still running: the async plane
DMA-copies each bucket into its owners' inboxes over xGMI (one hipMemcpyAsync per owner), the
collective plane reduce-scatters it. Small buckets start moving earlier and overlap more of the
backward pass; large ones amortise the per-transfer cost (launch, protocol, DMA setup: tens of us)
and reach the link's bandwidth. An MI355X node links every GPU pair directly (7 xGMI links per
GPU, ~153 GB/s each), so the knee of the curve is a property of the node, not of NVSwitch-style
topology guesses: measure it, then take the smallest size that reaches ``frac`` of the best
measured bandwidth, capped so that the model still splits into ``min_buckets`` buckets (otherwise
nothing overlaps).

The reference moves whole models in one gRPC message per push (src/worker.cpp:254-272) and has no
buckets; its only collective is one ncclAllReduce per tensor (src/nccl_manager.cpp:102-121).
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist


def choose_bucket_mb(table: dict, model_mb: float, min_buckets: int = 4, frac: float = 0.9,
                     default: float = 16.0) -> float:
    """Smallest measured size (MB) whose bandwidth is >= ``frac`` x the best, capped at
    ``model_mb / min_buckets`` (and at least the smallest measured size). ``table``: {MB: GB/s};
    entries that are not positive numbers (failed probes) are ignored; an empty table -> ``default``."""
    pts = sorted((float(k), float(v)) for k, v in table.items()
                 if isinstance(v, (int, float)) and v == v and v > 0)
    if not pts:
        return float(default)
    best = max(v for _, v in pts)
    knee = next(s for s, v in pts if v >= frac * best)
    cap = max(model_mb / max(min_buckets, 1), pts[0][0])
    return float(min(knee, cap))


def probe_p2p(dev: torch.device, sizes_mb=(1, 2, 4, 8, 16, 32, 64), iters: int = 5) -> dict:
    """Per-link bandwidth (GB/s) vs message size on the current process group: every rank sends
    to rank+1 and receives from rank-1 at once (one xGMI link per transfer, all links busy, as in
    the push of one bucket to one owner); the max over ranks of the time. {MB: GB/s} on every
    rank. Collective; needs world >= 2."""
    rank, world = dist.get_rank(), dist.get_world_size()
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    out = {}
    for mb in sizes_mb:
        n = int(mb * (1 << 20)) // 2
        a = torch.ones(n, dtype=torch.bfloat16, device=dev)
        b = torch.empty_like(a)

        def step():
            ops = [dist.P2POp(dist.isend, a, nxt), dist.P2POp(dist.irecv, b, prv)]
            for r in dist.batch_isend_irecv(ops):
                r.wait()

        step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(iters):
            step()
        torch.cuda.synchronize(dev)
        el = torch.tensor([(time.perf_counter() - t0) / iters], device=dev, dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        out[mb] = float(f"{n * 2 / float(el.item()) / 1e9:.3g}")  # (3 significant digits: a slow gloo link is not 0)
        del a, b
    return out
