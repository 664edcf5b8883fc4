#!/usr/bin/env python3
"""Multi-rank data-plane consistency check (diagnostic for the overlapped GPU push/apply/pull).

Runs the bench step (ResNet-50 or MLP through ``CollectivePS`` + ``Trainer``) and after every step
compares, across ranks, a bit-exact fingerprint of the published bf16 working weights
(``params_flat``): after a pull every rank must hold the same bytes. It also records each rank's
loss, the fp32 master fingerprint of the owned slices, and the norm of the gradient slot that
the step applied, so a divergence can be placed at its first step and phase.

  torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/rank_check.py --backend gloo --steps 8

Rank 0 prints one JSON line per step and a final summary line {"consistent": bool, ...}.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

from parameter_server_distributed_amd.utils import miopen as _miopen  # noqa: E402

_miopen.install()

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from parameter_server_distributed_amd import models  # noqa: E402
from parameter_server_distributed_amd.ops.optim import OptimConfig  # noqa: E402
from parameter_server_distributed_amd.parallel.collective_ps import CollectivePS  # noqa: E402
from parameter_server_distributed_amd.parallel.transport import make_transport  # noqa: E402
from parameter_server_distributed_amd.runtime.trainer import Trainer  # noqa: E402
from parameter_server_distributed_amd.utils import tunableop as _tunableop  # noqa: E402


def fingerprint(t: torch.Tensor) -> list[int]:
    """Bit-exact fingerprint of a flat tensor: (sum of raw words, position-weighted sum)."""
    w = t.view(torch.int16 if t.element_size() == 2 else torch.int32).to(torch.int64)
    pos = torch.arange(w.numel(), device=w.device, dtype=torch.int64) % 1009 + 1
    return [int(w.sum().item()), int((w * pos).sum().item())]


def _where(ps, flat_idx: torch.Tensor) -> dict:
    """Map flat element offsets to parameter names (or 'pad') with counts."""
    out: dict = {}
    spans = sorted((o, o + n, name) for b in ps.buckets for (name, _p, o, n) in b.params)
    import bisect

    starts = [s for s, _, _ in spans]
    for i in flat_idx.tolist():
        j = bisect.bisect_right(starts, i) - 1
        nm = spans[j][2] if j >= 0 and i < spans[j][1] else "pad"
        out[nm] = out.get(nm, 0) + 1
    return out


def deep_check(ps, world: int, rank: int) -> dict:
    """After a step (S >= 1, grads of this step still in grads_flat): locate non-finite local
    gradients, and compare this rank's reduced slot slices with an fp32 CPU all-reduce."""
    g = ps.grads_flat.float()
    bad_local = torch.nonzero(~torch.isfinite(g)).flatten()
    rep = {"local_nonfinite": _where(ps, bad_local[:4096]) if bad_local.numel() else {}}
    slot = ps.slots[(ps.step_idx - 1) % (ps.S + 1)].float()
    ref = g.cpu()
    if world > 1:
        dist.all_reduce(ref)
    worst, bad_slot = 0.0, []
    for b in ps.buckets:
        for j, k in enumerate(ps.my_shards):
            got = slot.narrow(0, b.local_offset + j * b.slice_numel, b.slice_numel).cpu()
            want = ref.narrow(0, b.offset + k * b.slice_numel, b.slice_numel)
            nf = torch.nonzero(~torch.isfinite(got)).flatten()
            if nf.numel():
                bad_slot.append(nf[:4096] + b.offset + k * b.slice_numel)
            fin = torch.isfinite(got) & torch.isfinite(want)
            d = (got[fin] - want[fin]).abs()
            if d.numel():
                rel = float(d.max() / (want[fin].abs().max() + 1e-12))
                worst = max(worst, rel)
    rep["slot_nonfinite"] = _where(ps, torch.cat(bad_slot)) if bad_slot else {}
    rep["slot_vs_fp32_allreduce_maxrel"] = worst
    return rep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--staleness", type=int, default=1)
    ap.add_argument("--ps-shards", type=int, default=2)
    ap.add_argument("--bucket-mb", type=float, default=16.0)
    ap.add_argument("--overlap", type=int, default=1)
    ap.add_argument("--backend", default="gloo", choices=["gloo", "nccl"])
    ap.add_argument("--transport", default="auto")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--out", default="")
    ap.add_argument("--seed", type=int, default=0, help="batch seed offset (rank + seed)")
    ap.add_argument("--deep", type=int, default=0, help="locate non-finite grads / check the reduced slot")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    _tunableop.install("auto")
    torch.manual_seed(1234)
    spec = models.build(a.model, dev, torch.bfloat16, image_size=a.image_size)
    ps = CollectivePS(spec.model, OptimConfig("momentum", lr=a.lr, momentum=0.9, weight_decay=5e-5),
                      make_transport(a.transport, dev), num_shards=max(1, min(a.ps_shards, world)),
                      staleness=a.staleness, bucket_mb=a.bucket_mb, device=dev, overlap=bool(a.overlap))
    tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(a.batch, dev, seed=rank + a.seed), use_graph=False)
    ok = True
    first_bad = None
    rows = []
    for step in range(a.steps):
        loss = tr.step()
        torch.cuda.synchronize(dev)
        slot_norm = None
        if ps.S > 0 and step >= ps.S:
            slot_norm = float(ps.slots[(ps.step_idx - 1 - ps.S) % (ps.S + 1)].float().norm().item())
        mine = {"rank": rank, "loss": float(loss.float().item()), "params": fingerprint(ps.params_flat),
                "master": fingerprint(ps.master), "slot_norm": slot_norm}
        if a.deep and ps.S > 0:
            mine["deep"] = deep_check(ps, world, rank)
            pf = ps.params_flat.float()
            mine["params_nonfinite"] = _where(ps, torch.nonzero(~torch.isfinite(pf)).flatten()[:4096])
        allr = [None] * world
        if world > 1:
            dist.all_gather_object(allr, mine)
        else:
            allr = [mine]
        same = all(r["params"] == allr[0]["params"] for r in allr)
        if not same:
            ok = False
            first_bad = step if first_bad is None else first_bad
        row = {"step": step, "params_consistent": same, "loss": [r["loss"] for r in allr],
               "slot_norm": [r["slot_norm"] for r in allr], "params_fp": [r["params"] for r in allr]}
        if a.deep:
            row["deep"] = [r.get("deep") for r in allr]
            row["params_nonfinite"] = allr[0].get("params_nonfinite")
        rows.append(row)
        if rank == 0:
            print(json.dumps(row), flush=True)
    if rank == 0:
        summ = {"consistent": ok, "first_inconsistent_step": first_bad, "world": world, "model": a.model,
                "batch": a.batch, "staleness": a.staleness, "overlap": a.overlap, "backend": a.backend,
                "transport": ps.t.name, "final_loss": rows[-1]["loss"]}
        print(json.dumps(summ), flush=True)
        if a.out:
            with open(a.out, "w") as f:
                for r in rows:
                    f.write(json.dumps(r) + "\n")
                f.write(json.dumps(summ) + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
