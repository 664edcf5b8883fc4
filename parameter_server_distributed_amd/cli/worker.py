"""``worker_main [coordinator] [worker_id] [iterations] [worker_addr] [worker_port] [checkpoint_path]``
-- argv-compatible with the reference's worker_main (src/worker_main.cpp:5-45), printing the same
``worker <id> iter <it> done=<bool>`` lines. A checkpoint path resumes from the checkpoint's
iteration (the reference restarted at 0, D11)."""
from __future__ import annotations

import argparse
import json
import signal
import sys
import time

from ..runtime.worker import Worker


def main(argv=None):
    ap = argparse.ArgumentParser(prog="worker_main")
    ap.add_argument("coordinator", nargs="?", default="localhost:50052")
    ap.add_argument("worker_id", nargs="?", type=int, default=0)
    ap.add_argument("iterations", nargs="?", type=int, default=1)
    ap.add_argument("worker_addr", nargs="?", default="")
    ap.add_argument("worker_port", nargs="?", type=int, default=0)
    ap.add_argument("checkpoint_path", nargs="?", default="")
    ap.add_argument("--model", default="mlp")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--mode", default="sync", choices=["sync", "async"])
    ap.add_argument("--heartbeat-s", type=float, default=5.0)
    ap.add_argument("--bf16-wire", action="store_true", help="push gradients as bf16 bytes")
    ap.add_argument("--reference-wire", action="store_true",
                    help="encode tensors as the reference did (repeated float), not bulk bytes")
    ap.add_argument("--stats-json", default="", help="write final PS stats + losses to this file")
    # elastic collective data plane (runtime/elastic.py): RCCL/gloo world rebuilt on join/leave
    ap.add_argument("--elastic", action="store_true",
                    help="train on the collective PS data plane; join/leave mid-run via the coordinator")
    ap.add_argument("--ps-shards", type=int, default=0, help="elastic: PS shards (0: one per rank)")
    ap.add_argument("--staleness", type=int, default=0, help="elastic: staleness bound S")
    ap.add_argument("--optimizer", default="momentum")
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--bucket-mb", type=float, default=16.0)
    ap.add_argument("--pull-dtype", default="bf16")
    ap.add_argument("--check-every", type=int, default=5, help="elastic: membership check period (steps)")
    ap.add_argument("--min-workers", type=int, default=1, help="elastic: workers to wait for at start")
    ap.add_argument("--elastic-ckpt-dir", default="",
                    help="elastic: shared directory for canonical checkpoints (crash recovery)")
    ap.add_argument("--elastic-ckpt-every", type=int, default=0, help="elastic: checkpoint period (steps)")
    ap.add_argument("--collective-timeout-s", type=float, default=0.0,
                    help="elastic: bound on any collective of a generation (0: the agent timeout)")
    ap.add_argument("--ps-plane", default="collective", choices=["collective", "async"],
                    help="elastic: lock-step RCCL plane, or the asynchronous peer-memory plane (K-batch rounds, SSP "
                         "bound --staleness; one node)")
    ap.add_argument("--fp8-compute", action="store_true",
                    help="fp8 (e4m3 MFMA) forward / e5m2 bwd-data of the ResNet bottleneck convolutions "
                         "(BASELINE config 5: Wide-ResNet-101-2 fp8)")
    ap.add_argument("--image-size", type=int, default=224, help="ResNet models: synthetic image size")
    from ..utils.config import apply_config

    apply_config(ap, argv)
    a = ap.parse_intermixed_args(argv)
    if a.elastic:
        return elastic_main(a)
    w = Worker(a.coordinator, a.worker_id, a.worker_addr, a.worker_port, model=a.model, batch=a.batch,
               device=a.device, heartbeat_s=a.heartbeat_s, bf16_wire=a.bf16_wire, mode=a.mode,
               raw_wire=not a.reference_wire)
    w.initialize()

    def _leave(signum, frame):  # scale_workers.sh down: deregister so the barrier shrinks at once
        print(f"worker {a.worker_id} leaving (signal {signum})", flush=True)
        w.shutdown(deregister=True)
        sys.exit(0)

    signal.signal(signal.SIGTERM, _leave)
    start = w.start_iteration
    if a.checkpoint_path:
        epoch, it = w.load_checkpoint_from_server(a.checkpoint_path)
        start = it + 1 if it > 0 else 0
        print(f"worker {a.worker_id} loaded checkpoint epoch {epoch}, resuming at iteration {start}", flush=True)
    losses, iter_s = [], []
    t0 = time.time()
    ok_all = True
    for it in range(start, start + a.iterations):
        ti = time.time()
        done, loss, r = w.run_iteration(it)
        iter_s.append(time.time() - ti)
        losses.append(loss)
        ok_all &= done
        print(f"worker {a.worker_id} iter {it} done={'true' if done else 'false'} loss={loss:.4f} "
              f"version={r.version} staleness={r.staleness}", flush=True)
    dt = time.time() - t0
    print(f"worker {a.worker_id} finished {a.iterations} iterations in {dt:.2f} s "
          f"({a.iterations / max(dt, 1e-9):.1f} it/s)", flush=True)
    if a.stats_json:
        st = w.stats()
        with open(a.stats_json, "w") as f:
            json.dump({"losses": losses, "iter_seconds": iter_s, "version": st.version,
                       "hist": list(st.staleness_histogram),
                       "counters": json.loads(st.counters_json or "{}"), "seconds": dt}, f)
    w.shutdown()
    return 0 if ok_all else 1


def build_model(a, dev, dtype):
    """The worker's model from the CLI flags (``--fp8-compute``: fp8 bottleneck convolutions)."""
    from .. import models

    kw = {}
    if a.model.lower().replace("-", "_") in ("resnet50", "resnet101", "wide_resnet101_2", "wrn101"):
        kw = dict(fp8=bool(a.fp8_compute), image_size=a.image_size)
    return models.build(a.model, dev, dtype, **kw)


def elastic_main(a) -> int:
    """Elastic worker on the collective data plane: prints the reference's per-iteration lines
    (``worker <id> iter <it> done=true``) with the generation / world it ran in."""
    import torch

    from ..ops.optim import OptimConfig
    from ..parallel.async_ps import AsyncPS
    from ..parallel.collective_ps import CollectivePS
    from ..runtime.elastic import ElasticAgent, ElasticTrainer
    from ..runtime.trainer import Trainer

    dev = torch.device("cuda", 0) if a.device == "cuda" else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    torch.manual_seed(0)
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    spec = build_model(a, dev, dtype)
    batch = spec.make_batch(a.batch, dev, seed=1000 + a.worker_id)
    optim = OptimConfig(a.optimizer, lr=a.lr, momentum=0.9)
    agent = ElasticAgent(a.coordinator, a.worker_id, heartbeat_s=min(a.heartbeat_s, 1.0))

    def make_ps(model, transport):
        shards = a.ps_shards if 0 < a.ps_shards <= transport.world else transport.world
        if a.ps_plane == "async":
            return AsyncPS(model, optim, num_shards=shards, staleness=a.staleness, bucket_mb=a.bucket_mb, device=dev,
                           overlap=not spec.tied_weights, param_dtype=dtype,
                           pull_dtype=a.pull_dtype if dev.type == "cuda" else "bf16")
        return CollectivePS(model, optim, transport, num_shards=shards, staleness=a.staleness,
                            bucket_mb=a.bucket_mb, device=dev, overlap=not spec.tied_weights,
                            grad_dtype=dtype, param_dtype=dtype, pull_dtype=a.pull_dtype)

    def make_trainer(ps):
        return Trainer(spec.model, spec.loss, ps, batch, use_graph=False)

    def on_step(step, loss, plan):
        print(f"worker {a.worker_id} iter {step - 1} done=true loss={float(loss.detach()):.4f} gen={plan.gen} "
              f"world={len(plan.members)}", flush=True)

    et = ElasticTrainer(agent, spec.model, make_ps, make_trainer, a.iterations, dev, check_every=a.check_every,
                        min_workers=a.min_workers, on_step=on_step, checkpoint_dir=a.elastic_ckpt_dir or None,
                        checkpoint_every=a.elastic_ckpt_every, collective_timeout_s=a.collective_timeout_s)
    et.install_signal_handler()
    t0 = time.time()
    res = et.run()
    dt = time.time() - t0
    if "left_at" in res:
        print(f"worker {a.worker_id} left at iteration {res['left_at']} (handed its shards over)", flush=True)
    else:
        print(f"worker {a.worker_id} finished {a.iterations} iterations ({len(res['losses'])} here) in {dt:.2f} s "
              f"after {res['resizes']} membership changes", flush=True)
        if res.get("params") is not None:  # (a joiner that arrived after the last step has none)
            csum = float(sum(p.double().sum() for p in res["params"].values()))
            print(f"worker {a.worker_id} param checksum {csum:.10e}", flush=True)
    if a.stats_json:
        out = {"history": res["history"], "losses": res["losses"], "seconds": dt,
               "left_at": res.get("left_at"), "finished_at": res.get("finished_at"),
               "staleness_hist": res.get("staleness_hist")}
        if res.get("params") is not None:
            out["param_checksum"] = float(sum(p.double().sum() for p in res["params"].values()))
        with open(a.stats_json, "w") as f:
            json.dump(out, f)
    return 0


if __name__ == "__main__":
    sys.exit(main())
