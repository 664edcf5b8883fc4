#!/usr/bin/env python3
"""Headline benchmark: whole-node samples/s of ResNet-50 bf16 training under the MI355X-native
parameter-server data plane, with gradient-staleness p50 and histogram (BASELINE.json).

  python bench.py [--gpus N] [--steps K] [--warmup W]                   (N=1: plain process)
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Config (BASELINE.json config 3): ResNet-50, bf16, NHWC, synthetic ImageNet-shaped data (224x224,
1000 classes), random init; every GPU is a worker; PS shards (default 2, capped at N) colocated on
evenly spaced ranks hold the fp32 masters + momentum in HBM. Default ``--ps-mode async``: each
worker DMA-copies its gradient buckets over xGMI into its inbox on the owning GPUs while backward
runs; the owner applies every push on arrival with the fused gfx950 SGD-momentum kernel and
publishes a new bf16 snapshot; a worker pulls the latest snapshots at the start of a step and
blocks only if it would lead the slowest worker by more than S steps (SSP, default S = 1). The
staleness histogram counts, per apply, the updates the shard took between the snapshot the
gradient was computed on and the apply. ``--ps-mode collective`` is the lock-step RCCL
reduce-scatter / all-gather plane (fixed S-step gradient delay; hipGraph replay at N = 1).

Timing: W untimed warmup steps (include MIOpen tuning and hipGraph capture), then exactly K timed
steps bracketed by barrier + device synchronize on both sides; the max over ranks is reported.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
from parameter_server_distributed_amd.utils import miopen as _miopen  # noqa: E402

from parameter_server_distributed_amd.utils import tunableop as _tunableop  # noqa: E402

_miopen.install()  # shipped gfx950 find-db + kernel cache (before torch initialises MIOpen)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from parameter_server_distributed_amd import models  # noqa: E402
from parameter_server_distributed_amd.ops.optim import OptimConfig  # noqa: E402
from parameter_server_distributed_amd.parallel.collective_ps import CollectivePS  # noqa: E402
from parameter_server_distributed_amd.parallel.transport import make_transport  # noqa: E402
from parameter_server_distributed_amd.runtime.trainer import Trainer  # noqa: E402
from parameter_server_distributed_amd.utils.config import FEATURES, feature, features  # noqa: E402

METRICS = {
    "resnet50": ("samples/sec (whole node) ResNet-50 async-SGD", "samples/s"),
    "bert_base": ("sequences/sec (whole node) BERT-base Adam", "sequences/s"),
    "wide_resnet101_2": ("samples/sec (whole node) Wide-ResNet-101-2 fp8-weights", "samples/s"),
    "resnet101": ("samples/sec (whole node) ResNet-101", "samples/s"),
    "mlp": ("samples/sec (whole node) 2-layer MLP", "samples/s"),
}
# Reference-semantics baseline (tools/reference_baseline.py, measured on 1x MI355X: the same worker
# model on the GPU, gRPC `repeated float` fp32 tensors, one host-memory PS, sync barrier, p -= g),
# samples/s per worker GPU. vs_baseline divides by this x n_workers, i.e. it credits the reference
# with perfect scaling (its single PS would in fact serialize N workers).
REF_BASELINE = {"resnet50": 285.119}
DEFAULT_BATCH = {"resnet50": 1024, "bert_base": 256, "wide_resnet101_2": 512, "resnet101": 256, "mlp": 4096}


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (0: model default)")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--seq-len", type=int, default=128)
    ap.add_argument("--ps-shards", type=int, default=2)
    ap.add_argument("--placement", default="colocated", choices=["colocated", "disjoint"],
                    help="disjoint: first half of the ranks are workers, second half PS shards")
    ap.add_argument("--staleness", type=int, default=1)
    ap.add_argument("--ps-mode", default="async", choices=["async", "collective"],
                    help="async: apply-on-arrival PS shards over xGMI peer memory with an SSP bound "
                         "(parallel/async_ps.py); collective: lock-step RCCL reduce-scatter/all-gather with a "
                         "fixed S-step gradient delay (parallel/collective_ps.py)")
    ap.add_argument("--bucket-mb", type=float, default=0.0,
                    help="push bucket size; 0 (default): at N > 1 probe the bandwidth vs size of the transport the "
                         "chosen plane pushes with (async: the engine's peer DMA into the owners' inboxes; "
                         "collective: RCCL send/recv) before the timed steps and take the knee "
                         "(parallel/bucketing.py), 16 MB at N = 1")
    ap.add_argument("--fp8-compute", type=int, default=-1,
                    help="fp8 (e4m3 MFMA) forward of the bottleneck convolutions, bf16 backward "
                         "(1/0; -1: on for Wide-ResNet-101-2, the BASELINE 'CDNA4 fp8 MFMA' config)")
    ap.add_argument("--pull-dtype", default="", help="bf16|fp8 published-weight dtype (default: fp8 for WRN-101)")
    ap.add_argument("--async-xfer", default="auto", choices=["auto", "kernel", "copy"],
                    help="async plane push / pull transport: scatter / gather kernels over every owner's peer memory "
                         "(auto: the kernels, copies if their self-test fails) or one hipMemcpyAsync per shard")
    ap.add_argument("--optimizer", default="", help="momentum|adam|adamw (default: momentum; adamw for BERT)")
    ap.add_argument("--lr", type=float, default=0.0)
    ap.add_argument("--graph", type=int, default=-1,
                    help="hipGraph capture of the whole step (1/0; -1: whenever the data plane is capturable: "
                         "the collective plane on the native RCCL transport or at N = 1; never the async engine)")
    ap.add_argument("--transport", default="auto", choices=["auto", "torch", "rccl"])
    # MIOpen immediate mode by default: solutions come from the shipped find-db / heuristics with no
    # per-shape Find (warmup ~1 s instead of ~2-4 min per rank; measured 1-2 % slower steps)
    ap.add_argument("--benchmark-miopen", type=int, default=0, help="torch.backends.cudnn.benchmark (MIOpen Find)")
    ap.add_argument("--tunableop", default="auto", choices=["auto", "off", "tune"],
                    help="library GEMM solution choice: shipped TunableOp results (auto), heuristic (off), "
                         "or time every hipBLASLt/rocBLAS solution per shape (tune; see --tunableop-out)")
    ap.add_argument("--tunableop-out", default="", help="tune mode: write the TunableOp results here")
    ap.add_argument("--out", default="", help="also write the JSON line to this file")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1: nccl (= RCCL, the data plane) or gloo (rehearsal of the "
                         "multi-rank flow with several ranks sharing one GPU; not a performance path)")
    ap.add_argument("--trace", default="", help="per-step phase trace (JSON lines, one file per rank); eager")
    ap.add_argument("--push-mode", default="reduce", choices=["auto", "reduce", "p2p"],
                    help="push/pull when PS shards < ranks: RCCL reduce/broadcast per slice (default) or "
                         "grouped send/recv into per-worker inboxes (p2p)")
    ap.add_argument("--ckpt-prefix", default="", help="sharded PS checkpoint path prefix")
    ap.add_argument("--ckpt-every", type=int, default=0, help="checkpoint every N steps (async, off the step)")
    ap.add_argument("--resume", default="", help="load PS shards from this checkpoint prefix before training")
    ap.add_argument("--comm-probe", type=int, default=1,
                    help="N > 1 with RCCL: after the timed steps, measure all-reduce / reduce-scatter / all-gather "
                         "bus bandwidth vs bucket size over xGMI and report it (comm_probe in the JSON)")
    ap.add_argument("--features", default="",
                    help="kernel-path / engine feature overrides for this run, e.g. 'async_direct_pull=0,convn=1' "
                         "(utils/config.py FEATURES; same syntax as PSD_FEATURES, which it replaces)")
    from parameter_server_distributed_amd.utils.config import apply_config

    apply_config(ap)
    ap.add_argument("--step-log", action="store_true",
                    help="diagnosis: print the host time of every timed step and of its begin / forward / backward "
                         "/ finish phases (stderr)")
    ap.add_argument("--prof-window", action="store_true",
                    help="under rocprofv3 --selected-regions: trace / count only the timed steps (roctx resume "
                         "before the timed loop, pause after it; utils/roctx.py)")
    ap.add_argument("--autotune-log", action="store_true",
                    help="print every autotune decision with its candidates' timings (ops/autotune.py)")
    a = ap.parse_args()
    if a.step_log:
        os.environ["PSD_STEP_LOG"] = "1"
    if a.autotune_log:
        os.environ["PSD_AUTOTUNE_LOG"] = "1"
    if a.features:  # before any kernel path or the native engine reads the registry
        os.environ["PSD_FEATURES"] = a.features
    return a


def comm_probe(dev, world: int, sizes_mb=(1, 4, 16, 64, 256), iters: int = 5) -> dict:
    """RCCL bus bandwidth (GB/s, NCCL-tests convention) per collective and bucket size on this node
    -- the measurement behind the bucket-size choice for 7 xGMI links per GPU.
    Runs outside the timed region, on the already-initialised process group."""
    out = {}
    for mb in sizes_mb:
        n = (mb << 20) // 2 // world * world  # bf16 elements, divisible by the world size
        x = torch.ones(n, dtype=torch.bfloat16, device=dev)
        part = torch.empty(n // world, dtype=torch.bfloat16, device=dev)
        res = {}
        for name, fn, factor in (
                ("all_reduce", lambda: dist.all_reduce(x), 2.0 * (world - 1) / world),
                ("reduce_scatter", lambda: dist.reduce_scatter_tensor(part, x), (world - 1) / world),
                ("all_gather", lambda: dist.all_gather_into_tensor(x, part), (world - 1) / world)):
            for _ in range(2):
                fn()
            torch.cuda.synchronize(dev)
            dist.barrier(device_ids=[dev.index])
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            torch.cuda.synchronize(dev)
            el = (time.perf_counter() - t0) / iters
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            res[name] = round(n * 2 * factor / float(t.item()) / 1e9, 1)
        out[f"{mb}MB"] = res
        del x, part
    return out


def autotune_summary() -> dict:
    """{op/kind: {choice: count}} of the per-shape kernel choices (ops/autotune.py) and the
    candidates rejected for wrong output."""
    from parameter_server_distributed_amd.ops import autotune

    out: dict = {}
    for key, how in autotune.decisions().items():
        k = f"{key[0]}/{key[1]}" if len(key) > 1 else str(key[0])
        out.setdefault(k, {}).setdefault(how, 0)
        out[k][how] += 1
    rej = autotune.rejected()
    if rej:
        out["rejected"] = {"/".join(map(str, k[:2])): v for k, v in rej.items()}
    return out


def _autotune_source() -> dict:
    """Per-rank decision sources (ops/autotune.py source()), summed over ranks: at N > 1 every
    shape is timed by exactly one rank ("claimed") and taken by the others ("peer")."""
    from parameter_server_distributed_amd.ops import autotune

    src = autotune.source()
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([src[k] for k in sorted(src)], dtype=torch.float64)
        if dist.get_backend() == "nccl":
            t = t.cuda()
        dist.all_reduce(t)
        src = {k: int(v) for k, v in zip(sorted(src), t.tolist())}
    return src


def main():
    a = parse()
    if a.prof_window:  # (--selected-regions starts paused: a pause before the first resume aborts it)
        from parameter_server_distributed_amd.utils import roctx
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and rank == 0:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (MI355X); CPU plumbing runs live in tests/ and scripts/test_local.sh")
    ndev = torch.cuda.device_count()
    if a.backend == "nccl" and world > 1 and local >= ndev:
        raise SystemExit(f"LOCAL_RANK {local} but only {ndev} visible GPU(s): RCCL needs one GPU per rank")
    dev = torch.device("cuda", local % ndev)  # gloo rehearsal: ranks may share a GPU
    torch.cuda.set_device(dev)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    torch.backends.cudnn.benchmark = bool(a.benchmark_miopen)
    tunable_mode = _tunableop.install(a.tunableop)
    torch.manual_seed(1234)  # identical init on every rank; the PS init pull makes it exact

    a.model = a.model.lower().replace("-", "_")
    a.batch = a.batch or DEFAULT_BATCH.get(a.model, 64)
    fp8_compute = a.fp8_compute == 1 or (a.fp8_compute < 0 and a.model.startswith("wide"))
    spec = models.build(a.model, dev, torch.bfloat16, image_size=a.image_size, seq_len=a.seq_len, fp8=fp8_compute)
    opt_kind = a.optimizer or ("adamw" if a.model.startswith("bert") else "momentum")
    lr = a.lr or (1e-4 if opt_kind.startswith("adam") else 0.1)
    optim = OptimConfig(opt_kind, lr=lr, momentum=0.9, weight_decay=0.01 if opt_kind == "adamw" else 5e-5)
    kw = {}
    if a.placement == "disjoint" and world >= 2:
        kw = dict(worker_ranks=list(range(world // 2)), ps_ranks=list(range(world // 2, world)))
        shards = world - world // 2
    else:
        shards = max(1, min(a.ps_shards, world))
    bucket_probe = None
    bucket_transport = None
    auto_bucket = a.bucket_mb <= 0
    if auto_bucket:
        a.bucket_mb = 16.0
    model_mb = sum(p.numel() for p in spec.model.parameters()) * 2 / 2**20
    pull_dtype = a.pull_dtype or ("fp8" if a.model.startswith("wide") else "bf16")
    mode = a.ps_mode  # both planes publish MX e4m3 weights for the fp8 config
    fallback = None
    if mode == "async":
        from parameter_server_distributed_amd.parallel.async_ps import AsyncPS

        try:
            ps = AsyncPS(spec.model, optim, num_shards=shards, staleness=a.staleness, bucket_mb=a.bucket_mb,
                         device=dev, overlap=not spec.tied_weights, pull_dtype=pull_dtype, xfer=a.async_xfer, **kw)
        except RuntimeError as e:  # collective on every rank (AsyncPS._agree): fall back together
            fallback = str(e)[:300]
            mode = "collective"
            if rank == 0:
                print(f"WARNING: async peer-memory plane unavailable ({fallback}); using the collective plane",
                      file=sys.stderr, flush=True)
            torch.manual_seed(1234)
            spec = models.build(a.model, dev, torch.bfloat16, image_size=a.image_size, seq_len=a.seq_len,
                                fp8=fp8_compute)
    if mode == "async" and auto_bucket and world > 1:
        # bucket size from the transport this plane pushes with (engine DMA into the owners'
        # inboxes, alternating push streams), probed before the timed steps (parallel/bucketing.py)
        from parameter_server_distributed_amd.parallel import bucketing

        try:
            bucket_probe = ps.probe_push_sizes()
            bucket_transport = f"async engine push into the owners' IPC inboxes ({ps.xfer_mode})"
            a.bucket_mb = bucketing.choose_bucket_mb(bucket_probe, model_mb)
            ps.rebucket(a.bucket_mb)
        except Exception as e:  # noqa: BLE001 -- collective (every rank raises together): keep 16 MB
            bucket_probe = {"error": str(e)[:200]}
    xfer_probe = None
    if mode == "async" and world > 1:
        # the scatter kernel's workgroup budget per owner segment: the smallest that keeps ~all of the
        # link bandwidth (fewest CUs taken from the backward pass the pushes run beside)
        try:
            xfer_probe = ps.probe_xfer_blocks() or None
        except Exception as e:  # noqa: BLE001 -- collective: every rank raises together; keep the default
            xfer_probe = {"error": str(e)[:200]}
    if mode == "collective" and auto_bucket and world > 1 and a.backend == "nccl":
        from parameter_server_distributed_amd.parallel import bucketing

        try:  # the collective plane's transport: RCCL point-to-point over xGMI
            bucket_probe = bucketing.probe_p2p(dev)
            bucket_transport = "RCCL send/recv"
            a.bucket_mb = bucketing.choose_bucket_mb(bucket_probe, model_mb)
        except Exception as e:  # noqa: BLE001
            bucket_probe = {"error": str(e)[:200]}
    if mode == "collective":
        transport = make_transport(a.transport, dev)
        ps = CollectivePS(spec.model, optim, transport, num_shards=shards, staleness=a.staleness,
                          bucket_mb=a.bucket_mb, device=dev, overlap=not spec.tied_weights, pull_dtype=pull_dtype,
                          push_mode=a.push_mode, **kw)
    n_workers = len(ps.worker_ranks)
    batch = spec.make_batch(a.batch, dev, seed=rank)
    use_graph = a.graph != 0  # the Trainer keeps eager steps unless ps.t is capturable
    tracer = None
    if a.trace:
        from parameter_server_distributed_amd.utils.trace import StepTracer, rank_path

        tracer = StepTracer(rank_path(a.trace, rank), rank, dev)
    if a.resume:
        ps.load(a.resume)
    tr = Trainer(spec.model, spec.loss, ps, batch, use_graph=use_graph, tracer=tracer,
                 checkpoint_prefix=a.ckpt_prefix or None, checkpoint_every=a.ckpt_every)

    def barrier():
        if world > 1:
            if a.backend == "nccl":
                dist.barrier(device_ids=[dev.index])
            else:
                dist.barrier()
        torch.cuda.synchronize(dev)

    t_w0 = time.perf_counter()
    warm_done = threading.Event()

    def heartbeat():  # a first step that autotunes many unseen shapes can run for minutes
        while not warm_done.wait(30.0):
            print(f"  ... warmup running, {time.perf_counter() - t_w0:.0f} s", file=sys.stderr, flush=True)

    if rank == 0:
        threading.Thread(target=heartbeat, daemon=True).start()
    for i in range(a.warmup):
        tr.step()
        if rank == 0:  # progress (MIOpen tuning of unseen shapes can take minutes)
            torch.cuda.synchronize(dev)
            print(f"warmup step {i + 1}/{a.warmup}: {time.perf_counter() - t_w0:.1f} s", file=sys.stderr, flush=True)
    warm_done.set()
    barrier()
    t_w = time.perf_counter() - t_w0
    mem_peak = torch.cuda.max_memory_allocated(dev)

    barrier()
    step_log = os.environ.get("PSD_STEP_LOG", "0") == "1"  # host time of each step() call (diagnosis)
    ts = []
    gc_log = []  # (generation, seconds) of every Python GC pass in the timed steps (step-log diagnosis)
    if step_log:
        import gc

        def _gc_cb(phase, info, _t=[0.0]):
            if phase == "start":
                _t[0] = time.perf_counter()
            else:
                gc_log.append((info.get("generation"), time.perf_counter() - _t[0]))

        gc.callbacks.append(_gc_cb)
    if a.prof_window:
        roctx.resume()
    t0 = time.perf_counter()
    c0 = time.thread_time()  # this (launching) thread's CPU time: how close the step is to host-bound
    loss = None
    for _ in range(a.steps):
        loss = tr.step()
        if step_log:
            ts.append(time.perf_counter())
    host_cpu_ms = (time.thread_time() - c0) / max(a.steps, 1) * 1e3
    torch.cuda.synchronize(dev)
    barrier()
    if a.prof_window:
        roctx.pause()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ms = el / max(a.steps, 1) * 1e3
    if step_log and rank == 0:
        prev = t0
        print("step host ms: " + " ".join(f"{(t - p) * 1e3:.1f}" for p, t in zip([t0] + ts[:-1], ts)), file=sys.stderr)
        bnd = [e0.elapsed_time(e1) for e0, e1 in getattr(tr, "boundary_evs", [])[-a.steps:] if e0 is not None]
        if bnd:
            print("GPU ms from each step's end to the next forward (begin_step on the compute stream): " +
                  " ".join(f"{x:.3f}" for x in bnd), file=sys.stderr)
        print(f"python gc in the timed steps: {len(gc_log)} passes, {sum(d for _, d in gc_log) * 1e3:.2f} ms, "
              f"by generation {[sum(1 for g, _ in gc_log if g == k) for k in range(3)]}, "
              f"longest {max((d for _, d in gc_log), default=0) * 1e3:.2f} ms", file=sys.stderr)
        for ph in (getattr(tr, "host_phases", None) or [])[-a.steps:]:
            print("host phases ms (begin forward backward finish) + GPU drained before / after begin: " +
                  " ".join(f"{x * 1e3:.2f}" for x in ph[:4]) + f" {ph[4]} {ph[5]}", file=sys.stderr)
    if mode == "async":
        ps.drain()  # outside the timed region: every push of the run applied before reporting
    samples = a.batch * n_workers * a.steps
    value = samples / el
    hist = ps.staleness_histogram()
    if world > 1:
        h = torch.tensor(hist, device=dev, dtype=torch.int64)
        dist.all_reduce(h)
        hist = h.tolist()
    tot = sum(hist)
    p50, acc = -1, 0
    for i, c in enumerate(hist):
        acc += c
        if tot and acc * 2 >= tot:
            p50 = i
            break
    while hist and hist[-1] == 0 and len(hist) > 1:
        hist.pop()
    probe = None
    async_bw = None
    if mode == "async" and a.comm_probe:
        try:
            async_bw = ps.probe_bandwidth()
        except Exception as e:  # noqa: BLE001
            async_bw = {"error": str(e)[:200]}
    if world > 1 and a.backend == "nccl" and a.comm_probe:
        try:
            probe = comm_probe(dev, world)
        except Exception as e:  # noqa: BLE001 -- a diagnostic must not cost the measurement
            probe = {"error": str(e)[:200]}
    final_loss = float(loss.float().item()) if loss is not None else float("nan")
    # health of the run: a silent NaN in the weights invalidates a throughput number (round-1 lesson:
    # a bad library GEMM produced NaN weights that a ReLU hid behind a finite loss)
    finite = torch.tensor([float(bool(torch.isfinite(ps.params_flat).all())) and float(final_loss == final_loss)],
                          device=dev)
    if world > 1:
        dist.all_reduce(finite, op=dist.ReduceOp.MIN)
    params_finite = bool(finite.item() > 0)
    at_src = _autotune_source()  # (a collective at N > 1: every rank)
    if rank == 0 and os.environ.get("PSD_AUTOTUNE_SAVE"):  # pin these choices in later runs (PSD_AUTOTUNE_FILE)
        from parameter_server_distributed_amd.ops import autotune as _at_mod

        _at_mod.save_decisions(os.environ["PSD_AUTOTUNE_SAVE"])
    if not params_finite and rank == 0:
        print("WARNING: non-finite weights or loss at the end of the timed steps", file=sys.stderr, flush=True)
    if rank == 0:
        metric, unit = METRICS.get(a.model, (f"samples/sec (whole node) {a.model}", "samples/s"))
        data = ("synthetic (random token ids, 15% MLM labels, random init)" if a.model.startswith("bert") else
                "synthetic (random ImageNet-shaped 224x224, random init)")
        rec = {
            "metric": metric, "value": round(value, 2), "unit": unit, "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": (round(value / (REF_BASELINE[a.model] * n_workers), 2)
                            if a.model in REF_BASELINE else None),
            "dtype": (("fp8 convs (MX e4m3 fwd, MX e5m2-dY bwd-data), bf16 rest" if feature("fp8_mx")
                       else "fp8-e4m3 fwd convs / bf16") if fp8_compute else "bf16"), "data": data,
            "config": {"model": a.model, "global_batch": a.batch * n_workers, "per_gpu_batch": a.batch,
                       "seq_len": a.seq_len if a.model.startswith("bert") else None,
                       "image_size": None if a.model.startswith("bert") else a.image_size,
                       "parallelism": (f"ps{shards}-async-ssp{a.staleness}-dp{n_workers}" if mode == "async" else
                                       f"ps{shards}-{'delayed' if a.staleness else 'sync'}-s{a.staleness}-dp{n_workers}")
                                      + ("-disjoint" if kw else ""),
                       "ps_mode": mode, "async_fallback": fallback,
                       "async_xfer": getattr(ps, "xfer_mode", None),
                       "features_changed": {k: v for k, v in features().items() if v != FEATURES[k][0]},
                       "async_xfer_fallback": getattr(ps, "xfer_fallback", None),
                       "ps_shards": shards, "ps_owner_ranks": ps.owners, "worker_ranks": ps.worker_ranks,
                       "staleness_bound": a.staleness, "optimizer": f"{opt_kind} fused gfx950", "bucket_mb": a.bucket_mb,
                       "pull_dtype": pull_dtype, "fp8_compute": fp8_compute, "tunableop": tunable_mode,
                       "transport": ps.t.name, "hipgraph": bool(tr.graphs), "graph_error": tr.graph_error},
            "ps_semantics": ((f"K-batch async SGD, K={ps.round} pushes per step (staleness bound {a.staleness}: "
                              f"gradients may be up to {a.staleness + 1} steps stale)" if a.staleness else
                              f"K-batch SGD at staleness bound 0, K={ps.round} pushes per step: exactly synchronous "
                              "(every gradient is applied to the weights it was computed on)")
                             if mode == "async" else
                             (f"synchronous, fixed {a.staleness}-step gradient delay" if a.staleness else "synchronous")),
            "vs_baseline_note": ("vs the reference-semantics baseline (sync barrier, gRPC fp32 tensors, one host PS, "
                                 "285.1 img/s x workers, tools/reference_baseline.py); "
                                 + (f"this run's weights may be up to {a.staleness + 1} steps stale (SSP bound "
                                    f"{a.staleness})" if a.staleness else "this run is synchronous (SSP bound 0)")
                                 if a.model in REF_BASELINE else None),
            "bucket_mb_chosen": a.bucket_mb, "bucket_probe_GBps": bucket_probe,
            "bucket_probe_transport": bucket_transport,
            "async_xfer_blocks": xfer_probe,
            "staleness_p50": p50, "staleness_hist": hist, "final_loss": round(final_loss, 4),
            "params_finite": params_finite, "comm_probe_busbw_GBps": probe, "async_plane_bw": async_bw,
            "warmup_s": round(t_w, 2), "peak_mem_gb": round(mem_peak / 2**30, 2),
            "host_cpu_ms_per_step": round(host_cpu_ms, 2),  # rank 0 launching thread (CPU time, not wall)
            "autotune": autotune_summary(),
            "autotune_source": at_src,
        }
        line = json.dumps(rec)
        print(line, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(line + "\n")
    if tunable_mode == "tune" and a.tunableop_out:
        _tunableop.dump(a.tunableop_out if world == 1 else f"{a.tunableop_out}.{rank}")
    if tracer is not None:
        tracer.close()
    if mode == "async":
        ps.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
