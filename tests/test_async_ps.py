"""Asynchronous apply-on-arrival PS (parallel/async_ps.py + csrc/async_ps.cpp), multi-process on
CPU: the same engine and shared-memory protocol as on the GPUs, with host shared memory instead of
xGMI peer memory. Every run is checked against an fp32 replay of the *recorded* apply order:

  * the final fp32 master of every shard equals the replay of the logged (worker, step) pushes,
    grouped into the rounds (versions) the engine applied them in (no lost, doubled or torn update);
  * the weights a worker pulled for step t equal the replayed snapshot of the version it reported;
  * every logged staleness equals (version before the apply) - (version the gradient was computed
    on);
  * the SSP bound held at every pull: each worker's clock at each shard was >= t - S.
"""
import os
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from parameter_server_distributed_amd import models
from parameter_server_distributed_amd.ops.optim import OptimConfig
from parameter_server_distributed_amd.parallel.async_ps import AsyncPS

CFG = dict(kind="momentum", lr=0.05, momentum=0.9, weight_decay=1e-3)
CFGS = {"momentum": CFG, "adamw": dict(kind="adamw", lr=2e-3, weight_decay=0.01, beta1=0.9, beta2=0.999, eps=1e-8)}


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, shards, stale, steps, out_dir, slow_rank, delay_s, disjoint, device="cpu",
            kind="momentum", pull="bf16", xfer="auto"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    dt = torch.bfloat16 if dev.type == "cuda" else torch.float32
    spec = models.build("mlp", dev, dt, hidden=64)
    kw = {}
    if disjoint:
        kw = dict(worker_ranks=list(range(world // 2)), ps_ranks=list(range(world // 2, world)))
    ps = AsyncPS(spec.model, OptimConfig(**CFGS[kind]), num_shards=shards, staleness=stale, bucket_mb=0.0005,
                 param_dtype=dt, log=True, device=dev, pull_dtype=pull, xfer=xfer, **kw)
    init_master = {k: v.cpu().clone() for k, v in ps.master.items()}
    x, y = spec.make_batch(16, dev, seed=rank)
    rec = []
    if ps.is_worker:
        for t in range(steps):
            if rank == slow_rank:
                time.sleep(delay_s)
            ps.begin_step()
            clocks = [min(ps.engine.clocks(k)) for k in range(ps.P)]
            spec.loss(spec.model(x), y).backward()
            ps.finish_step()
            if dev.type == "cuda":
                torch.cuda.synchronize()
            g = ps.grads[(ps.step_idx - 1) % 2].float().cpu().clone()
            rec.append({"step": t, "pulled": list(ps.pulled), "clock_min": clocks, "grad": g,
                        "weights": ps.params_flat.float().cpu().clone()})
    ps.drain()
    torch.save({"rank": rank, "rec": rec, "log": ps.apply_log(), "init": init_master,
                "master": {k: v.cpu() for k, v in ps.master.items()}, "mem": ps.engine.memory_kind(),
                "hist": ps.staleness_histogram(), "shard_off": ps.shard_off, "shard_len": ps.shard_len,
                "workers": ps.worker_ranks, "owners": ps.owners, "xfer": ps.xfer_mode,
                "xfer_fallback": ps.xfer_fallback},
               os.path.join(out_dir, f"r{rank}.pt"))
    ps.close()
    dist.barrier()
    dist.destroy_process_group()


def _replay_opt(kind, p, g, st, step):
    """One fp32 step of the fused apply kernel's math (kernels/optim.hip opt_update) on a shard."""
    c = CFGS[kind]
    if kind == "momentum":
        g = g + c["weight_decay"] * p
        st["buf"] = g.clone() if "buf" not in st else c["momentum"] * st["buf"] + g
        return p - c["lr"] * st["buf"]
    p = p * (1.0 - c["lr"] * c["weight_decay"])
    st["m"] = c["beta1"] * st.get("m", torch.zeros_like(p)) + (1 - c["beta1"]) * g
    st["v"] = c["beta2"] * st.get("v", torch.zeros_like(p)) + (1 - c["beta2"]) * g * g
    bc1, bc2 = 1 - c["beta1"] ** step, 1 - c["beta2"] ** step
    return p - (c["lr"] / bc1) * (st["m"] / (st["v"].sqrt() / bc2 ** 0.5 + c["eps"]))


def _mx_roundtrip(x):
    from parameter_server_distributed_amd.ops import dequantize_mx_ref, quantize_mx_ref

    return dequantize_mx_ref(*quantize_mx_ref(x))


def _replay_and_check(out_dir, world, stale, bf16=False, kind="momentum", mx=False):
    R = [torch.load(os.path.join(out_dir, f"r{r}.pt"), weights_only=False) for r in range(world)]
    workers, owners = R[0]["workers"], R[0]["owners"]
    off, ln = R[0]["shard_off"], R[0]["shard_len"]
    W = len(workers)
    K = W  # "round" semantics: K = W pushes per optimizer step (grouped by 16 inside the engine)
    recs = {R[r]["rank"]: {e["step"]: e for e in R[r]["rec"]} for r in range(world)}
    hist_total = [0] * 64
    for k, o in enumerate(owners):
        log = [e for e in R[o]["log"] if e[0] == k]
        p = R[o]["init"][k].clone()
        opt_state = {}
        snaps = {0: p.clone()}
        assert len(log) % K == 0
        for i in range(len(log) // K):
            rnd = log[i * K:(i + 1) * K]
            assert all(e[4] == i + 1 for e in rnd), rnd  # one version per round of K pushes
            g = torch.zeros_like(p)
            for (_k, w, t, st, v) in rnd:
                e = recs[w][t]
                assert st == i - e["pulled"][k], (k, w, t, st, i, e["pulled"][k])
                g = g + e["grad"].narrow(0, off[k], ln[k])
                hist_total[min(st, 63)] += 1
            p = _replay_opt(kind, p, g * (1.0 / K), opt_state, i + 1)
            snaps[i + 1] = p.clone()
        assert len(log) == W * len(recs[workers[0]]), "every push applied exactly once"
        mtol = dict(rtol=1e-5, atol=1e-6) if kind == "momentum" else dict(rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(R[o]["master"][k], p, **mtol)
        for w in workers:
            for t, e in recs[w].items():
                want = snaps[e["pulled"][k]]
                tol = dict(rtol=1e-5, atol=1e-6) if kind == "momentum" else dict(rtol=1e-4, atol=1e-5)
                if mx:  # MX e4m3 publish: the worker's weights are dequant(quant_mx(master))
                    want = _mx_roundtrip(want)
                    tol = dict(rtol=2 ** -3, atol=2 ** -9 * float(want.abs().max()))
                elif bf16:  # published snapshots are bf16(master): one ulp where the replay sits on a tie
                    want = want.to(torch.bfloat16).float()
                    tol = dict(rtol=2 ** -7, atol=1e-6)
                torch.testing.assert_close(e["weights"].narrow(0, off[k], ln[k]), want, **tol)
                assert min(e["clock_min"]) >= t - stale, (w, t, e["clock_min"])
    return hist_total


@pytest.mark.slow
@pytest.mark.parametrize("world,shards,stale", [(2, 2, 0), (2, 1, 1), (3, 2, 1), (4, 4, 2)])
def test_async_matches_replay_of_apply_order(tmp_path, world, shards, stale):
    mp.spawn(_worker, args=(world, _port(), shards, stale, 5, str(tmp_path), -1, 0.0, False), nprocs=world,
             join=True)
    _replay_and_check(str(tmp_path), world, stale)


@pytest.mark.slow
def test_async_w17_round_semantics_completes(tmp_path):
    """with K = min(W, 16) a 17-worker round left one push of every step stranded and
    that worker's clock behind forever (every later pull timed out). K = W now, with the engine
    summing the inbox slots in groups of 16 into fp32 partials: 17 workers at SSP bound 0 finish
    and match the replay."""
    world = 17
    mp.spawn(_worker, args=(world, _port(), 2, 0, 3, str(tmp_path), -1, 0.0, False), nprocs=world, join=True)
    _replay_and_check(str(tmp_path), world, 0)


@pytest.mark.slow
@pytest.mark.parametrize("disjoint", [False, True], ids=["2owners_8workers", "4ps_4workers_disjoint"])
def test_async_world8_baseline_layouts(tmp_path, disjoint):
    """World 8 on the CPU plane, the BASELINE layouts the driver's 8-GPU run uses: config 3 (2 PS
    shards colocated on ranks 0 and 4, all 8 ranks workers, SSP bound 1, momentum) and config 4 (4
    PS-only ranks + 4 worker ranks, disjoint, AdamW). Replay-checked like every async run."""
    world = 8
    shards = 4 if disjoint else 2
    kind = "adamw" if disjoint else "momentum"  # config 4 runs the Adam update kernel
    mp.spawn(_worker, args=(world, _port(), shards, 1, 4, str(tmp_path), 3, 0.02, disjoint, "cpu", kind),
             nprocs=world, join=True)
    _replay_and_check(str(tmp_path), world, 1, kind=kind)


@pytest.mark.slow
def test_async_slow_worker_bounded_staleness(tmp_path):
    """One worker 20x slower: the fast ones run ahead by at most S steps (never blocked beyond
    the bound), and the staleness histogram spreads over several values."""
    world, stale, steps = 3, 1, 6
    mp.spawn(_worker, args=(world, _port(), 2, stale, steps, str(tmp_path), 2, 0.15, False), nprocs=world, join=True)
    hist = _replay_and_check(str(tmp_path), world, stale)
    assert sum(1 for c in hist if c) >= 2, hist
    assert sum(hist) == 2 * world * steps


@pytest.mark.slow
def test_async_disjoint_placement(tmp_path):
    """PS shards on ranks that do no compute (BASELINE config 4 layout in miniature)."""
    mp.spawn(_worker, args=(4, _port(), 2, 1, 4, str(tmp_path), -1, 0.0, True), nprocs=4, join=True)
    _replay_and_check(str(tmp_path), 4, 1)


def test_async_world1_sync_matches_reference():
    from test_collective_ps import _reference

    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.float32, hidden=64)
    from test_collective_ps import CFG as CCFG

    ps = AsyncPS(spec.model, OptimConfig(**CCFG), staleness=0, bucket_mb=0.0005, param_dtype=torch.float32)
    x, y = spec.make_batch(16, torch.device("cpu"), seed=0)
    for _ in range(4):
        ps.begin_step()
        spec.loss(spec.model(x), y).backward()
        ps.finish_step()
    ps.drain()
    ps.begin_step()  # pull the final version
    want = _reference(1, 0)
    for n, p in spec.model.named_parameters():
        torch.testing.assert_close(p.detach(), want[n], rtol=1e-5, atol=1e-6)
    assert ps.versions() == [4] and ps.staleness_histogram()[0] == 4
    ps.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world,stale", [(2, 1), (3, 0)])
def test_async_gpu_ipc_matches_replay(tmp_path, gpu, world, stale):
    """Several ranks on one MI355X: inbox / publish buffers in uncached device memory mapped across
    processes with hipIpcOpenMemHandle, DMA push/pull copies, applies by the fused gfx950 kernel on
    the owner's engine stream; checked against the replay of the logged apply order."""
    mp.spawn(_worker, args=(world, _port(), 2, stale, 5, str(tmp_path), world - 1, 0.05, False, "cuda:0"),
             nprocs=world, join=True)
    _replay_and_check(str(tmp_path), world, stale, bf16=True)
    r0 = torch.load(os.path.join(str(tmp_path), "r0.pt"), weights_only=False)
    assert r0["mem"] in ("uncached", "finegrained"), r0["mem"]
    assert r0["xfer"] == "kernel", r0["xfer"]


@pytest.mark.gpu
def test_async_gpu_xfer_kernel_bitwise_equals_copies(tmp_path, gpu):
    """the scatter / gather kernels (kernels/xfer.hip: every owner's slice of a
    push / pull in one launch) against the per-shard hipMemcpyAsync path -- 3 ranks on one MI355X,
    2 shards, SSP bound 0 (rounds sum in worker order: bitwise reproducible): every pulled weight,
    every pushed gradient and the final masters are bitwise equal."""
    res = {}
    for xfer in ("kernel", "copy"):
        d = tmp_path / xfer
        d.mkdir()
        mp.spawn(_worker, args=(3, _port(), 2, 0, 4, str(d), -1, 0.0, False, "cuda:0", "momentum", "bf16", xfer),
                 nprocs=3, join=True)
        _replay_and_check(str(d), 3, 0, bf16=True)
        res[xfer] = [torch.load(os.path.join(str(d), f"r{r}.pt"), weights_only=False) for r in range(3)]
    assert [r["xfer"] for r in res["kernel"]] == ["kernel"] * 3
    assert [r["xfer"] for r in res["copy"]] == ["hipMemcpyAsync"] * 3
    for a, b in zip(res["kernel"], res["copy"]):
        for k in a["master"]:
            assert torch.equal(a["master"][k], b["master"][k]), k
        for ea, eb in zip(a["rec"], b["rec"]):
            assert ea["pulled"] == eb["pulled"]
            assert torch.equal(ea["weights"], eb["weights"]) and torch.equal(ea["grad"], eb["grad"])


@pytest.mark.gpu
def test_async_gpu_kernel_selftest_failure_falls_back_on_every_rank(tmp_path, gpu, monkeypatch):
    """with xfer="auto" a failed kernel-transport self-test on ONE rank retries the
    self-test on the copy path under fresh store keys; every rank must end on hipMemcpyAsync (none
    raises, none starts on the kernel path) and the run replays exactly."""
    monkeypatch.setenv("PSD_FAULT", "selftest_fail_kernel=1")
    mp.spawn(_worker, args=(3, _port(), 2, 0, 3, str(tmp_path), -1, 0.0, False, "cuda:0", "momentum", "bf16", "auto"),
             nprocs=3, join=True)
    _replay_and_check(str(tmp_path), 3, 0, bf16=True)
    for r in range(3):
        res = torch.load(os.path.join(str(tmp_path), f"r{r}.pt"), weights_only=False)
        assert res["xfer"] == "hipMemcpyAsync", (r, res["xfer"])
        assert "injected kernel-transport" in (res["xfer_fallback"] or ""), (r, res["xfer_fallback"])


# World 8 on ONE MI355X (8 processes, real IPC mappings, the scatter / gather kernels): the BASELINE
# layouts the driver's 8-GPU run uses, replay-checked like every async run.
@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["config3_2owners_8workers_ssp1", "config4_4ps_4workers_disjoint_adamw",
                                    "config5_8shards_mx_fp8"])
def test_async_gpu_world8_baseline_layouts(tmp_path, gpu, layout):
    world = 8
    if layout.startswith("config3"):
        args, chk = (2, 1, 4, str(tmp_path), 3, 0.02, False, "cuda:0", "momentum", "bf16"), dict(bf16=True)
    elif layout.startswith("config4"):
        args, chk = (4, 1, 4, str(tmp_path), 1, 0.02, True, "cuda:0", "adamw", "bf16"), dict(bf16=True, kind="adamw")
    else:
        args, chk = (8, 1, 4, str(tmp_path), 5, 0.02, False, "cuda:0", "momentum", "fp8"), dict(mx=True)
    mp.spawn(_worker, args=(world, _port()) + args, nprocs=world, join=True)
    _replay_and_check(str(tmp_path), world, 1, **chk)
    for r in range(world):
        assert torch.load(os.path.join(str(tmp_path), f"r{r}.pt"), weights_only=False)["xfer"] == "kernel"


# ---------------------------------------------------------------------------------------------
# optimizer semantics at W > 1: the async trajectory against the synchronous one


SEM_STEPS = 30
# learning rates at which the synchronous run with gradients delayed by 0, 1 or 2 steps all train
# to 0.53-0.57 of the initial loss (at lr 0.02 / 2e-3 a fixed 1-step delay alone left the momentum
# run at 0.96 of it: no useful bar for S >= 1)
SEM_CFGS = {"momentum": dict(kind="momentum", lr=0.002, momentum=0.9),
            "adamw": dict(kind="adamw", lr=5e-4, weight_decay=0.01)}


def _sem_batches(W):
    """W batches of one learnable task (labels from a fixed random linear teacher), one per worker:
    the workers' gradients estimate the same objective, as data-parallel shards of one dataset do."""
    g = torch.Generator().manual_seed(1234)
    teacher = torch.randn(784, 10, generator=g)
    out = []
    for _ in range(W):
        x = torch.rand(64, 1, 28, 28, generator=g)
        out.append((x, (x.flatten(1) @ teacher).argmax(1)))
    return out


def _sem_loss(spec, batches):
    with torch.no_grad():
        return sum(float(spec.loss(spec.model(x), y)) for x, y in batches) / len(batches)


def _sem_sync(kind, delay=0):
    """The synchronous reference: torch.optim on the average of the W workers' gradients, each
    gradient computed on the weights of ``delay`` steps earlier (delay 0: plain synchronous SGD).
    Returns the loss after every step."""
    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.float32, hidden=64)
    c = SEM_CFGS[kind]
    ps = list(spec.model.parameters())
    if kind == "momentum":
        opt = torch.optim.SGD(ps, lr=c["lr"], momentum=c["momentum"])
    else:
        opt = torch.optim.AdamW(ps, lr=c["lr"], weight_decay=c["weight_decay"])
    batches = _sem_batches(4)
    hist = [[p.detach().clone() for p in ps]]
    losses = []
    for _ in range(SEM_STEPS):
        cur = [p.detach().clone() for p in ps]
        with torch.no_grad():
            for p, o in zip(ps, hist[max(0, len(hist) - 1 - delay)]):
                p.copy_(o)
        opt.zero_grad()
        sum(spec.loss(spec.model(x), y) for x, y in batches).div(len(batches)).backward()
        with torch.no_grad():
            for p, o in zip(ps, cur):
                p.copy_(o)
        opt.step()
        hist.append([p.detach().clone() for p in ps])
        losses.append(_sem_loss(spec, batches))
    return losses


def _sem_worker(rank, world, port, kind, semantics, stale, out_dir, schedule="free", slow_rank=-1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.float32, hidden=64)
    ps = AsyncPS(spec.model, OptimConfig(**SEM_CFGS[kind]), num_shards=2, staleness=stale, bucket_mb=0.0005,
                 param_dtype=torch.float32, semantics=semantics, schedule=schedule)
    batches = _sem_batches(world)
    x, y = batches[rank]
    pulled = []
    for t in range(SEM_STEPS):
        if rank == slow_rank and t % 3 == 0:
            time.sleep(0.02)  # uneven timing: must not change a fixed-schedule run
        ps.begin_step()
        pulled.append(list(ps.pulled))
        spec.loss(spec.model(x), y).backward()
        ps.finish_step()
    ps.drain()
    if schedule == "fixed":  # the final version (the fixed pull of step T + S)
        ps.engine.pull(SEM_STEPS + stale, ps.params_flat, 0)
    else:
        ps.engine.pull(0, ps.params_flat, 0)  # the final version (no SSP wait: everything is applied)
    if rank == 0:
        with open(os.path.join(out_dir, "loss.txt"), "w") as f:
            f.write(repr(_sem_loss(spec, batches)))
        torch.save({"params": ps.params_flat.clone(), "pulled": pulled}, os.path.join(out_dir, "final.pt"))
    ps.close()
    dist.barrier()
    dist.destroy_process_group()


def _sem_sync_params(kind, delay):
    """Final flat parameters of the delayed synchronous reference (the AsyncPS layout order)."""
    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.float32, hidden=64)
    c = SEM_CFGS[kind]
    ps = list(spec.model.parameters())
    opt = torch.optim.SGD(ps, lr=c["lr"], momentum=c["momentum"]) if kind == "momentum" else \
        torch.optim.AdamW(ps, lr=c["lr"], weight_decay=c["weight_decay"])
    batches = _sem_batches(4)
    hist = [[p.detach().clone() for p in ps]]
    for _ in range(SEM_STEPS):
        cur = [p.detach().clone() for p in ps]
        with torch.no_grad():
            for p, o in zip(ps, hist[max(0, len(hist) - 1 - delay)]):
                p.copy_(o)
        opt.zero_grad()
        sum(spec.loss(spec.model(x), y) for x, y in batches).div(len(batches)).backward()
        with torch.no_grad():
            for p, o in zip(ps, cur):
                p.copy_(o)
        opt.step()
        hist.append([p.detach().clone() for p in ps])
    return {n: p.detach().clone() for n, p in spec.model.named_parameters()}


@pytest.mark.slow
@pytest.mark.parametrize("kind", ["momentum", "adamw"])
def test_async_fixed_schedule_is_delayed_sync_and_deterministic(tmp_path, kind):
    """the asynchronous plane at SSP bound 1 under the fixed schedule (round r =
    every worker's step-r push; the pull of step t = exactly version t - 1), with one worker
    sleeping on every third step to perturb the timing:
      * every step's pulled versions are exactly max(t - 1, 0) at both shards;
      * two runs end bitwise identical (the schedule, not the thread timing, decides everything);
      * the final weights equal synchronous SGD whose gradients are computed one step late
        (torch.optim, fp32) to 1e-4 relative, and the loss is below 0.7 of the initial one."""
    res = []
    for run in range(2):
        d = tmp_path / f"run{run}"
        d.mkdir()
        mp.spawn(_sem_worker, args=(4, _port(), kind, "round", 1, str(d), "fixed", 2), nprocs=4, join=True)
        res.append((float(open(d / "loss.txt").read()), torch.load(d / "final.pt", weights_only=True)))
    (l0, f0), (l1, f1) = res
    assert torch.equal(f0["params"], f1["params"]) and l0 == l1
    assert f0["pulled"] == [[max(t - 1, 0)] * 2 for t in range(SEM_STEPS)]
    want = _sem_sync_params(kind, 1)
    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.float32, hidden=64)
    ps = AsyncPS(spec.model, OptimConfig(**SEM_CFGS[kind]), staleness=0, bucket_mb=0.0005, param_dtype=torch.float32)
    ps.params_flat.copy_(f0["params"])
    for n, p in spec.model.named_parameters():
        assert (p.detach() - want[n]).norm() <= 1e-4 * want[n].norm() + 1e-7, n
    ps.close()
    ref = _sem_sync(kind, 1)[-1]
    assert abs(l0 - ref) <= 1e-4 * ref, (l0, ref)
    assert l0 < 0.7 * _sem_loss_init(), l0


@pytest.mark.slow
@pytest.mark.parametrize("kind", ["momentum", "adamw"])
def test_async_w4_tracks_sync_trajectory(tmp_path, kind):
    """W = 4 workers on shards of one learnable task, 2 PS shards, against synchronous SGD
    (torch.optim on the averaged gradient), free-running (arrival-order) schedule:
      * "round" semantics at SSP bound 0 reproduce the synchronous trajectory -- the rounds are
        exactly the synchronous steps, so the final loss agrees to 1e-3;
      * at bound 1 every gradient is 0-2 rounds stale, in a timing-dependent pattern. "round" and
        "push" must train (final loss < 0.7 of the initial one) and end no worse than 1.1 x the
        worst synchronous run whose gradients are delayed by a fixed 0, 1 or 2 steps. The exact S = 1
        semantics are pinned by the fixed-schedule test above."""
    sync = _sem_sync(kind)
    worst_delayed = max(_sem_sync(kind, d)[-1] for d in (0, 1, 2))
    res = {}
    for sem, stale in (("round", 0), ("round", 1), ("push", 1)):
        d = tmp_path / f"{sem}{stale}"
        d.mkdir()
        mp.spawn(_sem_worker, args=(4, _port(), kind, sem, stale, str(d)), nprocs=4, join=True)
        res[(sem, stale)] = float(open(d / "loss.txt").read())
    start = _sem_loss_init()
    ref = sync[-1]
    assert ref < 0.6 * start, (start, ref)  # the reference is actually training
    assert abs(res[("round", 0)] - ref) < 1e-3 * ref, (kind, ref, res)
    for key in (("round", 1), ("push", 1)):
        assert res[key] < 0.7 * start, (kind, start, res)
        assert res[key] < 1.1 * worst_delayed, (kind, worst_delayed, res)


def _sem_loss_init():
    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.float32, hidden=64)
    return _sem_loss(spec, _sem_batches(4))


def test_async_hyper_reduces_to_sync_at_w1(C):
    for kind in range(4):
        h = C.async_hyper(kind, 1, 0.9, 0.9, 0.999, 1e-3)
        assert h == dict(lr_factor=1.0, grad_scale=1.0, momentum=0.9, beta1=0.9, beta2=0.999, weight_decay=1e-3)
    h = C.async_hyper(1, 8, 0.9, 0.9, 0.999, 1e-3)
    assert abs(h["momentum"] ** 8 - 0.9) < 1e-12 and abs(h["grad_scale"] - 0.125) < 1e-12
    assert abs(h["lr_factor"] - (1 - 0.9 ** 0.125) / 0.1) < 1e-12
    h = C.async_hyper(3, 8, 0.9, 0.9, 0.999, 1e-2)
    assert abs(h["beta2"] ** 8 - 0.999) < 1e-12 and h["lr_factor"] == 0.125 and h["grad_scale"] == 1.0


# ---------------------------------------------------------------------------------------------
# checkpoint / resume on the async plane


def _ckpt_worker(rank, world, port, mode, prefix, out_dir, steps, stale, kind):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.float32, hidden=64)
    cfg = dict(CFG) if kind == "momentum" else dict(kind="adamw", lr=2e-3, weight_decay=0.01)
    ps = AsyncPS(spec.model, OptimConfig(**cfg), num_shards=2, staleness=stale, bucket_mb=0.0005,
                 param_dtype=torch.float32)
    from parameter_server_distributed_amd.runtime.trainer import Trainer

    tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(16, torch.device("cpu"), seed=rank),
                 checkpoint_prefix=prefix if mode == "save" else None, checkpoint_every=3 if mode == "save" else 0)
    if mode == "resume":
        ps.load(prefix)
        assert ps.step_idx == 3
    for _ in range(steps):
        tr.step()
    tr.wait_checkpoint()
    ps.drain()
    ps.refresh_weights()
    torch.save({"master": {k: v.clone() for k, v in ps.master.items()}, "versions": ps.versions(),
                "params": ps.params_flat.clone(), "step": ps.step_idx},
               os.path.join(out_dir, f"{mode}{rank}.pt"))
    ps.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize("kind", ["momentum", "adamw"])
def test_async_save_resume_exact(tmp_path, kind):
    """a 3-rank async run (2 PS shards, SSP bound 0) checkpointed by the Trainer
    every 3 steps (non-blocking writer thread) and resumed from the step-3 checkpoint in new
    processes ends bitwise equal to the uninterrupted 6-step run: masters, optimizer state and
    step scalars, shard versions and SSP clocks are restored (round sums are in worker order, so
    bound-0 runs are reproducible bit for bit)."""
    prefix = str(tmp_path / "ck")
    mp.spawn(_ckpt_worker, args=(3, _port(), "full", prefix, str(tmp_path), 6, 0, kind), nprocs=3, join=True)
    mp.spawn(_ckpt_worker, args=(3, _port(), "save", prefix, str(tmp_path), 3, 0, kind), nprocs=3, join=True)
    assert os.path.exists(prefix + ".manifest.json")
    mp.spawn(_ckpt_worker, args=(3, _port(), "resume", prefix, str(tmp_path), 3, 0, kind), nprocs=3, join=True)
    for r in range(3):
        full = torch.load(os.path.join(str(tmp_path), f"full{r}.pt"), weights_only=True)
        res = torch.load(os.path.join(str(tmp_path), f"resume{r}.pt"), weights_only=True)
        assert res["versions"] == full["versions"] == [6, 6]
        assert res["step"] == full["step"] == 6
        for k in full["master"]:
            assert torch.equal(full["master"][k], res["master"][k]), (r, k)
        assert torch.equal(full["params"], res["params"]), r


@pytest.mark.slow
def test_async_resume_rejects_other_layout(tmp_path):
    prefix = str(tmp_path / "ck")
    mp.spawn(_ckpt_worker, args=(3, _port(), "save", prefix, str(tmp_path), 3, 0, "momentum"), nprocs=3, join=True)
    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.float32, hidden=64)
    ps = AsyncPS(spec.model, OptimConfig(**CFG), staleness=0, bucket_mb=0.0005, param_dtype=torch.float32)
    with pytest.raises((ValueError, RuntimeError)):
        ps.load(prefix)
    ps.close()


def _selftest_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PSD_FAULT="selftest_fail_rank=1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    spec = models.build("mlp", torch.device("cpu"), torch.float32, hidden=64)
    try:
        AsyncPS(spec.model, OptimConfig(**CFG), num_shards=2, staleness=1, param_dtype=torch.float32)
        res = "no error"
    except RuntimeError as e:
        res = str(e)
    with open(os.path.join(out_dir, f"st{rank}.txt"), "w") as f:
        f.write(res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
def test_async_selftest_failure_is_collective(tmp_path):
    """A peer-memory self-test failure on one rank raises on every rank (bench.py then falls back to
    the collective plane on all of them together instead of hanging)."""
    mp.spawn(_selftest_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        txt = open(os.path.join(str(tmp_path), f"st{r}.txt")).read()
        assert "selftest failed" in txt and "injected" in txt, txt
