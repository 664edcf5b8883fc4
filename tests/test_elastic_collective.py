"""Elastic join/leave on the collective data plane (runtime/elastic.py): layout-independent PS
state hand-over (canonical_state / load_canonical_state), draining of in-flight bounded-staleness
gradients, and a multi-process run through deploy.sh MODE=collective + scale_workers.sh up/down
(gloo ranks on CPU; the same code builds RCCL worlds on GPUs)."""
import os
import re
import socket
import subprocess
import sys
import time

import pytest
import torch

from parameter_server_distributed_amd import models
from parameter_server_distributed_amd.ops.optim import OptimConfig
from parameter_server_distributed_amd.parallel.collective_ps import CollectivePS
from parameter_server_distributed_amd.runtime.trainer import Trainer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPU = torch.device("cpu")


def _mlp(seed=0):
    torch.manual_seed(seed)
    return models.build("mlp", CPU, torch.float32)


def _ps(spec, S, bucket_mb, opt="adam"):
    return CollectivePS(spec.model, OptimConfig(opt, lr=1e-3), staleness=S, bucket_mb=bucket_mb,
                        grad_dtype=torch.float32, param_dtype=torch.float32)


@pytest.mark.parametrize("opt", ["momentum", "adam"])
def test_canonical_state_roundtrip_across_layouts(opt):
    spec = _mlp()
    ps = _ps(spec, 1, 0.05, opt)
    tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(16, CPU))
    for _ in range(4):
        tr.step()
    ps.drain()
    sd = ps.canonical_state(root=0)
    ref = {n: p.detach().clone() for n, p in spec.model.named_parameters()}
    ps.close()
    for n, p in spec.model.named_parameters():  # close() keeps the values, detached from the buffers
        torch.testing.assert_close(p.detach(), ref[n], rtol=0, atol=0)
    with torch.no_grad():
        for p in spec.model.parameters():
            p.zero_()
    ps2 = _ps(spec, 2, 1.0, opt)  # different bucketing and staleness
    ps2.load_canonical_state(sd)
    for n, p in spec.model.named_parameters():
        torch.testing.assert_close(p.detach(), ref[n], rtol=0, atol=0)
    sd2 = ps2.canonical_state(root=0)
    for k in sd:
        torch.testing.assert_close(sd2[k], sd[k], rtol=0, atol=0)
    assert ps2.step_idx == 0 and all(float(s.abs().sum()) == 0 for s in ps2.slots)


def test_drain_applies_each_pending_gradient_once():
    """S=2: after 5 steps only 3 updates were applied; drain applies the 2 in flight."""
    spec = _mlp()
    ps = _ps(spec, 2, 0.05, "momentum")
    tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(16, CPU))
    for _ in range(5):
        tr.step()
    assert ps.dyn.step == 3
    ps.drain()
    assert ps.dyn.step == 5
    assert sum(ps.staleness_histogram()) == 5


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _read(p):
    try:
        with open(p) as f:
            return f.read()
    except FileNotFoundError:
        return ""


def _iters(txt):
    return [int(m) for m in re.findall(r"iter (\d+) done=true", txt)]


def _wait_exit(pids, timeout):
    t0 = time.time()
    while time.time() - t0 < timeout:
        alive = 0
        for p in pids:
            try:
                os.kill(p, 0)
                alive += 1
            except ProcessLookupError:
                pass
        if not alive:
            return True
        time.sleep(0.3)
    return False


@pytest.mark.slow
@pytest.mark.parametrize("plane", ["collective", "async"])
def test_collective_deploy_scale_up_down(tmp_path, plane):
    """deploy 2 elastic workers, scale up to 3 mid-run (the joiner starts at the step the world
    grew), scale down to 2 (the leaver hands its shards over); survivors run every global step
    exactly once across three generations and end with identical weights. ``async``: the same on
    the asynchronous peer-memory plane (AsyncPS canonical-state hand-over between generations)."""
    cd = str(tmp_path / "cluster")
    it = 500 if plane == "collective" else 4000  # the async plane runs ~10x more steps/s on CPU
    env = dict(os.environ, CLUSTER_DIR=cd, MODE="collective", WORKER_COUNT="2", ITERATIONS=str(it), NUM_GPUS="0",
               COORDINATOR_PORT=str(_port()), PS_PORT=str(_port()),
               WORKER_FLAGS=f"--batch 32 --lr 0.01 --staleness 1 --check-every 5 --ps-plane {plane}",
               PYTHONPATH=ROOT)
    try:
        subprocess.run(["bash", f"{ROOT}/scripts/deploy.sh"], env=env, check=True, timeout=60, capture_output=True)
        t0 = time.time()
        while max(_iters(_read(f"{cd}/worker_0.log")) or [0]) < 40 and time.time() - t0 < 90:
            time.sleep(0.2)
        r = subprocess.run(["bash", f"{ROOT}/scripts/scale_workers.sh", "up", "3"], env=env, capture_output=True,
                           text=True, timeout=60)
        assert r.returncode == 0, r.stdout + r.stderr
        t0 = time.time()
        while "world=3" not in _read(f"{cd}/worker_2.log") and time.time() - t0 < 90:
            time.sleep(0.2)
        assert "world=3" in _read(f"{cd}/worker_2.log"), _read(f"{cd}/worker_2.log")[-3000:]
        r = subprocess.run(["bash", f"{ROOT}/scripts/scale_workers.sh", "down", "2"], env=env, capture_output=True,
                           text=True, timeout=60)
        assert r.returncode == 0, r.stdout + r.stderr
        pids = [int(_read(f"{cd}/worker_{i}.pid")) for i in range(3)]
        assert _wait_exit(pids, 360)  # 4000 async steps: ~60 s idle, several times that on a loaded host
        logs = [_read(f"{cd}/worker_{i}.log") for i in range(3)]
        assert f"worker 0 finished {it} iterations" in logs[0], logs[0][-3000:]
        assert f"worker 1 finished {it} iterations" in logs[1], logs[1][-3000:]
        assert "worker 2 left at iteration" in logs[2], logs[2][-3000:]
        for i in (0, 1):
            assert _iters(logs[i]) == list(range(it)), i
            assert "world=2" in logs[i] and "world=3" in logs[i]
        j = _iters(logs[2])
        assert j and j[0] > 0 and j == list(range(j[0], j[-1] + 1))
        sums = [re.findall(r"param checksum ([-0-9.e+]+)", lg) for lg in logs[:2]]
        assert sums[0] and sums[0] == sums[1], sums
    finally:
        for name in ("worker_0", "worker_1", "worker_2", "coordinator"):
            p = _read(f"{cd}/{name}.pid").strip()
            if p:
                try:
                    os.kill(int(p), 9)
                except (ProcessLookupError, ValueError):
                    pass


@pytest.mark.gpu
def test_handover_roundtrip_gpu_bf16(gpu):
    """The hand-over path on the GPU data plane (bf16 working copy, fp32 masters in HBM, fused
    apply): drain + canonical_state on one layout, load_canonical_state on another."""
    torch.manual_seed(0)
    spec = models.build("resnet50", gpu, torch.bfloat16, image_size=32, num_classes=10)
    ps = CollectivePS(spec.model, OptimConfig("momentum", lr=0.01), staleness=1, bucket_mb=4, device=gpu)
    tr = Trainer(spec.model, spec.loss, ps, spec.make_batch(4, gpu))
    for _ in range(3):
        tr.step()
    ps.drain()
    sd = ps.canonical_state(root=0)
    ref = {n: p.detach().clone() for n, p in spec.model.named_parameters()}
    ps.close()
    ps2 = CollectivePS(spec.model, OptimConfig("momentum", lr=0.01), staleness=0, bucket_mb=16, device=gpu)
    ps2.load_canonical_state(sd)
    torch.cuda.synchronize()
    for n, p in spec.model.named_parameters():
        torch.testing.assert_close(p.detach(), ref[n], rtol=0, atol=0, msg=n)
    sd2 = ps2.canonical_state(root=0)
    for k in sd:
        torch.testing.assert_close(sd2[k], sd[k], rtol=0, atol=0)
    tr2 = Trainer(spec.model, spec.loss, ps2, spec.make_batch(4, gpu))
    assert torch.isfinite(tr2.step()).item()


def _crash_recovery(tmp_path, device, plane="collective"):
    """SIGKILL one of 3 ranks mid-run (no hand-over, no deregistration). The
    survivors' blocked collective fails, the coordinator expires the dead worker, one survivor
    publishes a restore plan and both rebuild a 2-rank world from the last canonical checkpoint
    (step 10; the crash is at step 12) and finish all 30 steps. Their final parameters equal an
    fp32 replay of steps 10..29 with 2 workers starting from that checkpoint."""
    from parameter_server_distributed_amd import native

    cport = _port()
    coord = subprocess.Popen([os.path.join(ROOT, "bin", "coordinator"), f"127.0.0.1:{cport}", "127.0.0.1:1",
                              "--expiry-s", "2", "--sweep-s", "0.3", "--store-port", "0"],
                             stdout=open(tmp_path / "coord.log", "w"), stderr=subprocess.STDOUT,
                             env=dict(os.environ, PYTHONPATH=ROOT))
    procs = []
    try:
        ck = str(tmp_path / "ck")
        steps, kill_at = 30, 12
        for w in range(3):
            procs.append(subprocess.Popen(
                [sys.executable, os.path.join(ROOT, "tests", "elastic_crash_worker.py"), f"127.0.0.1:{cport}", str(w),
                 str(steps), ck, str(tmp_path / f"w{w}.json"), str(kill_at if w == 2 else -1), device, plane],
                stdout=open(tmp_path / f"w{w}.log", "w"), stderr=subprocess.STDOUT,
                env=dict(os.environ, PYTHONPATH=ROOT, PSD_ASYNC_DEAD_S="3")))
        rcs = [p.wait(timeout=240) for p in procs]
        logs = [open(tmp_path / f"w{w}.log").read() for w in range(3)]
        assert rcs[2] == -9 and rcs[0] == 0 and rcs[1] == 0, (rcs, logs[0][-3000:], logs[1][-3000:])
        import json

        res = [json.load(open(tmp_path / f"w{w}.json")) for w in (0, 1)]
        for r in res:
            assert r["finished_at"] == steps and r["recovered_at"], r
            assert r["history"][-1][1] == [0, 1] and r["history"][-1][2] == 10, r["history"]
        got = [torch.load(str(tmp_path / f"w{w}.json.pt"), weights_only=True) for w in (0, 1)]
        for n in got[0]:
            assert torch.equal(got[0][n], got[1][n]), n
        # replay from the checkpoint the survivors restored
        man, ts = native().load_native_ckpt(os.path.join(ck, "elastic_canonical.psd"))
        m = json.loads(man)
        sd = dict(zip(m["keys"], ts))
        assert m["step"] >= 10
        torch.manual_seed(0)
        spec = models.build("mlp", CPU, torch.float32, hidden=64)
        params = list(spec.model.parameters())
        off = 0
        for p in params:
            p.data.copy_(sd["master"][off:off + p.numel()].view_as(p))
            off += p.numel()
        opt = torch.optim.SGD(params, lr=0.05, momentum=0.9, weight_decay=1e-3)
        off = 0
        for p in params:
            opt.state[p]["momentum_buffer"] = sd["state1"][off:off + p.numel()].view_as(p).clone()
            off += p.numel()
        batches = [spec.make_batch(16, CPU, seed=1000 + w) for w in (0, 1)]
        for _ in range(m["step"], steps):
            grads = [torch.zeros_like(p) for p in params]
            for x, y in batches:
                spec.model.zero_grad()
                spec.loss(spec.model(x), y).backward()
                for g, p in zip(grads, params):
                    g += p.grad / 2
            for p, g in zip(params, grads):
                p.grad = g
            opt.step()
        tol = dict(rtol=1e-5, atol=1e-6) if device == "cpu" else dict(rtol=1e-4, atol=1e-5)
        for n, p in spec.model.named_parameters():
            torch.testing.assert_close(got[0][n], p.detach(), msg=n, **tol)
    finally:
        for p in procs + [coord]:
            if p.poll() is None:
                p.kill()


@pytest.mark.slow
def test_crash_recovery_from_canonical_checkpoint(tmp_path):
    _crash_recovery(tmp_path, "cpu")


@pytest.mark.slow
def test_async_plane_crash_recovery(tmp_path):
    """the same SIGKILL scenario on the asynchronous peer-memory plane. The
    dead rank's engine heartbeat stops; within PSD_ASYNC_DEAD_S (3 s here, not the 600 s SSP
    deadline) every survivor's SSP wait fails, the survivors abort their engines (no barrier with
    the dead peer), rebuild a 2-rank AsyncPS from the canonical checkpoint and finish; K-batch rounds
    at bound 0 are the synchronous steps, so they match the same fp32 replay."""
    _crash_recovery(tmp_path, "cpu", plane="async")


@pytest.mark.gpu
def test_crash_recovery_gpu_ranks(tmp_path, gpu):
    """the multi-rank elastic path on device tensors -- 3 ranks on the one GPU
    (gloo group over cuda tensors, fused apply kernel on the HBM shards), one SIGKILLed mid-run,
    survivors restore from the canonical checkpoint and match the fp32 replay."""
    _crash_recovery(tmp_path, "cuda:0")


def test_reshard_resets_grad_scale_to_the_new_world():
    """A canonical state from a W-worker world loaded into another world keeps lr / step / bias
    corrections but averages over the *new* worker count (a W=3 scale in a 2-worker world made every
    update 2/3 too small until the crash-recovery replay test caught it)."""
    spec = _mlp()
    ps = _ps(spec, 0, 0.05, "momentum")
    sd = ps.canonical_state(root=0)
    f = sd["dyn"].view(torch.float32)
    f[1] = 1.0 / 3.0
    sd["dyn"][4] = 7
    ps.load_canonical_state(sd)
    assert float(ps.dyn.t.view(torch.float32)[1]) == 1.0 / len(ps.worker_ranks)
    assert int(ps.dyn.t[4]) == 7


def test_elastic_worker_fp8_compute_flag():
    """the elastic worker builds BASELINE config 5's model with fp8 compute
    (``--fp8-compute``): every bottleneck convolution is an fp8-capable module with fp8 on."""
    from parameter_server_distributed_amd.cli.worker import build_model
    from parameter_server_distributed_amd.ops.conv import Conv1x1, ConvNHWC

    class A:
        model, fp8_compute, image_size = "resnet50", True, 32

    spec = build_model(A, CPU, torch.float32)
    convs = [m for m in spec.model.modules() if isinstance(m, (Conv1x1, ConvNHWC))]
    assert len(convs) >= 48 and all(m.fp8 for m in convs)
    A.fp8_compute = False
    assert not any(m.fp8 for m in build_model(A, CPU, torch.float32).model.modules()
                   if isinstance(m, (Conv1x1, ConvNHWC)))
