"""One elastic worker for tests/test_elastic_collective.py::test_crash_recovery (run as a
subprocess so that it can be SIGKILLed). argv: coordinator worker_id steps ckpt_dir out_json kill_at
[device] [plane] (device cpu, or cuda:0 -- every rank on the one GPU, gloo process group over cuda
tensors; plane collective (CollectivePS) or async (AsyncPS, K-batch rounds at SSP bound 0))"""
import json
import os
import signal
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from parameter_server_distributed_amd import models  # noqa: E402
from parameter_server_distributed_amd.ops.optim import OptimConfig  # noqa: E402
from parameter_server_distributed_amd.parallel.async_ps import AsyncPS  # noqa: E402
from parameter_server_distributed_amd.parallel.collective_ps import CollectivePS  # noqa: E402
from parameter_server_distributed_amd.runtime.elastic import ElasticAgent, ElasticTrainer  # noqa: E402
from parameter_server_distributed_amd.runtime.trainer import Trainer  # noqa: E402

CFG = dict(kind="momentum", lr=0.05, momentum=0.9, weight_decay=1e-3)


def main():
    coord, wid, steps, ckpt_dir, out, kill_at = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], \
        sys.argv[5], int(sys.argv[6])
    dev = torch.device(sys.argv[7] if len(sys.argv) > 7 else "cpu")
    plane = sys.argv[8] if len(sys.argv) > 8 else "collective"
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    torch.manual_seed(0)
    spec = models.build("mlp", dev, torch.float32, hidden=64)
    batch = spec.make_batch(16, dev, seed=1000 + wid)
    agent = ElasticAgent(coord, wid, heartbeat_s=0.3, timeout_s=60.0)
    trace = []

    def make_ps(model, transport):
        if plane == "async":
            return AsyncPS(model, OptimConfig(**CFG), num_shards=transport.world, staleness=0, bucket_mb=0.0005,
                           param_dtype=torch.float32, device=dev, timeout_s=60.0)
        return CollectivePS(model, OptimConfig(**CFG), transport, num_shards=transport.world, staleness=0,
                            bucket_mb=0.0005, grad_dtype=torch.float32, param_dtype=torch.float32, device=dev)

    def make_trainer(ps):
        return Trainer(spec.model, spec.loss, ps, batch, use_graph=False)

    def on_step(step, loss, plan):
        trace.append((step, plan.gen, list(plan.members)))
        if step == kill_at:
            os.kill(os.getpid(), signal.SIGKILL)  # crash: no hand-over, no deregistration

    et = ElasticTrainer(agent, spec.model, make_ps, make_trainer, steps, dev, check_every=1000, min_workers=3,
                        on_step=on_step, checkpoint_dir=ckpt_dir, checkpoint_every=5, collective_timeout_s=20.0,
                        backend="gloo")
    res = et.run()
    with open(out, "w") as f:
        json.dump({"trace": trace, "recovered_at": res.get("recovered_at"), "finished_at": res.get("finished_at"),
                   "history": res["history"]}, f)
    torch.save({n: p.detach().cpu().clone() for n, p in res["params"].items()}, out + ".pt")


if __name__ == "__main__":
    main()
