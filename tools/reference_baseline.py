#!/usr/bin/env python3
"""Reference-semantics baseline on the same MI355X box ("the reference-semantics
baseline row is the comparator for match or beat").

Runs the reference's architecture end to end -- coordinator + ONE host-memory parameter server with
the reference's semantics (sync barrier over all workers, fp32 tensors as protobuf ``repeated
float`` over gRPC, ``p -= g`` with the first aggregate becoming the parameters) + worker
process(es) computing real ResNet-50 gradients on the GPU -- and reports whole-job samples/s in
the bench.py JSON shape. Nothing here uses RCCL, the HBM shard or the fused kernels.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--iterations", type=int, default=4)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--wire", default="reference", choices=["reference", "raw"])
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    env = dict(os.environ, PYTHONPATH=ROOT)
    cp, pp = _port(), _port()
    tmp = f"/tmp/psd_refbase_{os.getpid()}"
    os.makedirs(tmp, exist_ok=True)
    procs = []
    try:
        procs.append(subprocess.Popen([f"{ROOT}/bin/coordinator", f"127.0.0.1:{cp}", f"127.0.0.1:{pp}"], env=env,
                                      stdout=open(f"{tmp}/coord.log", "w"), stderr=subprocess.STDOUT))
        procs.append(subprocess.Popen([f"{ROOT}/bin/parameter_server", f"127.0.0.1:{pp}", str(a.workers), "0",
                                       "--reference-compat"], env=env, stdout=open(f"{tmp}/ps.log", "w"),
                                      stderr=subprocess.STDOUT))
        ws = []
        for w in range(a.workers):
            args = [f"{ROOT}/bin/worker_main", f"127.0.0.1:{cp}", str(w), str(a.iterations + 1), "--model", a.model,
                    "--batch", str(a.batch), "--device", "cuda", "--stats-json", f"{tmp}/w{w}.json"]
            if a.wire == "reference":
                args.append("--reference-wire")
            ws.append(subprocess.Popen(args, env=env, stdout=open(f"{tmp}/w{w}.log", "w"), stderr=subprocess.STDOUT))
        rc = [p.wait(timeout=3000) for p in ws]
        if any(rc):
            print(open(f"{tmp}/w0.log").read()[-3000:], file=sys.stderr)
            raise SystemExit(f"worker failed: {rc}")
        # iteration 0 includes warmup (MIOpen, first pushes); time iterations 1..N from the logs
        txt = open(f"{tmp}/w0.log").read()
        st = json.load(open(f"{tmp}/w0.json"))
        per_it = sum(st["iter_seconds"][1:]) / max(1, len(st["iter_seconds"]) - 1)  # skip warmup iter 0
        lines = [ln for ln in txt.splitlines() if " iter " in ln]
        value = a.batch * a.workers / per_it
        rec = {"metric": f"samples/sec reference-semantics baseline ({a.model}, gRPC {a.wire} fp32 tensors, "
                         f"1 host-memory PS, sync barrier)", "value": round(value, 3), "unit": "samples/s",
               "n_gpus": a.workers, "iterations": a.iterations + 1, "sec_per_iteration": round(per_it, 3),
               "per_gpu_batch": a.batch, "worker_log_tail": lines[-3:]}
        print(json.dumps(rec))
        if a.out:
            with open(a.out, "w") as f:
                f.write(json.dumps(rec) + "\n")
    finally:
        for p in procs:
            p.kill()


if __name__ == "__main__":
    main()
