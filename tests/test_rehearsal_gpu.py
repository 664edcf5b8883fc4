"""The driver's N = 8 launch of bench.py rehearsed on ONE MI355X: 8 ranks over
gloo share the GPU (real IPC peer mappings, the scatter / gather kernels between the ranks' buffers),
BASELINE config 3's layout (2 PS shards, SSP bound 1) at a small shape, checked by
tools/rehearsal_check.py: the async plane did not fall back, the kernel transport ran, every autotune
decision came through the rendezvous store, the staleness histogram holds one entry per
(worker push, shard), and the weights are finite. The full-size runs of all three BASELINE layouts
are in profiles/r6/rehearsal8/ (scripts/gpu_r6_rehearsal8.sh)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from rehearsal_check import check  # noqa: E402


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_bench_world8_on_one_gpu(tmp_path, gpu):
    out = tmp_path / "rh8.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "8", "--backend", "gloo", "--model", "resnet50", "--batch", "8", "--image-size", "64",
           "--ps-shards", "2", "--staleness", "1", "--steps", "3", "--warmup", "2", "--comm-probe", "0",
           "--out", str(out)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads(out.read_text().strip().splitlines()[-1])
    bad = check(rec, 8)
    print(rec["value"], rec["config"]["parallelism"], rec.get("async_xfer_blocks"), rec["staleness_hist"])
    assert not bad, bad
